cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for a in ${ABL:-0 1 2 3}; do
  export PCA_HALO_ABLATE=$a
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl$a -o run -- python3 tools/probes/halo_ablate.py > gpurun_out/abl$a.log 2>&1 || exit 1
done
