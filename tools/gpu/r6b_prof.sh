cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6b
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6b/pytest.log 2>&1
echo "pytest rc=$?"; tail -5 gpurun_out/r6b/pytest.log
BENCH_ARGS="--model ResNet152" bash tools/gpu/prof_bench.sh r6_r152 1024 128 || exit 1
for m in DenseNet121 GoogLeNet DLA SimpleDLA DPN26 ShuffleNetV2_1; do
  BENCH_ARGS="--model $m" bash tools/gpu/prof_bench.sh r6_$m 256 || exit 1
done
