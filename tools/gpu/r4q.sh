#!/bin/bash
# dual-BN aux2 in LDS + halo wgrad DMA interleave: numerics, same-box A/B vs round 3, traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_kernels_gpu.py -q -k "dual or dgrad or every_tile or wgrad or halo" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit 1
PCA_HALO_ILV=1 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -k "wgrad or halo" --timeout 300 --timeout-method thread > $O/pytest_ilv.log 2>&1
rc=$?; echo "pytest(halo ilv) rc=$rc"; tail -2 $O/pytest_ilv.log; grep -E "^FAILED|^E " $O/pytest_ilv.log | head -20
[ $rc -ne 0 ] && exit 1
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 1024 128; do
    (cd baseline_r3 && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/r3_${b}_$rep.json 2>$O/r3.err || exit $?
    for v in 0 1; do
      PCA_HALO_ILV=$v timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/ilv${v}_${b}_$rep.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
    done
    (cd variant_sp && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/sp_${b}_$rep.json 2>$O/sp.err || { tail -5 $O/sp.err; exit 1; }
    echo "rep$rep bs$b r3 $(ms $O/r3_${b}_$rep.json) cur $(ms $O/ilv0_${b}_$rep.json) halo-ilv $(ms $O/ilv1_${b}_$rep.json) igemm-dma-spread $(ms $O/sp_${b}_$rep.json)"
  done
done
PCA_HALO_ILV=1 PCA_TUNE_LOG=1 timeout -k 10 300 python bench.py --batch 1024 --steps 5 --warmup 2 > $O/tune1.json 2> $O/tune1.log || exit 1
PCA_TUNE_LOG=1 timeout -k 10 300 python bench.py --batch 1024 --steps 5 --warmup 2 > $O/tune0.json 2> $O/tune0.log || exit 1
bash tools/gpu/prof_bench.sh r4q 1024 128 || exit 1
exit 0
