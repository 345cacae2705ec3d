#!/bin/bash
# c64 versions 2 / 3 / 4: numerics, per-call timing, PMC counters (forward + dgrad).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "c64" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do for V in 2 3 4; do for P in fwd dgrad; do
  PCA_C64_V=$V timeout -k 10 60 python tools/conv_one.py --pass $P --iters 20 2>&1 | tail -1 | sed "s/^/v$V /" || exit 1
done; done; done
for V in 2 3 4; do for P in fwd dgrad; do
  PCA_C64_V=$V PMC_EXTRA=1 bash tools/pmc_conv.sh c64v${V}_$P --pass $P --iters 3 || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc/c64v${V}_${P}_p* > $O/pmc_v${V}_$P.txt || exit 1
done; done
