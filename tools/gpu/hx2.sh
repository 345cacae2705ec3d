#!/bin/bash
# stride-2 dgrad through the halo kernel: numerics, then timing vs the parity-class kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo_kernel" -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
for b in 1024 128; do
for shp in "64 128 32" "128 256 16" "256 512 8"; do
  set -- $shp
  PCA_CONV_HX=0 timeout -k 10 120 python tools/time_conv.py --batch $b --cin $1 --cout $2 --h $3 --s 2 --passes dgrad,dgrad_bn --tag old || exit 1
  timeout -k 10 120 python tools/time_conv.py --batch $b --cin $1 --cout $2 --h $3 --s 2 --passes dgrad,dgrad_bn --cfg 30 --tag hx || exit 1
done
done
