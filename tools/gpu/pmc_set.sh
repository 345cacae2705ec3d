#!/bin/bash
# PMC passes for a set of conv shapes/passes (bs1024 ResNet-18 census) + time per kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
set -o pipefail
for spec in "c64f:--cin 64 --cout 64 --h 32 --pass fwd" "c64d:--cin 64 --cout 64 --h 32 --pass dgrad" \
            "l2f:--cin 128 --cout 128 --h 16 --pass fwd" "l2d:--cin 128 --cout 128 --h 16 --pass dgrad" \
            "l1w:--cin 64 --cout 64 --h 32 --pass wgrad" "l3f:--cin 256 --cout 256 --h 8 --pass fwd"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 120 python3 tools/conv_one.py $args || exit 1
  PMC_EXTRA=1 bash tools/pmc_conv.sh $tag $args || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc/${tag}_p* > gpurun_out/pmc/${tag}_summary.txt || exit 1
done
