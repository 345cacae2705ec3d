#!/bin/bash
# PMC counter passes on the stem forward (stem.hip) and the layer-1 c64 forward at bs1024
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/pmc_conv.sh stem --batch 1024 --cin 8 --cout 64 --h 32 --pass fwd || exit 1
bash tools/pmc_conv.sh c64 --batch 1024 --cin 64 --cout 64 --h 32 --pass fwd || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc/stem_p1 gpurun_out/pmc/stem_p2 > gpurun_out/pmc/stem_summary.txt
python3 tools/pmc_summary.py gpurun_out/pmc/c64_p1 gpurun_out/pmc/c64_p2 > gpurun_out/pmc/c64_summary.txt
cat gpurun_out/pmc/stem_summary.txt gpurun_out/pmc/c64_summary.txt
