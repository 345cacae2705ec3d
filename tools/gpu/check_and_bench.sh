set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK
timeout -k 10 240 python bench.py --steps 30 --warmup 10 > gpurun_out/bench1024.json 2> gpurun_out/bench1024.err && cat gpurun_out/bench1024.json &&
timeout -k 10 240 python bench.py --steps 30 --warmup 10 --batch 128 > gpurun_out/bench128.json 2> gpurun_out/bench128.err && cat gpurun_out/bench128.json &&
timeout -k 10 240 python bench.py --steps 30 --warmup 10 --batch 256 > gpurun_out/bench256.json 2>&1 && cat gpurun_out/bench256.json &&
timeout -k 10 240 python bench.py --steps 30 --warmup 10 --batch 512 > gpurun_out/bench512.json 2>&1 && cat gpurun_out/bench512.json
