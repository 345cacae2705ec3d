set -o pipefail
mkdir -p gpurun_out/final2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final2/gputests.log 2>&1 && tail -2 gpurun_out/final2/gputests.log && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final2/smoke.log 2>&1 && tail -1 gpurun_out/final2/smoke.log && \
timeout -k 10 300 python bench.py > gpurun_out/final2/bench.log 2>&1 && tail -1 gpurun_out/final2/bench.log
