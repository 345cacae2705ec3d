cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
( for cfg in -1 13 6 10 11 1 4 5 0 3; do timeout -k 5 60 python tools/conv_one.py --cin 64 --cout 128 --h 32 --s 2 --pass dgrad --cfg $cfg --iters 20 || exit 1; done
  for cfg in -1 13 6 10 11 1 4 0 3 9 12; do timeout -k 5 60 python tools/conv_one.py --cin 128 --cout 256 --h 16 --s 2 --pass dgrad --cfg $cfg --iters 20 || exit 1; done
  timeout -k 5 60 python tools/conv_one.py --cin 64 --cout 128 --h 32 --s 2 --pass fwd --iters 20
  timeout -k 5 60 python tools/conv_one.py --cin 128 --cout 128 --h 16 --s 1 --pass dgrad --iters 20
) > gpurun_out/diag/conv.txt 2>&1 || exit 1
cat gpurun_out/diag/conv.txt
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "stem or augment" > gpurun_out/diag/pytest.log 2>&1 || { tail -30 gpurun_out/diag/pytest.log; exit 1; }
tail -2 gpurun_out/diag/pytest.log
for pc in 4096 16384 65536; do
  for b in 1024 128; do
    PCA_PREP_CHUNK=$pc timeout -k 10 300 python bench.py --steps 30 --warmup 10 --batch $b > gpurun_out/diag/pc${pc}_b$b.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/diag/pc${pc}_b$b.json').read().strip().splitlines()[-1]); print('prep $pc b$b %.3f ms %.1f img/s' % (d['ms_per_step'], d['value']))"
  done
done
PCA_PREP_CHUNK=16384 bash tools/gpu/prof_bench.sh s2 1024 128
