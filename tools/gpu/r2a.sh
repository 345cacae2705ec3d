bash tools/gpu/round_check.sh && bash tools/gpu/prof_bench.sh r2a 1024 128
