#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for arm in 0 1; do
  PCA_DW_BN_FUSE=$arm BENCH_ARGS="--model MobileNetV2" bash tools/gpu/prof_bench.sh mnv2_f$arm 1024 > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import re, collections
for arm in (0, 1):
    fam = collections.defaultdict(lambda: [0.0, 0])
    for line in open(f"gpurun_out/prof/mnv2_f{arm}_b1024_timeline.txt"):
        p = line.split(None, 4)
        if len(p) == 5 and p[0].isdigit():
            k = re.sub(r"^_ZN3pca\d+", "", p[4].strip())[:60]
            fam[k][0] += float(p[2]); fam[k][1] += 1
    print("== fuse", arm, open(f"gpurun_out/prof/mnv2_f{arm}_b1024_timeline.txt").readline().strip())
    for k, (t, n) in sorted(fam.items(), key=lambda x: -x[1][0])[:16]:
        print(f"{t:9.1f} {n:4d} {k}")
PY
