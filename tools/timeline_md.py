#!/usr/bin/env python3
"""Markdown profile page from a tools/step_timeline.py output: header line, per-family table
(us per step, launches) and the step's kernel timeline.

  python tools/timeline_md.py gpurun_out/prof/x_b128_timeline.txt "title" "how it was run" > profiles/x.md
"""
import collections
import re
import sys


def family(name):
    n = re.sub(r"^_ZN3pca\d+", "", name)
    n = re.sub(r"(I|E)[LEb].*$", "", n) if not n.startswith(("conv_", "wgrad_", "dwk_", "se_", "bn_")) else n
    return re.sub(r"<.*", "", n)


def main():
    path, title, how = sys.argv[1], sys.argv[2], sys.argv[3]
    lines = open(path).read().splitlines()
    head = lines[0]
    rows = []
    for ln in lines[1:]:
        p = ln.split(None, 4)
        if len(p) == 5 and p[0].isdigit():
            rows.append((float(p[2]), p[4].strip()))
    fam = collections.defaultdict(lambda: [0.0, 0])
    for us, name in rows:
        f = family(name)
        fam[f][0] += us
        fam[f][1] += 1
    print(f"# {title}\n\n{how}\n\n{head}\n\n## Time per kernel family (us per step, launches)\n```")
    for f, (t, n) in sorted(fam.items(), key=lambda x: -x[1][0]):
        print(f"{t:9.1f} {n:4d} {f[:80]}")
    print("```\n\n## Step timeline (index, start us, duration us, gap us, kernel)\n```")
    for ln in lines[1:]:
        if ln.strip():
            print(ln)
    print("```")


if __name__ == "__main__":
    main()
