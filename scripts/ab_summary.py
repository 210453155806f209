"""Median [min-max] device time per size of an ab_ll_latency.sh run: python scripts/ab_summary.py TAG"""
import collections
import glob
import statistics
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "ll"
res = collections.defaultdict(lambda: collections.defaultdict(list))
wrong = 0
for f in sorted(glob.glob(f"gpurun_out/ab_{tag}_*_*.txt")):
    v = f.split("_")[-2]
    for ln in open(f):
        t = ln.split()
        if t and t[0].isdigit():
            res[int(t[0])][v].append(float(t[2]))
            wrong += int(t[5])
print(f"# bytes   A median [min-max]        B median [min-max]      (#wrong over all runs: {wrong})")
for b in sorted(res):
    a, bb = res[b]["A"], res[b]["B"]
    print(f"{b:8d}  {statistics.median(a):6.2f} [{min(a):.2f}-{max(a):.2f}]   {statistics.median(bb):6.2f} [{min(bb):.2f}-{max(bb):.2f}]")
