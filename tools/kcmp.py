"""Side-by-side per-kernel average times (µs) of several rocprofv3 kernel_stats.csv files (engine kernels).
usage: python tools/kcmp.py DIR_OR_CSV...   (a directory: its run_kernel_stats.csv)"""
import csv
import os
import sys


def load(p):
    if os.path.isdir(p):
        p = os.path.join(p, "run_kernel_stats.csv")
    return {r["Name"]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3)
            for r in csv.DictReader(open(p)) if "anonymous namespace" in r["Name"]}


runs = [load(p) for p in sys.argv[1:]]
names = sorted(set().union(*runs), key=lambda n: -max(r.get(n, (0, 0, 0))[2] for r in runs))
calls0 = max(r.get(names[0], (1, 0, 0))[0] for r in runs) if names else 1
for n in names[:40]:
    cells = []
    for r in runs:
        c, a, t = r.get(n, (0, 0.0, 0.0))
        cells.append(f"{t / max(c, 1) * c / calls0:9.1f}" if c else "        -")
    short = n.replace("(anonymous namespace)::", "").split("(")[0][:48]
    print(f"{short:48s}" + "".join(cells))
tot = [sum(v[2] for v in r.values()) / calls0 for r in runs]
print(f"{'TOTAL per step (us)':48s}" + "".join(f"{t:9.1f}" for t in tot))
