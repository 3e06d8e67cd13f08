"""Steady-state per-kernel us/step of the variants of one tools/ab.sh run: the mean over the LAST
--tail dispatches of each kernel (the window workload's first steps fill the rings and are lighter).
usage: tools/abss.py TAG [--tail 10]"""
import csv
import glob
import sys
from collections import defaultdict

d = f"gpurun_out/{sys.argv[1]}"
tail = int(sys.argv[sys.argv.index("--tail") + 1]) if "--tail" in sys.argv else 10
vs = sorted(glob.glob(f"{d}/v*/run_kernel_trace.csv"), key=lambda p: int(p.split("/v")[-1].split("/")[0]))
tabs = []
for p in vs:
    per = defaultdict(list)
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:34]
        per[n].append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    t = {}
    for n, v in per.items():
        v.sort()
        calls_per_step = max(1, round(len(v) / 13))
        last = [x for _, x in v[-tail * calls_per_step:]]
        t[n] = sum(last) / tail
    tabs.append(t)
tot = [sum(x for n, x in t.items() if n.startswith("k_")) for t in tabs]
print("engine-kernel us/step:", " ".join(f"{x:8.1f}" for x in tot))
names = sorted({n for t in tabs for n in t}, key=lambda n: -max(t.get(n, 0) for t in tabs))
for n in names:
    if not n.startswith("k_"):
        continue
    row = [t.get(n, 0) for t in tabs]
    if max(row) > 2:
        print(f"  {n:34s} " + " ".join(f"{x:8.1f}" for x in row))
