"""Per-kernel us/step of the variants of one tools/ab.sh run.  usage: tools/abcmp.py TAG"""
import csv
import glob
import json
import os
import sys

d = f"gpurun_out/{sys.argv[1]}"
vs = sorted(glob.glob(f"{d}/v*/run_kernel_stats.csv"), key=lambda p: int(p.split("/v")[-1].split("/")[0]))
tabs, heads = [], []
for p in vs:
    t = {}
    for r in csv.DictReader(open(p)):
        n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:34]
        t[n] = t.get(n, 0) + float(r["AverageNs"]) / 1000 * int(r["Calls"]) / 13
    tabs.append(t)
    j = os.path.join(os.path.dirname(os.path.dirname(p)), os.path.basename(os.path.dirname(p)) + ".json")
    try:
        b = json.loads(open(j).read().strip().splitlines()[-1])
        heads.append(f"{b['stages_ms']['pipeline']:.4f}")
    except Exception:
        heads.append("?")
print("pipeline ms:", " ".join(heads))
names = sorted({n for t in tabs for n in t}, key=lambda n: -max(t.get(n, 0) for t in tabs))
for n in names:
    if n.startswith("at::") or "rocclr" in n or "elementwise" in n or "compute_cuda" in n or "rocprim" in n:
        continue
    row = [t.get(n, 0) for t in tabs]
    if max(row) > 3:
        print(f"  {n:34s} " + " ".join(f"{x:8.1f}" for x in row))
