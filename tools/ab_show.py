"""Per-variant summary of a tools/ab_spec.sh run: the bench line's ms_per_step and the engine kernels'
average time per call (rocprofv3 kernel stats).   usage: python3 tools/ab_show.py gpurun_out/TAG [N]"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
vs = sorted((p for p in glob.glob(os.path.join(d, "v*.json")) if os.path.basename(p)[1:-5].isdigit()),
            key=lambda p: int(os.path.basename(p)[1:-5]))
stats = {}
for p in vs:
    v = os.path.basename(p)[:-5]
    line = [l for l in open(p) if l.startswith("{")]
    b = json.loads(line[-1]) if line else {}
    rows = list(csv.DictReader(open(os.path.join(d, v, "run_kernel_stats.csv"))))
    stats[v] = (b.get("ms_per_step"), {r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]:
                                       float(r["AverageNs"]) / 1e3 for r in rows if "::k_" in r["Name"]})
names = sorted({k for _, s in stats.values() for k in s}, key=lambda k: -max(s.get(k, 0) for _, s in stats.values()))
print("%-34s" % "ms_per_step" + "".join("%10s" % stats[v][0] for v in stats))
for k in names[:top]:
    print("%-34s" % k[:34] + "".join("%10.1f" % stats[v][1].get(k, float("nan")) for v in stats))
