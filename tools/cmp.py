"""Compare two quick_perf runs: bench line + per-kernel average times.  usage: tools/cmp.py TAG_A TAG_B"""
import csv
import json
import sys


def load(tag):
    b = json.load(open(f"gpurun_out/{tag}/bench.json"))
    k = {}
    for r in csv.DictReader(open(f"gpurun_out/{tag}/prof/run_kernel_stats.csv")):
        name = r["Name"].replace("(anonymous namespace)::", "")
        name = name.split("(")[0][:40]
        k[name] = float(r["AverageNs"]) / 1000 * int(r["Calls"]) / 13
    return b, k


a, ka = load(sys.argv[1])
b, kb = load(sys.argv[2])
print(f"value {a['value']:.0f} -> {b['value']:.0f}   pipeline {a['stages_ms']['pipeline']} -> {b['stages_ms']['pipeline']}")
print("stages", {s: (a['stages_ms'][s], b['stages_ms'][s]) for s in b['stages_ms']})
for n in sorted(set(ka) | set(kb), key=lambda n: -max(ka.get(n, 0), kb.get(n, 0))):
    if n.startswith("void at::") or "rocclr" in n or "elementwise" in n:
        continue
    x, y = ka.get(n, 0), kb.get(n, 0)
    if max(x, y) > 3:
        print(f"  {n:40s} {x:8.1f} {y:8.1f}  {y - x:+7.1f} us/step")
