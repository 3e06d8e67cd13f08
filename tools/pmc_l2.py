"""L2 (TCC) hit rate per kernel of a `rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum` pass over
`bench.py --workload config5` (SURVEY §8 ★X1: the config-5 automata spill LDS into L2).
usage: pmc_l2.py DIR [--write]   (--write: profiles/config5_l2.json, keyed to the kernel sources)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    d = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if not k.startswith("k_") and "k_" not in k:
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == "TCC_HIT_sum":
                n[k] += 1
    out = {}
    for k, cs in sorted(acc.items(), key=lambda kv: -(kv[1]["TCC_HIT_sum"] + kv[1]["TCC_MISS_sum"])):
        h, m = cs["TCC_HIT_sum"], cs["TCC_MISS_sum"]
        if h + m == 0:
            continue
        out[k] = {"hit_rate": round(h / (h + m), 4), "requests_per_dispatch": int((h + m) / max(n[k], 1))}
        print(f"{k[:40]:40s} hit {h / (h + m):6.3f}  requests/dispatch {(h + m) / max(n[k], 1):14.0f}")
    if "--write" in sys.argv:
        import bench
        json.dump({"source_digest": bench.source_digest(), "counters": "TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)",
                   "workload": "bench.py --workload config5", "kernels": out},
                  open(os.path.join(ROOT, "profiles", "config5_l2.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
