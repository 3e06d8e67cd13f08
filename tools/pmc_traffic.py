"""Aggregate tools/pmc_traffic.sh output into profiles/traffic.json (read by bench.py).

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (TCC EA request counters).  The guide
(MI355X_MICROARCH.md, HBM section) says gfx950 FETCH_SIZE under-reports wide streaming reads by 2x and
that other access shapes must be calibrated: the correction used here is measured on
tools/micro/lane_read's k_lane_rev, which reads exactly 1200 MiB per dispatch in the k_scan pattern
(per-lane 1 KiB ranges, right to left, 64-byte blocks).  usage: pmc_traffic.py OUTDIR [--write]
"""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ["context-based-pii_amd/csrc/pii_engine.hip", "context-based-pii_amd/csrc/pii_device.h"]
CALIB_BYTES = 1200 * (1 << 20)


def per_kernel(d, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            acc[(k, r.get("Dispatch_Id", len(acc)))].append(float(r["Counter_Value"]))
    out = defaultdict(list)
    for (k, _), v in acc.items():
        out[k].append(sum(v))          # sum over the counter's instances of one dispatch
    return out


def main():
    d = sys.argv[1]
    fetch = per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "write"), "WRITE_SIZE")
    calib = per_kernel(os.path.join(d, "calib"), "FETCH_SIZE")
    rev = calib.get("k_lane_rev", [])
    # lane_read launches k_lane_rev at 512/1024/2048 B per lane, 6 times each: all read CALIB_BYTES
    corr = CALIB_BYTES / (sum(rev) / len(rev) * 1024) if rev else None
    bench = [json.loads(l) for l in open(os.path.join(d, "fetch.log")) if l.startswith("{")]
    n_bytes = bench[-1]["config"]["bytes_per_gpu"] if bench else None
    h = hashlib.sha256()
    for f in SOURCES:
        h.update(open(os.path.join(ROOT, f), "rb").read())
    res = {"source_digest": h.hexdigest()[:16], "bytes_per_gpu": n_bytes, "fetch_correction": corr,
           "note": "hbm_bytes = FETCH_SIZE*1024*fetch_correction + WRITE_SIZE*1024, mean per dispatch",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        f = sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [0]))) * 1024
        w = sum(write.get(k, [0])) / max(1, len(write.get(k, [0]))) * 1024
        res["kernels"][k] = {"fetch_reported_bytes": round(f), "write_bytes": round(w),
                             "hbm_bytes": round(f * (corr or 1.0) + w) if corr else None}
    print(json.dumps(res, indent=1))
    if "--write" in sys.argv:
        json.dump(res, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
