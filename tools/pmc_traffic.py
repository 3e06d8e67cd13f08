"""Aggregate tools/pmc_traffic.sh output into profiles/traffic.json, keyed by bench workload (read by
bench.py: every workload line quotes only the counters of its own workload, measured on the current
kernel sources, or null).

HBM bytes: FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (TCC EA request counters).  The guide
(MI355X_MICROARCH.md, HBM section) says gfx950 FETCH_SIZE under-reports wide streaming reads by 2x and
that other access shapes must be calibrated: the correction used here is measured on
tools/micro/lane_read's k_lane_rev, which reads exactly 1200 MiB per dispatch in the k_scan pattern
(per-lane 1 KiB ranges, right to left, 64-byte blocks).

LDS-array cycles (scan workloads): SQ_LDS_IDX_ACTIVE is converted to LDS-array cycles with the factor
tools/micro/lds_calib measures on ds_read_b32 patterns of known cost (2 / 4 / 8 cycles per
wave-instruction: conflict-free, 2-way, 4-way; guide LDS table), so bench.py can state k_scan's LDS
cycles per byte and the throughput ceiling they imply.
usage: pmc_traffic.py OUTDIR --workload NAME [--write]
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


def mean(x):
    return sum(x) / len(x) if x else 0.0


def lds_unit(d):
    """counter units per LDS-array cycle, from tools/micro/lds_calib"""
    idx = per_kernel(os.path.join(d, "lds_calib"), "SQ_LDS_IDX_ACTIVE")
    info = [json.loads(l) for l in open(os.path.join(d, "lds_calib.log")) if l.startswith("{")]
    if not idx or not info:
        return None, {}
    info = info[-1]
    per = {}
    for k, cyc in info["cycles_per_read"].items():
        if idx.get(k):
            per[k] = mean(idx[k]) / (info["waves_per_launch"] * info["reads_per_wave"] * cyc)
    return (mean(list(per.values())) if per else None), per


def main():
    d = sys.argv[1]
    w = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "scan"
    fetch = per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "write"), "WRITE_SIZE")
    calib = per_kernel(os.path.join(d, "calib"), "FETCH_SIZE")
    rev = calib.get("k_lane_rev", [])
    # lane_read launches k_lane_rev at 512/1024/2048 B per lane, 6 times each: all read CALIB_BYTES
    corr = CALIB_BYTES / (sum(rev) / len(rev) * 1024) if rev else None
    bench = [json.loads(l) for l in open(os.path.join(d, "fetch.log")) if l.startswith("{")]
    n_bytes = bench[-1]["config"].get("bytes_per_gpu", bench[-1]["config"].get("bytes_per_step")) if bench else None
    h = hashlib.sha256()
    for f in SOURCES:
        h.update(open(os.path.join(ROOT, f), "rb").read())
    res = {"workload": w, "source_digest": h.hexdigest()[:16], "bytes_per_gpu": n_bytes, "fetch_correction": corr,
           "note": "hbm_bytes = FETCH_SIZE*1024*fetch_correction + WRITE_SIZE*1024, mean per dispatch",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        f = mean(fetch.get(k, [0])) * 1024
        wr = mean(write.get(k, [0])) * 1024
        res["kernels"][k] = {"fetch_reported_bytes": round(f), "write_bytes": round(wr),
                             "hbm_bytes": round(f * (corr or 1.0) + wr) if corr else None}
    if os.path.isdir(os.path.join(d, "lds")):
        unit, per = lds_unit(d)
        idx = per_kernel(os.path.join(d, "lds"), "SQ_LDS_IDX_ACTIVE")
        conf = per_kernel(os.path.join(d, "lds"), "SQ_LDS_BANK_CONFLICT")
        ins = per_kernel(os.path.join(d, "lds"), "SQ_INSTS_LDS")
        res["lds_counter_per_cycle"] = unit
        res["lds_calibration"] = per
        for k in idx:
            if not k.startswith("k_"):
                continue
            e = res["kernels"].setdefault(k, {})
            e["lds_idx_active"] = round(mean(idx[k]))
            e["lds_bank_conflict"] = round(mean(conf.get(k, [0])))
            e["lds_insts"] = round(mean(ins.get(k, [0])))
            e["lds_array_cycles"] = round(mean(idx[k]) / unit) if unit else None
    print(json.dumps(res, indent=1))
    if "--write" in sys.argv:
        path = os.path.join(ROOT, "profiles", "traffic.json")
        try:
            allw = json.load(open(path))
            if "workloads" not in allw:
                allw = {"workloads": {}}
        except (OSError, ValueError):
            allw = {"workloads": {}}
        allw["workloads"][w] = res
        json.dump(allw, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
