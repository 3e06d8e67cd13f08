"""Aggregate tools/pmc_traffic.sh output into profiles/traffic.json, keyed by bench workload (read by
bench.py: every workload line quotes only the counters of its own workload, measured on the current
kernel sources, or null).

HBM bytes: FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (TCC EA request counters).  The guide
(MI355X_MICROARCH.md, HBM section) says gfx950 FETCH_SIZE under-reports wide streaming reads by 2x and
that other access shapes must be calibrated.  tools/micro/lane_read reads exactly 1200 MiB per
dispatch in four patterns, and each gives its own correction (bytes read / FETCH_SIZE bytes):
  lane_rev  k_lane_rev   per-lane 1 KiB ranges, right to left, 64-byte blocks (k_scan's text reads)
  stream16  k_coalesced  16 B per lane, consecutive (k_redact's text reads and tile stores' sources)
  stream8   k_stream8    8 B per lane (the scan events, pair records: the queue kernels' main loads)
  stream4   k_stream4    4 B per lane (offsets / counts / per-lane scalars)
  walk16    k_walk16     per-lane forward walks of 6 16-byte records, neighbouring lanes adjacent
                         (k_select's SelRec walk over each lane's matched pairs; round 6)
  gather16  k_gather16   16-byte records in a scattered order (k_pair_first / k_pair_eval: pair and
                         event records and text windows gathered per pair; round 6).  Its FETCH_SIZE is
                         4x the record bytes: each record costs a 64-byte line (CALIB_LINE_MULT), so the
                         correction is taken against the line bytes (~1.0), not the useful bytes
Every engine kernel is assigned the pattern of its dominant read stream (KERNEL_PATTERN), and its
hbm_bytes = FETCH_SIZE x that pattern's correction + WRITE_SIZE.  (one global factor,
calibrated on k_scan's pattern, under-counted k_redact's coalesced stream.)  Where the bench line
gives the work sizes, the kernel's algorithmic bytes and traffic / algorithmic ratio
are stored beside it.

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
CALIB_KERNELS = {"lane_rev": "k_lane_rev", "stream16": "k_coalesced", "stream8": "k_stream8", "stream4": "k_stream4",
                 "walk16": "k_walk16", "gather16": "k_gather16"}
# HBM bytes one calibration launch really moves, as a multiple of the bytes it reads: a scattered 16-byte
# gather brings a whole 64-byte line per record (its FETCH_SIZE reads 4x the record bytes: the counter is
# right at 64-byte requests, and the line's unused 48 bytes are real HBM traffic), so its correction is
# taken against the line bytes, not the record bytes.  Every other pattern reads each byte of its lines.
CALIB_LINE_MULT = {"gather16": 4}
# dominant read stream per engine kernel (name prefix); anything else: stream8
KERNEL_PATTERN = {"k_scan": "lane_rev", "k_scan_fix": "lane_rev", "k_redact": "stream16", "k_win_redact": "stream16",
                  "k_win_join": "stream16", "k_lane_bits": "stream8", "k_chunk_index": "stream8",
                  "k_pairs_flat": "stream8", "k_pairs_merge": "stream8", "k_pair_first": "gather16",
                  "k_pair_eval": "gather16", "k_select": "walk16", "k_sel_fix": "walk16", "k_spans": "stream8",
                  "k_ctx_scan": "stream4",
                  "k_ctx_apply": "stream4", "k_ctx_commit": "stream4", "k_lane_count": "stream4",
                  "k_lane_place": "stream4", "k_scan_reduce": "stream4", "k_scan_apply": "stream4",
                  "k_scan_blocks": "stream4", "k_scan_lb": "stream4", "k_tile_first": "stream8",
                  "k_hist_reduce": "stream4"}


def pattern_of(kernel):
    base = kernel.split("<")[0]
    return KERNEL_PATTERN.get(base, "stream8")


def algorithmic_bytes(kernel, b):
    """DESIGN.md §6 algorithmic bytes of one launch, from the bench line b (None if not derivable)"""
    if not b or "queues_per_step_per_gpu" not in b:
        return None
    n_bytes = b["config"].get("bytes_per_gpu")
    U = b["config"].get("utterances_per_gpu")
    q = b["queues_per_step_per_gpu"]
    E, P = q.get("scan_events", 0), q.get("candidate_pairs", 0)
    S = b.get("spans_per_step_per_gpu", 0)
    lanes = (n_bytes + 1023) // 1024
    base = kernel.split("<")[0]
    if base == "k_scan" and kernel.startswith("k_scan<true"):
        return b.get("roofline", {}).get("algorithmic_bytes")
    if base == "k_redact":
        return b.get("roofline_redact", {}).get("algorithmic_bytes")
    if base == "k_pairs_flat" and "<false" in kernel:
        # events in; the wavefronts' row offsets + roles staged; lane counts in, pair counts out
        return 8 * E + 8 * (U + 1) + U + 12 * lanes
    if base == "k_pairs_flat":
        return 8 * E + 8 * (U + 1) + 16 * E + 8 * P + 24 * lanes   # events + row offsets in; EvLoc + pairs out
    if base == "k_spans":
        # findings in, each one's row input / output base; API spans + RSpans out
        return 16 * S + 16 * S + 32 * S + 16 * lanes
    if base == "k_lane_bits":
        return 8 * ((n_bytes + 63) // 64) + 8 * U + 16 * lanes   # start words out; offsets + lanes in
    if base == "k_chunk_index":
        return 8 * (U + 1) + U + 4 * U + 4 * U                   # offsets + roles in; defaults out
    return None


def per_kernel(d, counter, tail=None):
    """counter value per dispatch, per kernel (dispatch order); tail = (steps, total steps): keep only
    the dispatches of the last `steps` of `total` bench steps (the timed, steady-state ones: a window
    re-scan's first N steps fill the windows)"""
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            acc[(k, int(r.get("Dispatch_Id", len(acc))))].append(float(r["Counter_Value"]))
    out = defaultdict(list)
    for (k, _), v in sorted(acc.items(), key=lambda kv: kv[0][1]):
        out[k].append(sum(v))          # sum over the counter's instances of one dispatch
    if tail:
        steps, total = tail
        for k in out:
            n = len(out[k])
            if n >= total and n % total == 0:            # the kernel runs n / total times per step
                out[k] = out[k][n - n // total * steps:]
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
    bench = [json.loads(l) for l in open(os.path.join(d, "fetch.log")) if l.startswith("{")]
    tail = None
    if bench and w.startswith("window"):
        # only the timed steps: the bench's warm-up fills the windows (warmup >= N)
        K, W0 = int(bench[-1]["steps"]), int(bench[-1]["warmup"])
        tail = (K, K + W0 + int(bench[-1].get("probe_steps", 0)))     # (+ the stage probe's calls)
    fetch = per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE", tail)
    write = per_kernel(os.path.join(d, "write"), "WRITE_SIZE", tail)
    calib = per_kernel(os.path.join(d, "calib"), "FETCH_SIZE")
    # every lane_read launch reads CALIB_BYTES (k_lane_rev at 512/1024/2048 B per lane, the streams)
    corrs = {pat: (CALIB_BYTES * CALIB_LINE_MULT.get(pat, 1) / (mean(calib[k]) * 1024) if calib.get(k) else None)
             for pat, k in CALIB_KERNELS.items()}
    corr = corrs["lane_rev"]
    cfg = bench[-1]["config"] if bench else {}
    n_bytes = cfg.get("resident_stream_bytes", cfg.get("bytes_per_gpu", cfg.get("bytes_per_step"))) if bench else None
    h = hashlib.sha256()
    for f in SOURCES:
        h.update(open(os.path.join(ROOT, f), "rb").read())
    res = {"workload": w, "source_digest": h.hexdigest()[:16], "bytes_per_gpu": n_bytes, "fetch_correction": corr,
           "fetch_corrections": corrs,
           "note": "hbm_bytes = FETCH_SIZE*1024*fetch_corrections[fetch_pattern] + WRITE_SIZE*1024, mean per "
                   "dispatch; algorithmic_bytes per DESIGN.md section 6 from the bench line's work sizes",
           "kernels": {}}
    b = bench[-1] if bench else None
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        f = mean(fetch.get(k, [0])) * 1024
        wr = mean(write.get(k, [0])) * 1024
        pat = pattern_of(k)
        c = corrs.get(pat) or corrs.get("stream8")        # (an older calibration run: no walk / gather)
        e = {"fetch_reported_bytes": round(f), "write_bytes": round(wr), "fetch_pattern": pat,
             "hbm_bytes": round(f * c + wr) if c else None}
        ab = algorithmic_bytes(k, b)
        if ab:
            e["algorithmic_bytes"] = int(ab)
            if e["hbm_bytes"]:
                e["traffic_over_algorithmic"] = round(e["hbm_bytes"] / ab, 3)
        res["kernels"][k] = e
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
