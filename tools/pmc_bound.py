"""Per-kernel bound table from tools/pmc_bound.sh (mean per dispatch).
usage: pmc_bound.py DIR [--json OUT]

Columns (shares of SQ_WAVE_CYCLES; SQ counters are in quad-cycles, MI355X_MICROARCH.md):
  VALU / LDS / VMEM / SCA  issue-active cycles by instruction kind (SQ_ACTIVE_INST_*)
  act    all issue-active cycles (SQ_ACTIVE_INST_ANY)
  stall  issue stalls (SQ_WAIT_INST_ANY; LDSst = its LDS part, SQ_WAIT_INST_LDS)
  park   parked on s_waitcnt / barriers (SQ_WAIT_ANY)
  occ    achieved waves per SIMD = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)
  occL   the same from SQ_ACCUM_PREV_HIRES (SQ_LEVEL_WAVES accumulated) when collected
  conf   LDS bank-conflict cycles / LDS-array cycles
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024
XCDS = 8


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            acc[k][(os.path.relpath(f, d).split(os.sep)[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return acc


def mean(cs, c, pas=None):
    vals = [v for (p, n), v in cs.items() if n == c and (pas is None or p == pas)]
    if not vals:
        return None
    flat = [x for v in vals for x in v]
    return sum(flat) / len(flat)


def table(d):
    rows = {}
    for k, cs in load(d).items():
        if not k.startswith("k_"):
            continue
        wc = mean(cs, "SQ_WAVE_CYCLES", "pass1") or mean(cs, "SQ_WAVE_CYCLES")
        if not wc:
            continue
        sh = lambda c: (mean(cs, c) or 0.0) / wc          # noqa: E731
        gui = mean(cs, "GRBM_GUI_ACTIVE", "pass1")
        occ = 4 * wc / (gui / XCDS * SIMDS) if gui else None
        occl = None
        prev, gui3, wc3 = mean(cs, "SQ_ACCUM_PREV_HIRES"), mean(cs, "GRBM_GUI_ACTIVE", "pass3"), None
        if prev and gui3:
            occl = prev / (gui3 / XCDS) / SIMDS
        idx = mean(cs, "SQ_LDS_IDX_ACTIVE")
        rows[k] = dict(wave_cycles=wc, valu=sh("SQ_ACTIVE_INST_VALU"), lds=sh("SQ_ACTIVE_INST_LDS"),
                       vmem=sh("SQ_ACTIVE_INST_VMEM"), sca=sh("SQ_ACTIVE_INST_SCA"), act=sh("SQ_ACTIVE_INST_ANY"),
                       stall=sh("SQ_WAIT_INST_ANY"), lds_stall=sh("SQ_WAIT_INST_LDS"), park=sh("SQ_WAIT_ANY"),
                       occ_waves_per_simd=occ, occ_level=occl,
                       lds_conflict=(mean(cs, "SQ_LDS_BANK_CONFLICT") or 0) / idx if idx else None,
                       valu_insts_M=(mean(cs, "SQ_INSTS_VALU") or 0) / 1e6, lds_insts_M=(mean(cs, "SQ_INSTS_LDS") or 0) / 1e6,
                       waves=mean(cs, "SQ_WAVES"))
    return rows


def main():
    d = sys.argv[1]
    rows = table(d)
    f = lambda x: "   -" if x is None else f"{100 * x:4.0f}"      # noqa: E731
    print(f"{'kernel':26s} {'wcyc_M':>7s} {'VALU':>4s} {'LDS':>4s} {'VMEM':>4s} {'SCA':>4s} {'act':>4s} "
          f"{'stall':>5s} {'LDSst':>5s} {'park':>4s} {'occ':>5s} {'occL':>5s} {'conf':>4s}")
    for k, r in sorted(rows.items(), key=lambda kv: -kv[1]["wave_cycles"]):
        o = "    -" if r["occ_waves_per_simd"] is None else f"{r['occ_waves_per_simd']:5.2f}"
        ol = "    -" if r["occ_level"] is None else f"{r['occ_level']:5.2f}"
        print(f"{k[:26]:26s} {r['wave_cycles'] / 1e6:7.1f} {f(r['valu'])} {f(r['lds'])} {f(r['vmem'])} {f(r['sca'])} "
              f"{f(r['act'])} {f(r['stall']):>5s} {f(r['lds_stall']):>5s} {f(r['park'])} {o} {ol} {f(r['lds_conflict'])}")
    if "--json" in sys.argv:
        json.dump(rows, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
