"""Compact per-kernel table of tools/pmc_passes.sh output (mean per dispatch).
usage: pmc_table.py DIR  -- FETCH/WRITE in MB (FETCH_SIZE raw KiB x 1024, uncorrected), instruction counts in
millions, wave-cycle shares: WAIT_ANY (parked on s_waitcnt/barrier), WAIT_INST (issue stalls), ACTIVE."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
m = lambda cs, c: sum(cs.get(c, [0])) / max(1, len(cs.get(c, [0])))
print(f"{'kernel':22s} {'fetchMB':>8s} {'writeMB':>8s} {'VALU_M':>7s} {'LDS_M':>6s} {'VMRD_M':>6s} "
      f"{'waves':>7s} {'wcyc_M':>8s} {'wait%':>6s} {'stall%':>6s} {'act%':>5s} {'ldsconf':>7s}")
for k, cs in sorted(acc.items(), key=lambda kv: -m(kv[1], "SQ_WAVE_CYCLES")):
    if not k.startswith("k_"):
        continue
    wc = m(cs, "SQ_WAVE_CYCLES") or 1
    idx = m(cs, "SQ_LDS_IDX_ACTIVE") or 1
    print(f"{k[:22]:22s} {m(cs, 'FETCH_SIZE') * 1024 / 1e6:8.1f} {m(cs, 'WRITE_SIZE') * 1024 / 1e6:8.1f} "
          f"{m(cs, 'SQ_INSTS_VALU') / 1e6:7.1f} {m(cs, 'SQ_INSTS_LDS') / 1e6:6.1f} {m(cs, 'SQ_INSTS_VMEM_RD') / 1e6:6.1f} "
          f"{m(cs, 'SQ_WAVES'):7.0f} {wc / 1e6:8.1f} {100 * m(cs, 'SQ_WAIT_ANY') / wc:6.1f} "
          f"{100 * m(cs, 'SQ_WAIT_INST_ANY') / wc:6.1f} {100 * m(cs, 'SQ_ACTIVE_INST_ANY') / wc:5.1f} "
          f"{m(cs, 'SQ_LDS_BANK_CONFLICT') / idx:7.2f}")
