"""Print a rocprofv3 kernel_stats.csv sorted by total time (engine kernels only with --engine)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
eng = "--engine" in sys.argv
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if eng and "anonymous namespace" not in r["Name"]:
        continue
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>5} avg_us={float(r['AverageNs']) / 1e3:9.1f} "
          f"tot_ms={float(r['TotalDurationNs']) / 1e6:8.2f}")
