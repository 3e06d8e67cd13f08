import csv, json, sys
tag = sys.argv[1]
try:
    d = json.loads(open(f"gpurun_out/bench_{tag}.log").read().strip().splitlines()[-1])
    print("value MB/s", d["value"], "ms/step", d["ms_per_step"], d["kernels_ms"], "roofline", d["roofline"]["achieved"], d["roofline"]["frac"])
except Exception as e:
    print("no bench", e)
try:
    for x in csv.DictReader(open(f"gpurun_out/prof_{tag}/run_kernel_stats.csv")):
        if "k_" in x["Name"]:
            print("  ", x["Name"].replace("(anonymous namespace)::", "").split("(")[0].ljust(16), x["Calls"].rjust(3), f"{float(x['AverageNs'])/1e3:10.1f} us")
except Exception as e:
    print("no prof", e)
