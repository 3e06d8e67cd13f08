import csv, json, sys
tag = sys.argv[1]
try:
    d = json.loads(open(f"gpurun_out/bench_{tag}.log").read().strip().splitlines()[-1])
    print("value MB/s", d["value"], "ms/step", d["ms_per_step"], d.get("stages_ms"), d["kernels_ms"])
    print("roofline", d["roofline"], "\nredact", d.get("roofline_redact"), "\ncpu", d.get("cpu_baseline"), "\nqueues", d.get("queues_per_step_per_gpu"))
except Exception as e:
    print("no bench", e)
try:
    for x in csv.DictReader(open(f"gpurun_out/prof_{tag}/run_kernel_stats.csv")):
        if "k_" in x["Name"]:
            print("  ", x["Name"].replace("(anonymous namespace)::", "").split("(")[0].ljust(16), x["Calls"].rjust(3), f"{float(x['AverageNs'])/1e3:10.1f} us")
except Exception as e:
    print("no prof", e)
