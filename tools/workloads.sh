#!/bin/bash
# The other bench workloads (window re-scan, config-4 stream, long rows, config 5, NER) and the PMC
# pass table of the config-2 bench, one GPU call.   usage: tools/workloads.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/wl_$1
mkdir -p "$O"
WL=${WL:-window stream long config5 ner}
for w in $WL; do
  extra=""
  [ "$w" = config5 ] && extra="--cpu-gb 0.03"     # the config-5 oracle runs ~1.5 MB/s on 16 cores
  timeout -k 10 300 python -u "$R/bench.py" --workload $w $extra > "$O/$w.json" 2> "$O/$w.err" || { echo "BENCH $w FAILED"; tail -5 "$O/$w.err"; exit 1; }
done
timeout -k 10 700 bash "$R/tools/pmc_passes.sh" "gpurun_out/wl_$1/pmc" --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc.log" 2>&1 || { echo PMC_FAIL; exit 1; }
python "$R/tools/pmc_table.py" "$O/pmc" > "$O/pmc_table.txt"
echo WORKLOADS_OK
