#!/bin/bash
# Round-3 evidence in one GPU call: every -m gpu test, smoke(), the config-2 bench line (with the CPU
# baseline), its rocprofv3 kernel-trace summary, PMC passes per workload (HBM bytes, and LDS-array
# cycles for the scan workloads: tools/pmc_traffic.sh), then the bench lines of the other workloads
# re-run so that they quote their own counters.   usage: tools/evidence_r03.sh TAG [quick]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$1
mkdir -p "$O"
stop() { echo "STOPPED at $1 (rc $2)"; exit 1; }
if [ "$2" != quick ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || stop tests $?
  timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || stop smoke $?
fi
for W in scan long config5 window; do
  bash "$R/tools/pmc_traffic.sh" "gpurun_out/$1/pmc_$W" "$W" --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc_$W.log" 2>&1 || stop "pmc $W" $?
  python "$R/tools/pmc_traffic.py" "gpurun_out/$1/pmc_$W" --workload "$W" --write > "$O/traffic_$W.json" || stop "pmc summary $W" $?
done
cp "$R/profiles/traffic.json" "$O/traffic.json"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || stop bench $?
for W in long config5 window ner ner-redact service stream; do
  timeout -k 10 400 python bench.py --workload "$W" --steps 5 --warmup 2 > "$O/bench_$W.json" 2> "$O/bench_$W.err" || stop "bench $W" $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/prof.log" 2>&1 || stop prof $?
echo EVIDENCE_OK
