#!/bin/bash
# Round-3 evidence in two GPU calls (each well inside gpurun's limit):
#   part 1: every -m gpu test, smoke(), the config-2 PMC passes (HBM bytes, LDS-array cycles:
#           tools/pmc_traffic.sh), the config-2 bench line (with the CPU baseline) quoting them, and
#           its rocprofv3 kernel-trace summary
#   part 2: PMC passes of the long / config5 / window workloads, then every other workload's line
#           (each quoting its own counters), a kernel-trace summary of config 5 and of the window step
# usage: tools/evidence_r03.sh TAG 1|2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$1
mkdir -p "$O"
stop() { echo "STOPPED at $1 (rc $2)"; exit 1; }
if [ "$2" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || stop tests $?
  timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || stop smoke $?
  bash "$R/tools/pmc_traffic.sh" "gpurun_out/$1/pmc_scan" scan --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc_scan.log" 2>&1 || stop "pmc scan" $?
  python "$R/tools/pmc_traffic.py" "gpurun_out/$1/pmc_scan" --workload scan --write > "$O/traffic_scan.json" || stop "pmc summary scan" $?
  timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || stop bench $?
  cp "$R/profiles/traffic.json" "$O/traffic.json"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/prof.log" 2>&1 || stop prof $?
else
  [ -f "$R/gpurun_out/$3/traffic.json" ] && cp "$R/gpurun_out/$3/traffic.json" "$R/profiles/traffic.json"
  for W in long config5 window; do
    bash "$R/tools/pmc_traffic.sh" "gpurun_out/$1/pmc_$W" "$W" --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc_$W.log" 2>&1 || stop "pmc $W" $?
    python "$R/tools/pmc_traffic.py" "gpurun_out/$1/pmc_$W" --workload "$W" --write > "$O/traffic_$W.json" || stop "pmc summary $W" $?
  done
  cp "$R/profiles/traffic.json" "$O/traffic.json"
  for W in long config5 window ner ner-redact stream; do
    extra=""
    [ "$W" = config5 ] && extra="--cpu-gb 0.03"
    timeout -k 10 400 python bench.py --workload "$W" $extra > "$O/bench_$W.json" 2> "$O/bench_$W.err" || stop "bench $W" $?
  done
  timeout -k 10 300 python bench.py --workload service --clients 64 --requests 100 > "$O/bench_service.json" 2> "$O/bench_service.err" || stop "bench service" $?
  timeout -k 10 300 python bench.py --workload service --clients 8 --requests 100 > "$O/bench_service8.json" 2> "$O/bench_service8.err" || stop "bench service8" $?
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c5" -o run -- python3 "$R/bench.py" --workload config5 --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof_c5.log" 2>&1 || stop prof_c5 $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_win" -o run -- python3 "$R/bench.py" --workload window --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof_win.log" 2>&1 || stop prof_win $?
fi
echo EVIDENCE_OK
