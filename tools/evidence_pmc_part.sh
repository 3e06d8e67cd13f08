#!/bin/bash
# tools/evidence_pmc.sh split over two GPU calls (each within gpurun's 20-minute limit):
#   PART=1: GPU tests, smoke(), PMC traffic of scan / config5 / long
#   PART=2: PMC traffic of window / window_config5, bound passes, rocprofv3 kernel-trace summaries
# usage: PART=1|2 tools/evidence_pmc_part.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
if [ "$PART" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "TESTS FAILED"; tail -40 "$O/gpu_tests.log"; exit 1; }
  tail -1 "$O/gpu_tests.log"
  timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || { echo "SMOKE FAILED"; tail -20 "$O/smoke.log"; exit 1; }
  for W in scan config5 long; do
    bash tools/pmc_traffic.sh "gpurun_out/$TAG/traffic_$W" "$W" --steps 2 --warmup 1 --no-cpu-baseline > "$O/traffic_$W.log" 2>&1 || { echo "PMC $W FAILED"; tail -5 "$O/traffic_$W.log"; exit 1; }
    echo "PMC $W ok"
  done
  echo EVIDENCE_A1_OK
  exit 0
fi
bash tools/pmc_traffic.sh "gpurun_out/$TAG/traffic_window" window --steps 2 --warmup 1 --no-cpu-baseline > "$O/traffic_window.log" 2>&1 || { echo "PMC window FAILED"; tail -5 "$O/traffic_window.log"; exit 1; }
echo "PMC window ok"
bash tools/pmc_traffic.sh "gpurun_out/$TAG/traffic_window_config5" window --window-rules config5 --conversations 50000 --steps 2 --warmup 1 --no-cpu-baseline > "$O/traffic_window_config5.log" 2>&1 || { echo "PMC window_config5 FAILED"; tail -5 "$O/traffic_window_config5.log"; exit 1; }
echo "PMC window_config5 ok"
for W in scan config5 window; do
  bash tools/pmc_bound.sh "gpurun_out/$TAG/bound_$W" --workload "$W" --steps 2 --warmup 1 --no-cpu-baseline > "$O/bound_$W.log" 2>&1 || { echo "BOUND $W FAILED"; tail -5 "$O/bound_$W.log"; exit 1; }
  echo "BOUND $W ok"
done
cd /tmp && export TMPDIR=/tmp
for W in scan config5 window; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$W" -o run -- python "$R/bench.py" --workload "$W" --steps 10 --warmup 3 --no-cpu-baseline > "$O/prof_$W.log" 2>&1 || { echo "PROF $W FAILED"; exit 1; }
done
echo EVIDENCE_A2_OK
