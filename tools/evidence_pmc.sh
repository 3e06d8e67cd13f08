#!/bin/bash
# Round evidence, part A (one GPU call): GPU tests, smoke(), the PMC passes of every workload that
# bench.py quotes traffic for, and rocprofv3 kernel-trace summaries.  Part B (tools/evidence_bench.sh)
# runs the bench lines after profiles/traffic.json has been refreshed from these passes
# (python tools/pmc_traffic.py gpurun_out/TAG/traffic_W --workload W --write, here in the container).
# usage: tools/evidence_pmc.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "TESTS FAILED"; tail -40 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || { echo "SMOKE FAILED"; tail -20 "$O/smoke.log"; exit 1; }
for W in scan config5 window long; do
  bash tools/pmc_traffic.sh "gpurun_out/$TAG/traffic_$W" "$W" --steps 2 --warmup 1 --no-cpu-baseline > "$O/traffic_$W.log" 2>&1 || { echo "PMC $W FAILED"; tail -5 "$O/traffic_$W.log"; exit 1; }
  echo "PMC $W ok"
done
# the window re-scan under the config-5 rules (its bench line's traffic field)
bash tools/pmc_traffic.sh "gpurun_out/$TAG/traffic_window_config5" window --window-rules config5 --conversations 50000 --steps 2 --warmup 1 --no-cpu-baseline > "$O/traffic_window_config5.log" 2>&1 || { echo "PMC window_config5 FAILED"; tail -5 "$O/traffic_window_config5.log"; exit 1; }
echo "PMC window_config5 ok"
# bound / occupancy passes (wave-cycle split, achieved waves per SIMD) of every k_scan instantiation:
# config 2 (group 0), config 5 (narrow and WIDE groups), the window step
for W in scan config5 window; do
  bash tools/pmc_bound.sh "gpurun_out/$TAG/bound_$W" --workload "$W" --steps 2 --warmup 1 --no-cpu-baseline > "$O/bound_$W.log" 2>&1 || { echo "BOUND $W FAILED"; tail -5 "$O/bound_$W.log"; exit 1; }
  echo "BOUND $W ok"
done
cd /tmp && export TMPDIR=/tmp
for W in scan config5 window; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$W" -o run -- python "$R/bench.py" --workload "$W" --steps 10 --warmup 3 --no-cpu-baseline > "$O/prof_$W.log" 2>&1 || { echo "PROF $W FAILED"; exit 1; }
done
echo EVIDENCE_A_OK
