#!/bin/bash
# Round evidence in one call, PMC passes first so the bench line carries the traffic of these sources:
# gpu tests, smoke(), PMC traffic -> profiles/traffic.json (copied out), bench (with the CPU baseline),
# rocprofv3 kernel-trace summary of the same bench.   usage: tools/round_run.sh TAG
set -o pipefail
TAG=$1
R=$PWD
O=$R/gpurun_out/round_$TAG
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "TESTS FAILED"; tail -40 "$O/gpu_tests.log"; exit 1; }
timeout -k 10 300 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || { echo "SMOKE FAILED"; tail -20 "$O/smoke.log"; exit 1; }
bash tools/pmc_traffic.sh "gpurun_out/round_$TAG/traffic" scan --steps 2 --warmup 1 --no-cpu-baseline > "$O/traffic.log" 2>&1 || { echo "PMC FAILED"; exit 1; }
python tools/pmc_traffic.py "gpurun_out/round_$TAG/traffic" --workload scan > "$O/traffic.json" || { echo "PMC SUMMARY FAILED"; exit 1; }
timeout -k 10 600 python bench.py > "$O/bench.log" 2>&1 || { echo "BENCH FAILED"; tail -20 "$O/bench.log"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo "PROF FAILED"; exit 1; }
echo ROUND_OK
