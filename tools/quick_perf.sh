#!/bin/bash
# GPU tests + default bench + kernel-trace stats (one call)  usage: tools/quick_perf.sh TAG [pytest-args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAIL; tail -30 "$O/gpu_tests.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { echo BENCH_FAIL; tail -5 "$O/bench.err"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo PROF_FAIL; exit 1; }
echo QUICK_OK
