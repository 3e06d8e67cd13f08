#!/bin/bash
# GPU tests, then the window and config-2 bench lines (wall clock, no profiler) and a rocprof of the window step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-c10}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 $R/bench.py --workload window --steps 20 --warmup 5 --no-cpu-baseline > $O/window.json 2> $O/window.err || { echo W_FAIL; tail -5 $O/window.err; exit 1; }
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/scan.json 2> $O/scan.err || { echo S_FAIL; tail -5 $O/scan.err; exit 1; }
WL=window bash $R/tools/ab_spec.sh ${1:-c10}/wprof - || exit 1
echo C10_OK
