#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/c9; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash $R/tools/ab_spec.sh c9/ab - exp_libs/abl2.so exp_libs/abl3.so || exit 1
timeout -k 10 600 python3 $R/bench.py --workload config5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { echo C5_FAIL; tail -5 $O/c5.err; exit 1; }
echo C9_OK
