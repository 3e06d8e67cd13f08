#!/bin/bash
# A/B of one workload (WL, default window; specs as tools/ab_spec.sh), then the whole GPU test
# suite.   usage: tools/r6_ab_full.sh TAG [extra ab specs...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
T=$1; shift
WL=${WL:-window} bash "$R/tools/ab_spec.sh" "$T" "$@" || exit 1
cd "$R" && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "gpurun_out/$T/tests.log" 2>&1 || { echo TESTS FAILED; tail -30 "gpurun_out/$T/tests.log"; exit 1; }
tail -2 "gpurun_out/$T/tests.log"
echo FULL_OK
