#!/bin/bash
# round-6 k_scan2 cycle: GPU tests of the in-tree build, then kernel A/B (env variants, then libraries)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTS:-} > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAIL; tail -60 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
fi
bash "$R/tools/ab_env.sh" "$TAG/env" "PII_SCAN2=0" "PII_SCAN2=1" || exit 1
if [ $# -gt 0 ]; then bash "$R/tools/ab.sh" "$TAG/lib" "$@" || exit 1; fi
echo CYCLE_OK
