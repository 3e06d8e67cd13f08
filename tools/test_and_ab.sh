#!/bin/bash
# GPU parity tests of the in-tree build, then an A/B kernel-time comparison of alternative builds.
# usage: tools/test_and_ab.sh TAG [LIB...]   (LIB = path relative to the repo; tools/ab.sh)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAIL; tail -40 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
if [ $# -gt 0 ]; then bash "$R/tools/ab.sh" "$TAG/ab" "$@" || exit 1; fi
echo CYCLE_OK
