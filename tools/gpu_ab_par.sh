#!/bin/bash
# parity tests of the current tree, then an A/B of libraries: tools/gpu_ab_par.sh TAG "TESTS" LIB...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=$1; shift; TESTS=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest $TESTS -x -v -m gpu --timeout 300 --timeout-method thread > "$O/t.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$O/t.log"; exit 1; }
bash tools/ab.sh $TAG/ab "$@" > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
echo ABPAR_OK
