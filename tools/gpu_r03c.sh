#!/bin/bash
# round-3 re-entry: every -m gpu test, smoke(), the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-r03c}
mkdir -p "$O"
stop() { echo "STOPPED at $1 (rc $2)"; exit 1; }
timeout -k 10 840 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || stop tests $?
timeout -k 10 200 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || stop smoke $?
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || stop bench $?
echo R03C_OK
