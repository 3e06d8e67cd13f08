#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-c5p}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --workload config5 --steps 5 --warmup 2 --no-cpu-baseline > "$O/c5.json" 2> "$O/c5.err" || { echo PROF_FAIL; tail "$O/c5.err"; exit 1; }
echo C5_OK
