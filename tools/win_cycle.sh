#!/bin/bash
# window re-scan (config 3) on one GPU: bench + kernel-trace profile.  usage: tools/win_cycle.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
R=$PWD
O=$R/gpurun_out/win_$TAG
mkdir -p "$O"
timeout -k 10 600 python bench.py --workload window "$@" > "$O/bench.log" 2>&1 || { echo "BENCH FAILED"; tail -30 "$O/bench.log"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python "$R/bench.py" --workload window --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo "PROF FAILED"; exit 1; }
echo WIN_OK
