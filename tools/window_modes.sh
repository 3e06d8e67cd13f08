#!/bin/bash
# Config-3 window re-scan lines: shipped rules (incremental), and config 5's rules incremental vs the
# forced full re-scan.   usage: tools/window_modes.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python bench.py --workload window --steps 20 --warmup 5 --no-cpu-baseline > "$O/window.json" 2> "$O/window.err" || { echo WIN_FAIL; tail -5 "$O/window.err"; exit 1; }
timeout -k 10 600 python bench.py --workload window --window-rules config5 --conversations 50000 --steps 10 --warmup 5 --no-cpu-baseline > "$O/window_c5.json" 2> "$O/window_c5.err" || { echo WINC5_FAIL; tail -5 "$O/window_c5.err"; exit 1; }
timeout -k 10 600 python bench.py --workload window --window-rules config5 --window-full --conversations 50000 --steps 10 --warmup 5 --no-cpu-baseline > "$O/window_c5_full.json" 2> "$O/window_c5_full.err" || { echo WINC5F_FAIL; tail -5 "$O/window_c5_full.err"; exit 1; }
echo WINDOW_MODES_OK
