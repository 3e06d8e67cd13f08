#!/bin/bash
# the two window bench lines of tools/evidence_bench.sh, alone (after a bench.py change that touches
# only the window loop).   usage: tools/r6_win_lines.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$1
mkdir -p "$O"
run() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/bench_$n.log" 2>&1 || { echo "BENCH $n FAILED"; tail -5 "$O/bench_$n.log"; return 1; }
  grep '^{' "$O/bench_$n.log" | tail -1 > "$O/bench_$n.json"
  python3 -c "import json,sys; b=json.load(open(sys.argv[1])); print(sys.argv[2], b['value'], b['unit'], b['ms_per_step'])" "$O/bench_$n.json" "$n"
}
run window 300 --workload window --steps 20 --warmup 5 --no-cpu-baseline && \
run window_config5 600 --workload window --window-rules config5 --conversations 50000 --steps 10 --warmup 5 --no-cpu-baseline && echo WIN_LINES_OK
