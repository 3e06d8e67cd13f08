#!/bin/bash
# whole GPU test suite, then the config-2 and window bench lines (no profiler).   usage: tools/r6_quick.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$1
mkdir -p "$O"
cd "$R" && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS FAILED; tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for a in "scan:" "window:--workload window --steps 20 --warmup 5"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python -u bench.py $args --no-cpu-baseline > "$O/bench_$n.log" 2>&1 || { echo "BENCH $n FAILED"; tail -5 "$O/bench_$n.log"; exit 1; }
  grep '^{' "$O/bench_$n.log" | tail -1 > "$O/bench_$n.json"
  python3 -c "import json,sys; b=json.load(open(sys.argv[1])); print(sys.argv[2], b['value'], b['ms_per_step'])" "$O/bench_$n.json" "$n"
done
echo QUICK_OK
