#!/bin/bash
# Round evidence, part B (one GPU call, after profiles/traffic.json holds the PMC passes of these
# sources): every bench workload line, the config-2 headline with its CPU baseline.
# usage: tools/evidence_bench.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
run() {   # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/bench_$n.log" 2>&1 || { echo "BENCH $n FAILED"; tail -5 "$O/bench_$n.log"; return 1; }
  grep '^{' "$O/bench_$n.log" | tail -1 > "$O/bench_$n.json"
  python3 -c "import json,sys; b=json.load(open(sys.argv[1])); print(sys.argv[2], b['value'], b['unit'], b['ms_per_step'])" "$O/bench_$n.json" "$n"
}
run scan 600 && run window 300 --workload window --steps 20 --warmup 5 --no-cpu-baseline && \
run window_config5 600 --workload window --window-rules config5 --conversations 50000 --steps 10 --warmup 5 --no-cpu-baseline && \
run config5 600 --workload config5 --no-cpu-baseline && run long 300 --workload long --no-cpu-baseline && \
run stream 600 --workload stream --no-cpu-baseline && run ner 300 --workload ner --no-cpu-baseline && \
run ner-redact 300 --workload ner-redact --no-cpu-baseline && \
run service8 300 --workload service --clients 8 --no-cpu-baseline && \
run service64 300 --workload service --clients 64 --no-cpu-baseline && echo EVIDENCE_B_OK
