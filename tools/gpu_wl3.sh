#!/bin/bash
# round-3 workload lines (no CPU baselines) + a kernel-trace summary of the window step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-wl3}
mkdir -p "$O"
for w in window config5 long ner-redact; do
  timeout -k 10 300 python -u "$R/bench.py" --workload $w --no-cpu-baseline > "$O/$w.json" 2> "$O/$w.err" || { echo "BENCH $w FAILED"; tail -5 "$O/$w.err"; exit 1; }
done
timeout -k 10 200 python -u "$R/bench.py" --workload service --clients 64 --requests 60 > "$O/service.json" 2> "$O/service.err" || { echo "BENCH service FAILED"; tail -5 "$O/service.err"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_window" -o run -- python3 "$R/bench.py" --workload window --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof_window.log" 2>&1 || { echo PROF_FAIL; exit 1; }
echo WL_OK
