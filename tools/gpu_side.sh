#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/side1
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$O/t.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$O/t.log"; exit 1; }
for L in exp_libs/libpii_h2.so context-based-pii_amd/libpii.so; do
  n=$(basename $L .so)
  PII_LIB=$R/$L timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/bench_$n.json" 2> "$O/bench_$n.err" || exit 1
  PII_LIB=$R/$L timeout -k 10 300 python bench.py --workload window --no-cpu-baseline > "$O/win_$n.json" 2> "$O/win_$n.err" || exit 1
done
bash tools/ab.sh side1/ab exp_libs/libpii_h2.so exp_libs/libpii_side.so context-based-pii_amd/libpii.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
echo SIDE_OK
