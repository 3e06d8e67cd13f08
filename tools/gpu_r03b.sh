#!/bin/bash
# round-3 GPU call: the service NOMEM test, the service bench (client processes), k_redact A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r03b
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_service.py -x -v -m gpu -k "nomem" --timeout 250 --timeout-method thread > "$O/t.log" 2>&1
rc=$?; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_config5.py -x -v -m gpu --timeout 400 --timeout-method thread > "$O/t5.log" 2>&1
rc=$?; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
timeout -k 10 400 python bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/c5.json" 2> "$O/c5.err"
rc=$?; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
bash tools/ab.sh r03b/ab exp_libs/libpii_u1.so context-based-pii_amd/libpii.so exp_libs/libpii_u4.so > "$O/ab.log" 2>&1 || exit 1
for c in 8 64 256; do
  timeout -k 10 200 python bench.py --workload service --clients $c --requests 60 --batch-wait-ms 2 > "$O/s_$c.json" 2> "$O/s_$c.err" || exit 1
done
echo R03B_OK
