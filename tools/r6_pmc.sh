#!/bin/bash
# bound tables of k_scan (PII_SCAN2=0) and k_scan2 (PII_SCAN2=1) at config 2
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$PWD}
for v in 0 1; do
  PII_SCAN2=$v bash "$R/tools/pmc_bound.sh" "gpurun_out/$TAG/s$v" --steps 3 --warmup 1 --no-cpu-baseline || exit 1
  python3 "$R/tools/pmc_bound.py" "$R/gpurun_out/$TAG/s$v" > "$R/gpurun_out/$TAG/s$v.txt" 2>&1 || true
done
echo PMC_OK
