#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${1:-pmct}
mkdir -p "$O"
timeout -k 10 900 bash "$R/tools/pmc_passes.sh" "gpurun_out/${1:-pmct}/pmc" --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc.log" 2>&1 || { echo PMC_FAIL; tail -5 "$O/pmc.log"; exit 1; }
python "$R/tools/pmc_table.py" "$O/pmc" > "$O/pmc_table.txt" || exit 1
echo PMCT_OK
