#!/bin/bash
# bound table of one env variant at config 2: tools/r6_pmc1.sh TAG VAR=val
set -o pipefail
TAG=$1; V=$2
R=${GRAFT_REPO_ROOT:-$PWD}
export $V
bash "$R/tools/pmc_bound.sh" "gpurun_out/$TAG" --steps 3 --warmup 1 --no-cpu-baseline || exit 1
python3 "$R/tools/pmc_bound.py" "$R/gpurun_out/$TAG" > "$R/gpurun_out/$TAG.txt" 2>&1 || true
echo PMC_OK
