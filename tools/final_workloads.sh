#!/bin/bash
# Config-5 L2 hit-rate pass (written to profiles/config5_l2.json on these sources, so the config-5 line
# carries it), then tools/workloads.sh.   usage: tools/final_workloads.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/l2_$1
mkdir -p "$O"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$O/pmc" -o run -- python3 "$R/bench.py" --workload config5 --steps 1 --warmup 1 --no-cpu-baseline > "$O/pmc.log" 2>&1) || { echo L2_FAIL; exit 1; }
python "$R/tools/pmc_l2.py" "$O/pmc" --write > "$O/l2.txt" || { echo L2_SUMMARY_FAIL; exit 1; }
bash "$R/tools/workloads.sh" "$1"
