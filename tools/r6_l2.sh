#!/bin/bash
# L2 behaviour per kernel (one rocprofv3 pass per workload: TCC hit / miss, fabric read requests and the
# L1->L2 read requests), plus the rule-table image sizes (PII_VERBOSE).   usage: tools/r6_l2.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for W in config5 scan; do
  PII_VERBOSE=1 timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum \
    --output-format csv -d "$O/l2_$W" -o pmc -- python "$R/bench.py" --workload "$W" --steps 3 --warmup 1 \
    --no-cpu-baseline > "$O/l2_$W.log" 2>&1 || { echo "L2 $W FAILED"; tail -5 "$O/l2_$W.log"; exit 1; }
done
echo L2_OK
