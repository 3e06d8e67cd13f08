#!/bin/bash
# A/B kernel timing of one library under environment variants (e.g. PII_FUSE=0 / 1): a rocprofv3
# kernel-trace summary of the config-2 bench (or WL=<workload>) per variant.   usage: [WL=..] tools/ab_env.sh TAG "VAR=x" "VAR=y" ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for V in "$@"; do
  i=$((i+1))
  export $V
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/v$i" -o run -- python3 "$R/bench.py" --workload "${WL:-scan}" --steps 10 --warmup 3 --no-cpu-baseline > "$O/v$i.json" 2> "$O/v$i.err" || { echo "FAIL $V"; tail -5 "$O/v$i.err"; exit 1; }
done
echo AB_OK
