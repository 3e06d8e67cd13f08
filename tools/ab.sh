#!/bin/bash
# A/B kernel timing of alternative builds of libpii.so in one GPU call: a rocprofv3 kernel-trace summary
# of the config-2 bench (or WL=<workload>) per library.   usage: [WL=window] tools/ab.sh TAG LIB...   (LIB = path relative to the repo)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for L in "$@"; do
  i=$((i+1))
  PII_LIB=$R/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/v$i" -o run -- python3 "$R/bench.py" --workload "${WL:-scan}" --steps 10 --warmup 3 --no-cpu-baseline > "$O/v$i.json" 2> "$O/v$i.err" || { echo "FAIL $L"; tail -5 "$O/v$i.err"; exit 1; }
done
echo AB_OK
