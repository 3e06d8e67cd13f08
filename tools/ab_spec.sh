#!/bin/bash
# A/B kernel timing of (library, environment) variants: each spec is LIB[:VAR=val[,VAR=val...]] (LIB
# relative to the repo, "-" = the in-tree build).  usage: [WL=..] tools/ab_spec.sh TAG SPEC...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for S in "$@"; do
  i=$((i+1))
  L=${S%%:*}; E=""; [ "$L" != "$S" ] && E=${S#*:}
  ( [ "$L" != "-" ] && export PII_LIB=$R/$L
    for kv in ${E//,/ }; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/v$i" -o run -- python3 "$R/bench.py" --workload "${WL:-scan}" --steps 10 --warmup 3 --no-cpu-baseline > "$O/v$i.json" 2> "$O/v$i.err" ) || { echo "FAIL $S"; tail -5 "$O/v$i.err"; exit 1; }
  echo "v$i = $S"
done
echo AB_OK
