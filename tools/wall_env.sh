#!/bin/bash
# wall-clock bench lines of one workload under environment variants (no profiler).
# usage: WL=config5 tools/wall_env.sh TAG "VAR=x" "VAR=y" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for V in "$@"; do
  i=$((i+1))
  env $V timeout -k 10 300 python bench.py --workload "${WL:-scan}" --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/v$i.json 2>&1 || exit 1
done
echo WALL_OK
