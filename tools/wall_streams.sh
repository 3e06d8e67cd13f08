#!/bin/bash
# wall-clock config-5 bench per PII_SCAN_STREAMS value (SCAN passes on 1-3 streams).  usage: tools/wall_streams.sh N...
set -o pipefail
for n in "$@"; do
  PII_SCAN_STREAMS=$n PII_LIB=${PII_LIB:-$PWD/context-based-pii_amd/libpii.so} timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/wall_streams_$n.json 2>&1 || exit 1
done
