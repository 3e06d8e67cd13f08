#!/bin/bash
# HBM traffic of the roofline kernels from PMC counters, in separate rocprofv3 passes (FETCH_SIZE and
# WRITE_SIZE never share a pass, no tracing mixed in), plus a FETCH_SIZE calibration of the scan's
# per-lane read pattern on a kernel with a known byte count (tools/micro/lane_read).
# usage (on the GPU box): tools/pmc_traffic.sh OUTDIR [bench args...]; then tools/pmc_traffic.py OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o pmc -- python "$R/bench.py" "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o pmc -- python "$R/bench.py" "$@" > "$OUT/write.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib" -o pmc -- "$R/tools/micro/lane_read" > "$OUT/calib.log" 2>&1
echo PMC_TRAFFIC_OK
