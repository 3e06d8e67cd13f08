#!/bin/bash
# PMC evidence for one bench workload, each counter group in its own rocprofv3 pass (FETCH_SIZE and
# WRITE_SIZE never share a pass, no tracing mixed in):
#   fetch / write      HBM bytes per dispatch (TCC EA request counters)
#   calib              FETCH_SIZE of tools/micro/lane_read (known bytes, k_scan's read pattern)
#   lds / lds_calib    SQ_LDS_IDX_ACTIVE / SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS of the workload and of
#                      tools/micro/lds_calib (known LDS-array cycles), scan workloads only
# usage (on the GPU box): tools/pmc_traffic.sh OUTDIR WORKLOAD [bench args...]; then
#                         tools/pmc_traffic.py OUTDIR --workload WORKLOAD [--write]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1; shift
W=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o pmc -- python "$R/bench.py" --workload "$W" "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o pmc -- python "$R/bench.py" --workload "$W" "$@" > "$OUT/write.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib" -o pmc -- "$R/tools/micro/lane_read" > "$OUT/calib.log" 2>&1
if [ "$W" = scan ] || [ "$W" = long ] || [ "$W" = config5 ]; then
  timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$OUT/lds" -o pmc -- python "$R/bench.py" --workload "$W" "$@" > "$OUT/lds.log" 2>&1
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$OUT/lds_calib" -o pmc -- "$R/tools/micro/lds_calib" > "$OUT/lds_calib.log" 2>&1
fi
echo PMC_TRAFFIC_OK
