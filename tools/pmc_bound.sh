#!/bin/bash
# What bounds each kernel (VERDICT r4 Next 2 / 4): the wave-cycle split (issue-active VALU / LDS /
# VMEM, issue stalls, parked on s_waitcnt) and the achieved occupancy, one rocprofv3 --pmc run per
# counter group (never combined with tracing), each counter group checked against `rocprofv3 -L`
# first.  Occupancy = 4 * SQ_WAVE_CYCLES (quad-cycles) / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs) waves
# per SIMD, plus SQ_LEVEL_WAVES / SQ_ACCUM_PREV_HIRES when the device lists them.
# usage: tools/pmc_bound.sh OUTDIR [bench args...]      (summary: python tools/pmc_bound.py OUTDIR)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "rocprofv3 -L failed (rc $?)"
have() { grep -qw "$1" "$OUT/counters.txt"; }
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  use=""
  for c in $grp; do
    if have "$c"; then use="$use $c"; else echo "pass $i: $c not listed, dropped"; fi
  done
  [ -z "$use" ] && continue
  echo "pass $i:$use"
  timeout -s KILL 300 rocprofv3 --pmc $use --output-format csv -d "$OUT/pass$i" -o pmc -- python3 "$R/bench.py" "$@" > "$OUT/pass$i.log" 2>&1 || { echo "pass $i FAILED"; tail -5 "$OUT/pass$i.log"; exit 1; }
done
echo BOUND_OK
