#!/bin/bash
# Memory-pipe PMC passes (TA / TD / TCP busy and stall cycles, TCP->TCC request latency) over the
# config-2 bench, one rocprofv3 run per pass.   usage: tools/pmc_mem.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pass$i" -o pmc -- python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pass$i.log" 2>&1
done
echo PMC_MEM_OK
