#!/bin/bash
# Copy one evidence set (tools/evidence_pmc.sh + tools/evidence_bench.sh output under gpurun_out/TAG)
# into profiles/DEST: bench lines, GPU test log, smoke, rocprofv3 kernel stats, per-kernel PMC traffic
# and the bound / occupancy tables.   usage: tools/collect_evidence.sh TAG DEST   (runs in the container)
set -e -o pipefail
TAG=$1
DEST=profiles/$2
S=gpurun_out/$TAG
mkdir -p "$DEST"
cp "$S"/bench_*.json "$DEST"/
cp "$S/gpu_tests.log" "$DEST/gpu_tests.txt"
cp "$S/smoke.log" "$DEST/smoke.txt"
for W in scan config5 window; do
  cp "$S/prof_$W/run_kernel_stats.csv" "$DEST/kernel_stats_$W.csv"
  python3 tools/pmc_bound.py "$S/bound_$W" --json "$DEST/bound_$W.json" > "$DEST/bound_$W.txt"
done
for W in scan config5 window long window_config5; do
  python3 tools/pmc_traffic.py "$S/traffic_$W" --workload "$W" > "$DEST/traffic_$W.json"
done
echo "collected $S -> $DEST"
