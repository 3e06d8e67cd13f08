#!/bin/bash
# Wall-clock A/B of libpii.so builds without a profiler attached: bench.py lines per build, ROUNDS
# interleaved rounds.   usage: [WL=workload] [ROUNDS=2] tools/ab_wall.sh TAG LIB...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
for r in $(seq 1 "${ROUNDS:-2}"); do
  i=0
  for L in "$@"; do
    i=$((i+1))
    PII_LIB=$R/$L timeout -k 10 300 python3 "$R/bench.py" --workload "${WL:-scan}" --steps 10 --warmup 3 --no-cpu-baseline > "$O/v${i}_r$r.json" 2> "$O/v${i}_r$r.err" || { echo "FAIL $L"; tail -5 "$O/v${i}_r$r.err"; exit 1; }
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], b['ms_per_step'], b.get('stages_ms'))" "$O/v${i}_r$r.json" "$L r$r"
  done
done
echo WALL_OK
