#!/bin/bash
# round-3: the service NOMEM test, smoke(), the config-2 bench line, its rocprofv3 kernel-trace summary,
# the config-2 PMC passes (HBM bytes + LDS-array cycles)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
T=${1:-r03d}
O=$R/gpurun_out/$T
mkdir -p "$O"
stop() { echo "STOPPED at $1 (rc $2)"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_service.py -x -v -m gpu -k nomem --timeout 250 --timeout-method thread > "$O/t_nomem.log" 2>&1 || stop nomem $?
timeout -k 10 200 python __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || stop smoke $?
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || stop bench $?
bash "$R/tools/pmc_traffic.sh" "gpurun_out/$T/pmc_scan" scan --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc_scan.log" 2>&1 || stop "pmc scan" $?
python "$R/tools/pmc_traffic.py" "gpurun_out/$T/pmc_scan" --workload scan --write > "$O/traffic_scan.json" || stop "pmc summary" $?
cp "$R/profiles/traffic.json" "$O/traffic.json"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/bench_pmc.json" 2> "$O/bench_pmc.err" || stop bench2 $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/prof.log" 2>&1 || stop prof $?
echo R03D_OK
