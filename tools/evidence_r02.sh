#!/bin/bash
# round-2 evidence: GPU tests, PMC passes (config 2), kernel stats, config-5 stats + L2 hit rate
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$1
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAIL; tail -30 "$O/gpu_tests.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { echo BENCH_FAIL; exit 1; }
bash "$R/tools/pmc_passes.sh" "gpurun_out/$1/pmc" --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmc.log" 2>&1 || { echo PMC_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c5_prof" -o run -- python3 "$R/bench.py" --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/c5_prof.log" 2>&1 || { echo C5PROF_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$O/c5_l2" -o pmc -- python3 "$R/bench.py" --workload config5 --steps 1 --warmup 0 --no-cpu-baseline > "$O/c5_l2.log" 2>&1 || { echo C5L2_FAIL; exit 1; }
echo EVIDENCE_OK
