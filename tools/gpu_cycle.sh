#!/bin/bash
# one GPU iteration: parity tests, bench, kernel-trace profile.  usage: tools/gpu_cycle.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$TAG.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo "PROF FAILED"; exit 1; }
echo CYCLE_OK
