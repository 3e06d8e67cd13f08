#!/bin/bash
# window-step A/B: kernel stats of the window workload for the HEAD build, the in-tree build and its
# env variants, then the window GPU tests (default and config-5 rules).
# usage: tools/r6_win.sh TAG [extra ab specs...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
T=$1; shift
WL=window bash "$R/tools/ab_spec.sh" "$T" exp_libs/head.so - "$@" || exit 1
cd "$R" && timeout -k 10 600 python -u -m pytest -x -v -m gpu tests/test_gpu_window.py tests/test_config5.py "tests/test_gpu_fullsize.py::test_config3_window_rescan_100k_conversations_vs_oracle" --timeout 300 --timeout-method thread > "gpurun_out/$T/tests.log" 2>&1 || { echo TESTS FAILED; tail -30 "gpurun_out/$T/tests.log"; exit 1; }
tail -2 "gpurun_out/$T/tests.log"
echo WIN_OK
