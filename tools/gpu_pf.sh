#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/pf1
mkdir -p "$O"
PII_LIB=$R/exp_libs/libpii_pf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_config5.py tests/test_gpu_long_rows.py tests/test_gpu_window.py tests/test_context_variants.py -x -v -m gpu --timeout 300 --timeout-method thread > "$O/t.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$O/t.log"; exit 1; }
bash tools/ab.sh pf1/ab context-based-pii_amd/libpii.so exp_libs/libpii_pf.so context-based-pii_amd/libpii.so exp_libs/libpii_pf.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
echo PF_OK
