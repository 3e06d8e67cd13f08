#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/mr1
mkdir -p "$O"
PII_LIB=$R/exp_libs/libpii_mr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_config5.py tests/test_gpu_long_rows.py tests/test_gpu_window.py tests/test_context_variants.py tests/test_gpu_fullsize.py -x -v -m gpu --timeout 300 --timeout-method thread > "$O/t.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$O/t.log"; exit 1; }
bash tools/ab.sh mr1/ab exp_libs/libpii_h4.so exp_libs/libpii_mr.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
WL=window bash tools/ab.sh mr1/abw exp_libs/libpii_h4.so exp_libs/libpii_mr.so > "$O/abw.log" 2>&1 || { cat "$O/abw.log"; exit 1; }
echo MR_OK
