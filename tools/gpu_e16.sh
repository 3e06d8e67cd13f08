#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/e16
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_config5.py tests/test_gpu_long_rows.py tests/test_gpu_window.py tests/test_gpu_fullsize.py tests/test_ner_redaction.py -x -v -m gpu --timeout 300 --timeout-method thread > "$O/t.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$O/t.log"; exit 1; }
bash tools/ab.sh e16/ab exp_libs/libpii_h5.so context-based-pii_amd/libpii.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
WL=config5 bash tools/ab.sh e16/ab5 exp_libs/libpii_h5.so context-based-pii_amd/libpii.so > "$O/ab5.log" 2>&1 || { cat "$O/ab5.log"; exit 1; }
echo E16_OK
