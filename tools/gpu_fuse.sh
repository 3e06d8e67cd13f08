#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/fuse1
mkdir -p "$O"
PII_DEBUG=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ner_redaction.py tests/test_config5.py tests/test_gpu_long_rows.py -x -v -m gpu --timeout 300 --timeout-method thread > "$O/t.log" 2>&1 || { echo TESTS_FAILED; exit 1; }
bash tools/ab_env.sh fuse1/ab PII_FUSE=1 PII_FUSE=0 > "$O/ab.log" 2>&1 || exit 1
echo FUSE_OK
