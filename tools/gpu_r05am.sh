#!/bin/bash
# Round 5: the push tests on the default grid of 16 paced blocks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MASTER_ADDR=127.0.0.1
O=$PWD/gpurun_out/r05am
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_copy.py tests/test_gpu_multirank.py tests/test_gpu_parity.py -k "push or order" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_push.log 2>&1 || { echo "push tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" $O/pytest_push.log | tail -20; exit 1; }
tail -1 $O/pytest_push.log
