#!/bin/bash
# Round 5: bench.py's rehearsals on the one GPU, with the crash-proof held line (a rank dying in
# the push set-up: the RCCL line must still print), and the watchdog's CPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$PWD/gpurun_out/r05w
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_bench.py tests/test_bench_watchdog.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_bench.log 2>&1 || { echo "bench tests failed rc=$?"; tail -40 $O/pytest_bench.log; exit 1; }
tail -3 $O/pytest_bench.log
