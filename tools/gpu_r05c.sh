#!/bin/bash
# Round 5, third GPU pass: the stale-import fix — exported buckets freed with their addresses kept
# reserved (fa_dev_retire), so no (exporter, address) pair is ever imported twice — checked with
# the probe, then the push tests that drive the product's set-up/teardown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r05c
mkdir -p $O/ipc
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python3 tools/ipc_probe.py --out $O/ipc/$tag "$@" > $O/ipc/$tag.json 2> $O/ipc/$tag.err || { echo "ipc $tag failed rc=$?"; return 1; }
  cat $O/ipc/$tag.json
}
run own_none_retire_fixed --alloc own --after-unmap none --free retire --sizes fixed &&
run own_bar_retire_fixed --alloc own --after-unmap barrier --free retire --sizes fixed &&
run own_bar_retire_vary --alloc own --after-unmap barrier --free retire --sizes vary &&
run own_bar_retire_fixed_w4 --alloc own --after-unmap barrier --free retire --sizes fixed --world 4 || exit 1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread \
  tests/test_gpu_multirank.py::test_push_setup_lifecycle tests/test_gpu_multirank.py::test_sharded_reducer_push_gather \
  > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
