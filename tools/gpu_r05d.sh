#!/bin/bash
# Round 5, fourth GPU pass: exported buckets never freed (a new one each iteration / three reused)
# vs the earlier variants; the copy-engine legs through hipMemcpyDeviceToDeviceNoCU (fa_copy_dma)
# beside the blit-kernel path, under rocprofv3 --memory-copy-trace; the push tests on that library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r05d
mkdir -p $O/ipc $O/dma
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python3 tools/ipc_probe.py --out $O/ipc/$tag "$@" > $O/ipc/$tag.json 2> $O/ipc/$tag.err || { echo "ipc $tag failed rc=$?"; return 1; }
  cat $O/ipc/$tag.json
}
run own_bar_keep_vary --alloc own --after-unmap barrier --free keep --sizes vary &&
run own_none_keep_fixed --alloc own --after-unmap none --free keep --sizes fixed &&
run own_bar_reuse --alloc own --after-unmap barrier --free reuse --sizes fixed &&
run own_bar_keep_w4 --alloc own --after-unmap barrier --free keep --sizes fixed --world 4 &&
run torch_none_del_nb_w4 --alloc torch --after-unmap none --free del --neighbours --world 4 || exit 1
cd /tmp
timeout -k 10 180 rocprofv3 --memory-copy-trace --kernel-trace --stats --output-format csv -d $O/dma/trace -o legs -- \
  python3 $R/tools/probe_dma_legs.py --legs 7 --mib 64 --out $O/dma/legs.json > $O/dma/legs.out 2> $O/dma/legs.err || { echo "dma probe failed"; tail -5 $O/dma/legs.err; exit 1; }
cat $O/dma/legs.json
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread \
  tests/test_gpu_multirank.py::test_sharded_reducer_push_gather tests/test_gpu_multirank.py::test_push_setup_lifecycle \
  > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
