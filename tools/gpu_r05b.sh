#!/bin/bash
# Round 5, second GPU pass: (1) the rest of the stale-import diagnosis (tools/ipc_probe.py), (2) the
# new push lifecycle and bench-phase tests, (3) the copy-engine legs' concurrency under
# rocprofv3 --memory-copy-trace, (4) row-pointer kernel counters: the product, the same kernel with
# the row pointers staged in LDS (no per-step scalar loads), and the product reading the stack.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r05b
mkdir -p $O/ipc $O/dma $O/rows_pmc
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python3 tools/ipc_probe.py --out $O/ipc/$tag "$@" > $O/ipc/$tag.json 2> $O/ipc/$tag.err || { echo "ipc $tag failed rc=$?"; return 1; }
  cat $O/ipc/$tag.json
}
run torch_none_empty --alloc torch --after-unmap none --free empty &&
run torch_bar_empty --alloc torch --after-unmap barrier --free empty &&
run own_none_vary --alloc own --after-unmap none &&
run own_bar_vary --alloc own --after-unmap barrier &&
run own_none_fixed --alloc own --after-unmap none --sizes fixed &&
run own_bar_fixed --alloc own --after-unmap barrier --sizes fixed || exit 1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread \
  tests/test_gpu_multirank.py::test_push_setup_lifecycle tests/test_gpu_multirank.py::test_sharded_reducer_push_gather \
  tests/test_gpu_bench.py::test_bench_line_survives_a_stalled_push_setup \
  tests/test_gpu_bench.py::test_bench_keeps_rccl_when_a_push_fails_its_check \
  tests/test_gpu_bench.py::test_bench_push_gather_is_verified > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -5 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
cd /tmp
timeout -k 10 120 rocprofv3 --memory-copy-trace --kernel-trace --stats --output-format csv -d $O/dma/trace -o legs -- \
  python3 $R/tools/probe_dma_legs.py --legs 7 --mib 64 --out $O/dma/legs.json > $O/dma/legs.out 2> $O/dma/legs.err || exit 1
cat $O/dma/legs.json
PASSES=(
  "sq:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY"
  "tcp:TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum"
  "utcl1:TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum"
  "busy:TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
)
for run in ns:clones:product ns:clones:lt ns:stack:product; do
  IFS=: read -r cfg al k <<< "$run"
  tag=${cfg}_${al}_${k}
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rows_pmc/trace_$tag -o $tag -- python3 $R/tools/rows_pmc.py --config $cfg --alloc $al --kernel $k --reps 10 > $O/rows_pmc/trace_$tag.json 2> $O/rows_pmc/trace_$tag.err || exit 1
  for p in "${PASSES[@]}"; do
    name=${p%%:*}
    ctrs=${p#*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex reduce_kernel --output-format csv -d $O/rows_pmc/${name}_$tag -o $tag -- python3 $R/tools/rows_pmc.py --config $cfg --alloc $al --kernel $k --reps 5 > /dev/null 2> $O/rows_pmc/${name}_$tag.err || exit 1
  done
  cat $O/rows_pmc/trace_$tag.json
done
echo r05b-done
