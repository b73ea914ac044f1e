# counters of the row-pointer kernel (reduce_kernel_segrows_rm) against the stack
# kernel (reduce_kernel_rowmajor) on the same uploads (tools/rows_pmc.py), one --pmc pass per
# counter group (MI355X_MICROARCH.md slot limits), each under its own time limit.
#   then: python tools/rows_pmc_table.py gpurun_out/$OUT > profiles/r04/rows_pmc/table.md
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-rows_pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "fetch:FETCH_SIZE"
  "write:WRITE_SIZE"
  "utcl1:TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum"
  "utcl1stall:TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum"
  "busy:TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
  "tcp:TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum"
  "tcc:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_MISS_sum"
  "sq:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY"
)
for run in ${RUNS:-ns:clones ns:stack c3:clones}; do
  IFS=: read -r cfg al <<< "$run"
  tag=${cfg}_${al}
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$tag -o $tag -- python3 $R/tools/rows_pmc.py --config $cfg --alloc $al --reps 10 > $O/trace_$tag.json 2> $O/trace_$tag.err
  for p in "${PASSES[@]}"; do
    name=${p%%:*}
    ctrs=${p#*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex reduce_kernel --output-format csv -d $O/${name}_$tag -o $tag -- python3 $R/tools/rows_pmc.py --config $cfg --alloc $al --reps 5 > /dev/null 2> $O/${name}_$tag.err
  done
done
timeout -k 10 300 python3 $R/tools/bench_client_update.py --ab --phases --rounds 4 > $O/client_update_ab2.json 2> $O/client_update_ab2.err
echo done
