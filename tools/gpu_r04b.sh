# Round 4, pass b: rocprofv3 counter list; row-pointer vs stack kernel times (clones / stack
# allocations, plain mean and fused AVGM); overlap diagnostics (ALU-only and L2-resident
# stand-ins); the client update's A/B with per-call traces.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04b}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || echo "list rc=$?" >> $O/rocprof_counters.txt
cd $R
for cfg in ns c3; do
  for al in clones stack; do
    timeout -k 10 200 python3 $R/tools/rows_pmc.py --config $cfg --alloc $al --reps 15 > $O/rows_${cfg}_${al}.json 2> $O/rows_${cfg}_${al}.err
  done
done
timeout -k 10 300 python3 $R/tools/overlap_probe.py --grids 0 --copy spin16,spin64,l2copy16,l2copy64,16,8 > $O/overlap_diag.json 2> $O/overlap_diag.err
timeout -k 10 300 python3 $R/tools/bench_client_update.py --ab --phases --rounds 4 > $O/client_update_ab.json 2> $O/client_update_ab.err
echo done
