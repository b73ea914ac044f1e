# Round 4, pass f: client-side update transfer modes (zero-copy kernel / DMA in+out / DMA in +
# zero-copy out), per-chunk phases each, and the chunk sizes of the zero-copy kernel mode.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04f}
mkdir -p $O
for t in kernel dma_in dma kernel; do
  timeout -k 10 300 python3 $R/tools/bench_client_update.py --phases --rounds 6 --transfer $t > $O/cu_$t.json 2> $O/cu_$t.err
done
for c in 16 64; do
  timeout -k 10 300 python3 $R/tools/bench_client_update.py --phases --rounds 6 --transfer kernel --chunk-mb $c > $O/cu_kernel_c$c.json 2> $O/cu_kernel_c$c.err
done
echo done
