# Round 4, pass l: PCIe probe (zero-copy vs copy engines, concurrent directions) and the client
# update's transfer modes side by side.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04l}
mkdir -p $O
for i in 1 2; do
  for t in kernel dma_in; do
    timeout -k 10 300 python3 $R/tools/bench_client_update.py --rounds 12 --phases --transfer $t > $O/cu_${t}_$i.json 2> $O/cu_${t}_$i.err
  done
done
echo done
