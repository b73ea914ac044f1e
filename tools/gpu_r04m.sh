# Round 4, pass m: where the client update's copy-engine-in mode loses time (kernel + copy trace).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04m}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/dma_in -o run -- python3 $R/tools/bench_client_update.py --rounds 4 --ref-rounds 1 --phases --transfer dma_in > $O/cu_dma_in.json 2> $O/cu_dma_in.err
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/kernel -o run -- python3 $R/tools/bench_client_update.py --rounds 4 --ref-rounds 1 --phases --transfer kernel > $O/cu_kernel.json 2> $O/cu_kernel.err
echo done
