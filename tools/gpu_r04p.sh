# Round 4, pass p: loopback pack, interleaved in one process — the Python pool vs native
# threads (all chunks queued / 2 ahead; 16 / 8 threads); zero-copy unpack in all.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04p2}
mkdir -p $O
AB='native_async=0;native_async=1,async_lookahead=0,async_threads=0;native_async=1,async_lookahead=2,async_threads=0;native_async=1,async_lookahead=0,async_threads=8;native_async=1,async_lookahead=2,async_threads=8'
for c in c2 c3; do
  timeout -k 10 400 python3 $R/tools/bench_e2e.py --config $c --rounds 10 --ab "$AB" > $O/ab_${c}.json 2> $O/ab_${c}.err
done
echo done
