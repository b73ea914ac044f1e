# Round 4, pass o: loopback host path — uploads packed by native threads in growing row chunks
# (AsyncPack) and results stored into fresh pinned buffers by fa_copy, vs the round-3 path
# (Python pool, ~8 equal chunks; copy-engine D2H + host copy); GPU suite first.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04o}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
for i in 1 2; do
  for c in c2 c3; do
    timeout -k 10 300 python3 $R/tools/bench_e2e.py --config $c --rounds 8 > $O/e2e_${c}_new_$i.json 2> $O/e2e_${c}_new_$i.err
    timeout -k 10 300 python3 $R/tools/bench_e2e.py --config $c --rounds 8 --native-pack 0 --zero-copy-out 0 > $O/e2e_${c}_old_$i.json 2> $O/e2e_${c}_old_$i.err
    timeout -k 10 300 python3 $R/tools/bench_e2e.py --config $c --rounds 8 --native-pack 1 --zero-copy-out 0 > $O/e2e_${c}_pack_$i.json 2> $O/e2e_${c}_pack_$i.err
  done
done
timeout -k 10 300 python3 $R/tools/bench_e2e.py --config c1 > $O/e2e_c1.json 2> $O/e2e_c1.err
echo done
