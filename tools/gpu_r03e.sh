# Round 3: GPU suite on the double-buffered fused state (ABI 6 v_out) + bench lines of the fused configs.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03e}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 180 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
for c in c3 c5 c3 c5 ns; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --steps 30 >> $O/bench_$c.jsonl 2>> $O/bench.err
done
echo done
