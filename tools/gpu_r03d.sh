# Round 3 (session 2): the driver's round-end steps on this tree (GPU suite, smoke, default bench)
# + the narrow-window L2-prefetch sweep (TUNE_SET=pf).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03d}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 180 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
SET=pf bash tools/gpu_tune_reduce.sh && TUNE_FLUSH=1 SET=pf OUTSET=pf_flush bash tools/gpu_tune_reduce.sh
echo done
