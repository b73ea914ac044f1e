# Round-3 first pass: multi-rank product paths on one GPU (gloo ranks), the GPU suite, the
# default bench line, an emulated 8-GPU per-rank run, and the dynamic-tail sweep.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03a}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/multirank.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider --ignore tests/test_gpu_multirank.py > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_ns.json 2> $O/bench_ns.err
timeout -k 10 300 python bench.py --emulate-world 8 --steps 20 --warmup 3 > $O/bench_emu8.json 2> $O/bench_emu8.err
for s in 100:25610176:avgm 100:25610176:mean 100:86567680:adagrad; do
  IFS=: read -r n p op <<< "$s"
  TUNE_SET=tail timeout -k 10 200 tools/tune_reduce $n $p 3 $op > $O/tail_n${n}_p${p}_$op.txt 2>&1
done
echo done
