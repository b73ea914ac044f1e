# parity suite + e2e + bench lines (no profiler), one GPU
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check
mkdir -p $O
timeout -k 10 600 python -m pytest $R/tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
for c in c1 c2 c3; do timeout -k 10 300 python $R/tools/bench_e2e.py --config $c > $O/e2e_$c.json 2> $O/e2e_$c.err; done
for c in c2 c3 c4 c5; do timeout -k 10 300 python $R/bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err; done
