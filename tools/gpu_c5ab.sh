# Same-box A/B: bench.py c5/c3 lines vs the tuner's in-process product geometry (TUNE_SET=epib4).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c5ab
mkdir -p $O
cd $R
timeout -k 10 200 python3 bench.py --config c5 --no-cpu-baseline --steps 30 > $O/bench_c5_a.json 2> $O/bench_c5_a.err
TUNE_SET=inplace timeout -k 10 200 tools/tune_reduce 100 86567680 3 adagrad > $O/tune_c5.txt 2>&1 || true
timeout -k 10 200 python3 bench.py --config c5 --no-cpu-baseline --steps 30 > $O/bench_c5_b.json 2> $O/bench_c5_b.err
timeout -k 10 200 python3 bench.py --config c3 --no-cpu-baseline --steps 30 > $O/bench_c3.json 2> $O/bench_c3.err
TUNE_SET=inplace timeout -k 10 200 tools/tune_reduce 100 25610176 3 avgm > $O/tune_c3.txt 2>&1 || true
timeout -k 10 200 python3 bench.py --config c5 --no-cpu-baseline --steps 30 > $O/bench_c5_c.json 2> $O/bench_c5_c.err
TUNE_SET=inplace timeout -k 10 200 tools/tune_reduce 100 86567680 3 adagrad > $O/tune_c5_b.txt 2>&1 || true
echo done
