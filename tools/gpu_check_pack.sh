set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pack
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
for c in c1 c2 c3; do timeout -k 10 300 python3 $R/tools/bench_e2e.py --config $c > $O/e2e_$c.json 2> $O/e2e_$c.err; done
timeout -k 10 200 python3 $R/tools/prof_host_c1.py > $O/prof_c1.txt 2>&1
echo done
