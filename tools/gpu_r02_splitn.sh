# Split-N path: its GPU tests, the full GPU suite, c1k bench lines (sequential and --reorder) with
# rocprof kernel stats
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r02_splitn}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 $R/bench.py --config c1k > $O/bench_c1k.json 2> $O/bench_c1k.err
timeout -k 10 300 python3 $R/bench.py --config c1k --reorder > $O/bench_c1k_reorder.json 2> $O/bench_c1k_reorder.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c1k_reorder -o c1k_reorder -- python3 $R/bench.py --config c1k --reorder --no-cpu-baseline > $O/trace_c1k_reorder_bench.json 2> $O/trace_c1k_reorder.err
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c1k_reorder -o c1k_reorder -- python3 $R/bench.py --config c1k --reorder --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2> $O/fetch.err
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c1k_reorder -o c1k_reorder -- python3 $R/bench.py --config c1k --reorder --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2> $O/write.err
echo done
