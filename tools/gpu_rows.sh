# Row-pointer (device-upload) path: its GPU tests, bench_rows for c2 / ns / c3, and a
# rocprofv3 kernel trace of the server() loop (no per-key copy kernels expected).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-rows}
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_rows.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_rows.log 2>&1
for c in c2 ns c3; do
  timeout -k 10 300 python3 $R/tools/bench_rows.py --config $c > $O/rows_$c.json 2> $O/rows_$c.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_rows_c2 -o c2 -- python3 $R/tools/bench_rows.py --config c2 --steps 5 > $O/trace_rows_c2.json 2> $O/trace_rows_c2.err
echo done
