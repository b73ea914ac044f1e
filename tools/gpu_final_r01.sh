set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 180 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python3 $R/tools/bench_wire.py --config c1 > $O/wire_c1.json 2> $O/wire_c1.err
timeout -k 10 300 python3 $R/tools/bench_e2e.py --config c1 > $O/e2e_c1.json 2> $O/e2e_c1.err
echo done
