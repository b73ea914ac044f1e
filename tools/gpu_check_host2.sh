set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/host2
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
for c in c1 c2 c3; do timeout -k 10 300 python3 $R/tools/bench_e2e.py --config $c > $O/e2e_$c.json 2> $O/e2e_$c.err; done
timeout -k 10 300 python3 $R/tools/bench_wire.py --config c1 > $O/wire_c1.json 2> $O/wire_c1.err
timeout -k 10 300 python3 $R/tools/bench_wire.py --config c2 > $O/wire_c2.json 2> $O/wire_c2.err
timeout -k 10 300 python3 $R/tools/bench_wire.py --config c2 --stage > $O/wire_c2_stage.json 2> $O/wire_c2_stage.err
echo done
