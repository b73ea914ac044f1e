set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wire2
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "wire" > $O/pytest_wire.log 2>&1
timeout -k 10 300 python3 $R/tools/bench_wire.py --config c2 > $O/wire_c2.json 2> $O/wire_c2.err
timeout -k 10 300 python3 $R/tools/bench_wire.py --config c2 --stage > $O/wire_c2_stage.json 2> $O/wire_c2_stage.err
timeout -k 10 400 python3 $R/tools/bench_wire.py --config c3 --stage > $O/wire_c3_stage.json 2> $O/wire_c3_stage.err
timeout -k 10 300 python3 $R/tools/bench_wire.py --config c1 > $O/wire_c1.json 2> $O/wire_c1.err
echo done
