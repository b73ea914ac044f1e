# What the driver runs at round end, plus the codec / loopback lines: GPU parity suite, smoke(),
# the default bench line, wire and e2e C1.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-suite}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 180 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err
echo done
