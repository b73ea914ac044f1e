# Round 4, first pass: GPU suite (incl. the bench self-check / loopback rehearsals and the
# all-or-nothing client update), smoke, default bench line, client update phases.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 180 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python3 $R/tools/bench_client_update.py --phases --rounds 6 > $O/client_update.json 2> $O/client_update.err
timeout -k 10 300 python3 $R/tools/bench_client_update.py --ab --rounds 4 > $O/client_update_ab.json 2> $O/client_update_ab.err
timeout -k 10 300 python3 $R/tools/overlap_probe.py > $O/overlap.json 2> $O/overlap.err
echo done
