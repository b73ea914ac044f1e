# The GPU parity suite + smoke() on this tree (what the driver runs at round end).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-suite}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 180 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo done
