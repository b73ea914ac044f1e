#!/bin/bash
# Round 5: whole-line f64 stores in the product row-pointer kernel — its tests, the parity suite,
# and the device-upload lines (tools/bench_rows.py) for c3 / ns / c2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05o
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_rows.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|passed|failed" $O/pytest.log | tail -20; exit 1; }
tail -1 $O/pytest.log
for c in c3 ns c2; do
  timeout -k 10 300 python3 tools/bench_rows.py --config $c > $O/rows_$c.json 2> $O/rows_$c.err || { echo "rows $c failed"; tail $O/rows_$c.err; exit 1; }
  cat $O/rows_$c.json
done
