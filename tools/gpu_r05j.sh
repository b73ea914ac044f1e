#!/bin/bash
# Round 5: wide windows as several launches (fa_reduce_windows) — parity on every BASELINE shape,
# then a bench line per config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05j
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_props.py tests/test_gpu_copy.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|passed|failed" $O/pytest.log | tail -20; exit 1; }
tail -2 $O/pytest.log
for c in c3 c5 c2 c4 ns; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail $O/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']; print('$c', d['ms_per_step'], r['frac'], r['launches_per_step'], d['verify']['verified'])"
done
