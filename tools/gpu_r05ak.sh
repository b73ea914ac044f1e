#!/bin/bash
# Round 5: the paced product push kernel — fa_push into pinned host memory beside the NS reduce
# on 4-32 blocks (compare round 5's unpaced numbers, profiles/r05/copy_paths/overlap_push_r05.json),
# then every push test and the bench rehearsals.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MASTER_ADDR=127.0.0.1
O=$PWD/gpurun_out/r05ak
mkdir -p $O
timeout -k 10 300 python3 tools/overlap_probe.py --config ns --grids 0 --copy pushhost4,pushhost8,pushhost16,pushhost32,pushhost64,wr1,wr2,wr4,dmahost --reps 5 > $O/overlap_push_paced.json 2> $O/overlap_push_paced.err || { echo "probe rc=$?"; tail -20 $O/overlap_push_paced.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/overlap_push_paced.json'))
for k, v in d['rows'][0]['with'].items(): print(k, v['copy_alone_gbs'], v['copy_concurrent_gbs'], v['reduce_slowdown'])"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_copy.py tests/test_gpu_multirank.py tests/test_gpu_bench.py -k "push or bench or rehears or order" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_push.log 2>&1 || { echo "push tests failed rc=$?"; grep -E "FAILED|Error|passed|failed" $O/pytest_push.log | tail -20; exit 1; }
tail -1 $O/pytest_push.log
