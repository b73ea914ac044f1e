#!/bin/bash
# Round 5: a paced push stand-in (each wave drains its stores before its next loads) into pinned
# host memory beside the NS reduce, against fa_push on 4 / 8 / 16 blocks and the copy engine.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05aj
mkdir -p $O
timeout -k 10 400 python3 tools/overlap_probe.py --config ns --grids 0 --copy pushhost4,pushhost8,pushhost16,paced1x16,paced1x32,paced1x64,paced2x16,paced2x32,paced4x8,paced4x16,paced4x32,paced8x8,paced8x16,dmahost --reps 5 > $O/paced.json 2> $O/paced.err || { echo "probe rc=$?"; tail -20 $O/paced.err; exit 1; }
grep "^grid" $O/paced.err
python3 -c "
import json; d=json.load(open('$O/paced.json'))
for k, v in d['rows'][0]['with'].items(): print(k, v['copy_alone_gbs'], v['copy_concurrent_gbs'], v['reduce_slowdown'])"
