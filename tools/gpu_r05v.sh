#!/bin/bash
# Round 5: the push contention probe again (round 4's set, profiles/r04/overlap/overlap_push.json):
# fa_push into pinned host memory on 4-256 blocks, write-only streams, and the copy engine into
# pinned host memory, beside the NS reduce, untraced.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05v
mkdir -p $O
timeout -k 10 400 python3 tools/overlap_probe.py --config ns --grids 0 --copy pushhost4,pushhost8,pushhost16,pushhost32,pushhost64,pushhost256,wr1,wr2,wr4,dmahost,dmadev --reps 7 > $O/overlap_push_r05.json 2> $O/overlap_push_r05.err || { echo "probe rc=$?"; tail -20 $O/overlap_push_r05.err; exit 1; }
grep "^grid" $O/overlap_push_r05.err
rocm-smi --showbus --showtopo > $O/topo.txt 2>&1 || true
