#!/bin/bash
# Round 5: does the profiler change the copy path?  The overlap probe's blit / copy-engine copies
# into pinned host memory under a kernel trace only (no memory-copy trace), and fa_push into
# pinned host memory at 4-32 blocks untraced.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05t
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ktrace -o ov -- python3 tools/overlap_probe.py --config ns --grids 0 --copy blithost,dmahost --reps 3 > $O/overlap_ktrace.json 2> $O/overlap_ktrace.err || { echo "ktrace rc=$?"; tail -20 $O/overlap_ktrace.err; exit 1; }
grep "^grid" $O/overlap_ktrace.err
timeout -k 10 300 python3 tools/overlap_probe.py --config ns --grids 0 --copy pushhost4,pushhost8,pushhost16,pushhost32,blithost --reps 7 > $O/overlap_push.json 2> $O/overlap_push.err || { echo "probe rc=$?"; tail -20 $O/overlap_push.err; exit 1; }
grep "^grid" $O/overlap_push.err
