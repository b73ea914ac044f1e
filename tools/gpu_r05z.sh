#!/bin/bash
# Round 5: CU-masked streams against the push kernel's cost to the reduce.  The NS reduce beside
# fa_push into pinned host memory (a link-bound store kernel), a write-only stream and the copy
# engine: unmasked; the copy stream fenced onto 8 / 16 CUs; and the reduce fenced onto the rest.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05z
mkdir -p $O
K="pushhost8,pushhost16,pushhost32,wr2"
timeout -k 10 200 python3 tools/overlap_probe.py --config ns --grids 0 --copy $K --reps 5 > $O/unmasked.json 2> $O/unmasked.err || { echo "unmasked rc=$?"; tail -20 $O/unmasked.err; exit 1; }
grep "^grid" $O/unmasked.err
for cus in 8 16; do
  timeout -k 10 200 python3 tools/overlap_probe.py --config ns --grids 0 --copy $K --reps 5 --push-cus $cus > $O/push${cus}.json 2> $O/push${cus}.err || { echo "push$cus rc=$?"; tail -20 $O/push${cus}.err; exit 1; }
  echo "push on $cus CUs, reduce unmasked"; grep "^grid" $O/push${cus}.err
  timeout -k 10 200 python3 tools/overlap_probe.py --config ns --grids 0,256,240 --copy $K --reps 5 --push-cus $cus --mask-reduce > $O/push${cus}_disjoint.json 2> $O/push${cus}_disjoint.err || { echo "disjoint$cus rc=$?"; tail -20 $O/push${cus}_disjoint.err; exit 1; }
  echo "push on $cus CUs, reduce on the others"; grep "^grid" $O/push${cus}_disjoint.err
done
