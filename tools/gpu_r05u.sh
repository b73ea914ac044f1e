#!/bin/bash
# Round 5: the copy paths untraced.  probe_dma_legs without a profiler (a leg's rate tells a copy
# engine, ~60 GB/s, from a copy kernel, ~2 TB/s, for device destinations), and the overlap probe
# with a device-to-device copy-engine copy (dmadev) and the runtime's device copy (dma) beside the
# NS reduce.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05u
mkdir -p $O
timeout -k 10 200 python3 tools/probe_dma_legs.py --legs 7 --mib 64 --out $O/legs_untraced.json > $O/legs.out 2> $O/legs.err || { echo "legs rc=$?"; tail -20 $O/legs.err; exit 1; }
timeout -k 10 300 python3 tools/overlap_probe.py --config ns --grids 0 --copy dmadev,dma,blithost,dmahost --reps 7 > $O/overlap_dev.json 2> $O/overlap_dev.err || { echo "probe rc=$?"; tail -20 $O/overlap_dev.err; exit 1; }
grep "^grid" $O/overlap_dev.err
python3 -c "
import json; d=json.load(open('$O/legs_untraced.json'))
for k,v in d.items():
    if isinstance(v,dict): print(k, v['one_leg_gbs'], v.get('legs7_gbs_total'), v.get('legs7_over_one'))"
