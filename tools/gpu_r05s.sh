#!/bin/bash
# Round 5: which link-bound store pattern leaves the reduce alone?  fa_push into pinned host memory
# at 32 / 64 blocks vs a plain one-load-one-store copy kernel (probe_copy16) at 32 / 256 / 512
# blocks vs the runtime's blit kernel vs the copy engine (fa_copy_dma, NoCU), beside the NS reduce;
# then the blit and fa_push runs again under a kernel + memory-copy trace, to see whether the two
# streams' kernels really overlap in time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05s
mkdir -p $O
timeout -k 10 300 python3 tools/overlap_probe.py --config ns --grids 0 --copy pushhost32,pushhost64,cphost32,cphost256,cphost512,blithost,dmahost --reps 7 > $O/overlap_host.json 2> $O/overlap_host.err || { echo "probe rc=$?"; tail -20 $O/overlap_host.err; exit 1; }
cat $O/overlap_host.err
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o ov -- python3 tools/overlap_probe.py --config ns --grids 0 --copy blithost,pushhost32,dmahost --reps 3 > $O/overlap_trace.json 2> $O/overlap_trace.err || { echo "trace rc=$?"; tail -20 $O/overlap_trace.err; exit 1; }
find $O/trace -name "*.csv" | head -20 || true
