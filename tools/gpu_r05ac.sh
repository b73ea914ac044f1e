#!/bin/bash
# Round 5: kernel traces of the stripe pipeline (tools/trace_pipeline.py) — one process, a 1-rank
# RCCL group, the NS stack in 4 stripes, RCCL all-gather / kernel push / copy-engine push.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$PWD/gpurun_out/r05ac
mkdir -p $O
for g in rccl push push_dma; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$g -o pipe -- python3 tools/trace_pipeline.py --gather $g --stripes 4 > $O/$g.out 2> $O/$g.err || { echo "$g rc=$?"; tail -20 $O/$g.err; exit 1; }
  f=$(find $O/$g -name "pipe_kernel_trace.csv" | head -1)
  python3 tools/trace_pipeline.py --analyze $f > $O/${g}_analysis.json
  python3 -c "import json; d=json.load(open('$O/${g}_analysis.json')); print('$g', {k: d.get(k) for k in ('reduce_launches','gather_launches','gather_streams','reduce_streams','gather_frac_beside_a_reduce','gather_us_total','reduce_us_total','gather_kernels')})"
done
