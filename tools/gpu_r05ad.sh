#!/bin/bash
# Round 5: which hardware queue does the gather's stream land on?  The stripe pipeline (4 stripes,
# NS, 1-rank RCCL group) timed untraced, then kernel-traced, for the gather's stream as created
# by the product (default), at high priority, with a CU mask of every CU, and for RCCL with its
# stream from the high-priority pool; and the default with GPU_MAX_HW_QUEUES=8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$PWD/gpurun_out/r05ad
mkdir -p $O
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python3 tools/trace_pipeline.py "$@" --steps 20 > $O/$tag.time.json 2> $O/$tag.time.err || { echo "$tag time rc=$?"; tail -5 $O/$tag.time.err; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o pipe -- python3 tools/trace_pipeline.py "$@" --steps 5 > $O/$tag.out 2> $O/$tag.err || { echo "$tag trace rc=$?"; tail -5 $O/$tag.err; exit 1; }
  f=$(find $O/$tag -name "pipe_kernel_trace.csv" | head -1)
  python3 tools/trace_pipeline.py --analyze $f > $O/${tag}_analysis.json
  python3 -c "import json; t=json.loads(open('$O/$tag.time.json').read().strip().splitlines()[-1]); d=json.load(open('$O/${tag}_analysis.json')); print('$tag', t['ms_per_step'], 'ms', 'q', d['reduce_queues'], d['gather_queues'], 'beside', d['gather_frac_beside_a_reduce'])"
}
run serial_push --gather push --stripes 1
run rccl --gather rccl
run rccl_high --gather rccl --nccl-high
run push --gather push
run push_high --gather push --pusher-stream high
run push_cumask --gather push --pusher-stream cumask
run dma --gather push_dma
run dma_high --gather push_dma --pusher-stream high
GPU_MAX_HW_QUEUES=8 run push_q8 --gather push
