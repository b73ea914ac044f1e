#!/bin/bash
# Round 5: the stripe pipeline with the product's high-priority side streams (and RCCL's stream
# from the high-priority pool, as bench.py now asks): queues and overlap traced; then the whole
# GPU suite on this tree (the host paths' copy streams changed too).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$PWD/gpurun_out/r05ae
mkdir -p $O
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python3 tools/trace_pipeline.py "$@" --steps 20 > $O/$tag.time.json 2> $O/$tag.time.err || { echo "$tag time rc=$?"; tail -5 $O/$tag.time.err; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o pipe -- python3 tools/trace_pipeline.py "$@" --steps 5 > $O/$tag.out 2> $O/$tag.err || { echo "$tag trace rc=$?"; tail -5 $O/$tag.err; exit 1; }
  f=$(find $O/$tag -name "pipe_kernel_trace.csv" | head -1)
  python3 tools/trace_pipeline.py --analyze $f > $O/${tag}_analysis.json
  python3 -c "import json; t=json.loads(open('$O/$tag.time.json').read().strip().splitlines()[-1]); d=json.load(open('$O/${tag}_analysis.json')); print('$tag', t['ms_per_step'], 'ms', 'q', d['reduce_queues'], d['gather_queues'], 'beside', d['gather_frac_beside_a_reduce'])"
}
run push --gather push
run push_normal --gather push --pusher-stream normal
run dma --gather push_dma
run rccl_high --gather rccl --nccl-high
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "suite failed rc=$?"; grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -20; exit 1; }
tail -1 $O/pytest_gpu.log
