#!/bin/bash
# Round 5: the product's streams after the fix (kernel push on a high-priority stream, copy-engine
# push on normal ones): the ordering probe with the test's sequence 6 times, the pipeline traces,
# then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MASTER_ADDR=127.0.0.1
O=$PWD/gpurun_out/r05ag
mkdir -p $O
timeout -k 10 600 python3 tests/push_order_probe.py --world 8 --steps 3 --reps 6 --priorities product --out $O/push_order_product_w8.json > $O/probe.out 2> $O/probe.err || { echo "probe rc=$?"; tail -30 $O/probe.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/push_order_product_w8.json')); [print(k, v['runs'], v['steps'], v['bad_steps'], v['examples'][:2]) for k, v in d['summary'].items()]"
for g in push push_dma rccl; do
  timeout -k 10 120 python3 tools/trace_pipeline.py --gather $g --steps 20 > $O/$g.time.json 2> $O/$g.time.err || { echo "$g time rc=$?"; tail -5 $O/$g.time.err; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$g -o pipe -- python3 tools/trace_pipeline.py --gather $g --steps 5 > $O/$g.out 2> $O/$g.err || { echo "$g trace rc=$?"; tail -5 $O/$g.err; exit 1; }
  f=$(find $O/$g -name "pipe_kernel_trace.csv" | head -1)
  python3 tools/trace_pipeline.py --analyze $f > $O/${g}_analysis.json
  python3 -c "import json; t=json.loads(open('$O/$g.time.json').read().strip().splitlines()[-1]); d=json.load(open('$O/${g}_analysis.json')); print('$g', t['ms_per_step'], 'ms', 'q', d['reduce_queues'], d['gather_queues'], 'beside', d['gather_frac_beside_a_reduce'])"
done
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "suite failed rc=$?"; grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -20; exit 1; }
tail -1 $O/pytest_gpu.log
