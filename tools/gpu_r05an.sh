#!/bin/bash
# Round 5 closing suite on the final tree (paced push kernel, default grid 16; profile archives not uploaded): the whole GPU suite, smoke(),
# default bench line, and a 2-rank bench rehearsal line with the push phase.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r05an
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "suite failed rc=$?"; grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -20; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 180 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_ns.json 2> $O/bench_ns.err || { echo bench failed; tail $O/bench_ns.err; exit 1; }
cat $O/bench_ns.json
FLEARN_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 5 --warmup 2 --config ns > $O/rehearsal_ns_g2.json 2> $O/rehearsal_ns_g2.err || { echo rehearsal failed; tail $O/rehearsal_ns_g2.err; exit 1; }
echo rehearsal-ok


