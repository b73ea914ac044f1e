#!/bin/bash
# Round 5: 4-rank gloo rehearsal of bench.py --gpus 4 (four processes share the box's GPU): the
# phased run with the push gathers among 4 processes, and the stalled-push rehearsal at world 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 FLEARN_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1
O=$PWD/gpurun_out/r05m
mkdir -p $O
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr=127.0.0.1 --master-port=29541 bench.py --gpus 4 --steps 5 --warmup 2 --config c5 > $O/rehearsal_c5_g4.json 2> $O/rehearsal_c5_g4.err || { echo "rehearsal c5 failed"; tail -20 $O/rehearsal_c5_g4.err; exit 1; }
echo c5-ok
FLEARN_BENCH_INJECT=push_stall timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr=127.0.0.1 --master-port=29542 bench.py --gpus 4 --steps 3 --warmup 1 --config c2 --no-weak --no-loopback --push-budget-s 30 > $O/stall_c2_g4.json 2> $O/stall_c2_g4.err || { echo "stall rehearsal failed rc=$?"; tail -20 $O/stall_c2_g4.err; exit 1; }
echo stall-ok
