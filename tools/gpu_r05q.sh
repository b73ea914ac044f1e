#!/bin/bash
# Round 5: 8-rank gloo rehearsal of bench.py --gpus 8 on the one GPU (eight processes), C2: the
# phased run with both push forms among eight processes (MAX_PUSH_RANKS), weak job, loopback.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 FLEARN_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1
O=$PWD/gpurun_out/r05q
mkdir -p $O
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29551 bench.py --gpus 8 --steps 5 --warmup 2 --config c2 > $O/rehearsal_c2_g8.json 2> $O/rehearsal_c2_g8.err || { echo "rehearsal failed rc=$?"; tail -30 $O/rehearsal_c2_g8.err; exit 1; }
grep "^{" $O/rehearsal_c2_g8.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); mg=d['multi_gpu']; print(d['value'], d['ms_per_step'], mg['gather'], json.dumps(mg['phases'])[:400], d['verify']['verified'], d.get('weak',{}).get('gather'), d['loopback_multi_gpu']['verified'])"
timeout -k 10 400 python3 -u -m pytest "tests/test_gpu_multirank.py::test_sharded_reducer_push_gather[8]" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_push_w8.log 2>&1 || { echo "push w8 failed rc=$?"; tail -30 $O/pytest_push_w8.log; exit 1; }
tail -1 $O/pytest_push_w8.log
