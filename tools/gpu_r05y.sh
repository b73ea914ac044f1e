#!/bin/bash
# Round 5: the 8-rank split of C4 (1000 x ResNet-18) and C5 (fused Adagrad, 100 x ViT-B/16) at FULL
# size, eight processes sharing the one GPU over gloo, both push forms calibrated and trialled:
# every line bit-checks its reassembled model (and C5's optimizer state) on >= 64 boundary windows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 FLEARN_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1
O=$PWD/gpurun_out/r05y
mkdir -p $O
for cfg in c4 c5; do
  timeout -k 10 540 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29561 bench.py --gpus 8 --steps 3 --warmup 1 --config $cfg --no-weak --no-loopback > $O/rehearsal_${cfg}_g8.json 2> $O/rehearsal_${cfg}_g8.err || { echo "$cfg rehearsal failed rc=$?"; tail -30 $O/rehearsal_${cfg}_g8.err; exit 1; }
  grep "^{" $O/rehearsal_${cfg}_g8.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); mg=d['multi_gpu']; v=d['verify']; print('$cfg', d['value'], d['ms_per_step'], mg['gather'], mg['phases']['push']['status'], v['verified'], v['windows'], v['state_windows'], v['ranks_checked'])"
done
