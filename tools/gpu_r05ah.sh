#!/bin/bash
# Round 5 closing evidence on the final tree (kernel push on its own hardware queue): smoke(), the
# default bench line, a 2-rank NS rehearsal and an 8-rank C2 rehearsal with every phase.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r05ah
mkdir -p $O
timeout -k 10 180 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_ns.json 2> $O/bench_ns.err || { echo bench failed; tail $O/bench_ns.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_ns.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['verify']['verified'])"
export FLEARN_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29581 bench.py --gpus 2 --steps 5 --warmup 2 --config ns > $O/rehearsal_ns_g2.json 2> $O/rehearsal_ns_g2.err || { echo rehearsal2 failed; tail $O/rehearsal_ns_g2.err; exit 1; }
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29582 bench.py --gpus 8 --steps 5 --warmup 2 --config c2 > $O/rehearsal_c2_g8.json 2> $O/rehearsal_c2_g8.err || { echo rehearsal8 failed; tail -30 $O/rehearsal_c2_g8.err; exit 1; }
for f in rehearsal_ns_g2 rehearsal_c2_g8; do
  python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); mg=d['multi_gpu']; print('$f', d['value'], d['ms_per_step'], mg['gather'], mg['phases']['push']['status'], d['verify']['verified'], d.get('weak',{}).get('gather'), d.get('loopback_multi_gpu',{}).get('verified'), mg.get('push_calibration',{}).get('grid'))"
done
