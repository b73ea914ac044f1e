#!/bin/bash
# Round 5: bench rehearsals after the contention-aware push grid (pair_us_by_grid).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$PWD/gpurun_out/r05aa
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_bench.log 2>&1 || { echo "bench tests failed rc=$?"; tail -40 $O/pytest_bench.log; exit 1; }
tail -2 $O/pytest_bench.log
FLEARN_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29571 bench.py --gpus 2 --steps 5 --warmup 2 --config ns --no-weak --no-loopback > $O/rehearsal_ns_g2.json 2> $O/rehearsal_ns_g2.err || { echo rehearsal failed; tail $O/rehearsal_ns_g2.err; exit 1; }
grep "^{" $O/rehearsal_ns_g2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); pc=d['multi_gpu']['push_calibration']; print(pc['grid'], pc['gather_us_by_grid'], pc['pair_us_by_grid'], pc['c_r'])"
