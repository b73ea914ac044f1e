#!/bin/bash
# Round 5: the push gather's ordering with the pusher's streams at normal vs high priority
# (tests/push_order_probe.py: 8 processes on the one GPU, the test's sequence (mean, in-place Adagrad, explicit registrations) 6 times, four
# stripe plans, both push forms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MASTER_ADDR=127.0.0.1
O=$PWD/gpurun_out/r05af
mkdir -p $O
timeout -k 10 600 python3 tests/push_order_probe.py --world 8 --steps 3 --reps 6 --out $O/push_order_w8.json > $O/probe.out 2> $O/probe.err || { echo "probe rc=$?"; tail -30 $O/probe.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/push_order_w8.json')); [print(k, v['runs'], v['steps'], v['bad_steps'], v['examples'][:2]) for k, v in d['summary'].items()]"
