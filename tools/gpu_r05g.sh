#!/bin/bash
# Round 5: column-slabbed stacks for C5 (tools/probe_slabs.py), fused Adagrad and plain mean.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05g
mkdir -p $O
timeout -k 10 400 python3 tools/probe_slabs.py --op adagrad --slabs 1,2,3,4,8 --allocs 3 > $O/slabs_c5_adagrad.json 2> $O/slabs_c5_adagrad.err || { echo slabs adagrad failed; tail $O/slabs_c5_adagrad.err; exit 1; }
cat $O/slabs_c5_adagrad.json
timeout -k 10 400 python3 tools/probe_slabs.py --op mean --slabs 1,2,4 --allocs 2 > $O/slabs_c5_mean.json 2> $O/slabs_c5_mean.err || { echo slabs mean failed; tail $O/slabs_c5_mean.err; exit 1; }
cat $O/slabs_c5_mean.json
timeout -k 10 400 python3 tools/probe_slabs.py --op mean --params 25610152 --slabs 1,2,4 --allocs 2 > $O/slabs_ns_mean.json 2> $O/slabs_ns_mean.err || { echo slabs ns failed; tail $O/slabs_ns_mean.err; exit 1; }
cat $O/slabs_ns_mean.json
