#!/bin/bash
# Round 5: the fused C5 kernel runs 1.5% faster as 3 launches over column windows of the same
# stack (r05h); which shapes / ops / window counts gain (tools/probe_slabs.py --windows)?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05i
mkdir -p $O
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 400 python3 tools/probe_slabs.py --windows "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail $O/$tag.err; return 1; }
  cat $O/$tag.json
}
run c5_adagrad --op adagrad --slabs 1,2,3,4,6 --allocs 2 &&
run c5_avgm --op avgm --slabs 1,3 --allocs 2 &&
run c5_mean --op mean --slabs 1,2,3 --allocs 2 &&
run c3_avgm --op avgm --params 25610152 --slabs 1,2,3 --allocs 2 &&
run ns_mean --op mean --params 25610152 --slabs 1,2 --allocs 2 &&
run c2_mean --op mean --params 11699112 --slabs 1,2 --allocs 2 &&
run c4_mean --op mean --clients 1000 --params 11699112 --slabs 1,2,3 --allocs 2
