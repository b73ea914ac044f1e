#!/bin/bash
# Round 5: refine the window-count rule (tools/probe_slabs.py --windows), two allocations each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05k
mkdir -p $O
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 400 python3 tools/probe_slabs.py --windows "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail $O/$tag.err; return 1; }
  cat $O/$tag.json
}
run ns_mean --op mean --params 25610152 --slabs 1,3,4,6 --allocs 2 &&
run c3_avgm --op avgm --params 25610152 --slabs 3,4,5,6 --allocs 2 &&
run c5_adagrad --op adagrad --slabs 3,5,9 --allocs 2 &&
run c2_mean --op mean --params 11699112 --slabs 2,3,4 --allocs 2 &&
run c4_mean --op mean --clients 1000 --params 11699112 --slabs 1,2,4 --allocs 2 &&
run c5_mean --op mean --slabs 1,3,4,6 --allocs 2
