#!/bin/bash
# Round 5: C5 fused Adagrad — column slabs (own pitch) vs column windows of the one stack (same
# pitch, S launches), same allocations' worth of trials (tools/probe_slabs.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05h
mkdir -p $O
timeout -k 10 500 python3 tools/probe_slabs.py --op adagrad --slabs 1,2,3 --allocs 3 --windows > $O/windows_c5_adagrad.json 2> $O/windows_c5_adagrad.err || { echo windows failed; tail $O/windows_c5_adagrad.err; exit 1; }
cat $O/windows_c5_adagrad.json
timeout -k 10 500 python3 tools/probe_slabs.py --op adagrad --slabs 1,3 --allocs 3 > $O/slabs_c5_adagrad.json 2> $O/slabs_c5_adagrad.err || { echo slabs failed; tail $O/slabs_c5_adagrad.err; exit 1; }
cat $O/slabs_c5_adagrad.json
