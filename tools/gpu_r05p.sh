#!/bin/bash
# Round 5: run-to-run spread of the default line (NS), eight fresh processes (placement differs per
# process: DESIGN.md section 4 finding 25).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/r05p
mkdir -p $O
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/ns_$i.json 2> $O/ns_$i.err || { echo "run $i failed"; tail $O/ns_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ns_$i.json')); print($i, d['ms_per_step'], d['roofline']['frac'], d['verify']['verified'])"
done
