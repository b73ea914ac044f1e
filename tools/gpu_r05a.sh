#!/bin/bash
# Round 5, first GPU pass: the push gather's stale-import diagnosis (tools/ipc_probe.py, seven
# variants of the export -> map -> unmap -> free -> re-export sequence) and the copy-engine legs'
# concurrency (tools/probe_dma_legs.py under rocprofv3 --memory-copy-trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05a
mkdir -p $O/ipc $O/dma
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python3 tools/ipc_probe.py --out $O/ipc/$tag "$@" > $O/ipc/$tag.json 2> $O/ipc/$tag.err || { echo "ipc $tag failed rc=$?"; return 1; }
  cat $O/ipc/$tag.json
}
run torch_none_del_nb --alloc torch --after-unmap none --free del --neighbours &&
run torch_none_empty --alloc torch --after-unmap none --free empty &&
run torch_bar_empty --alloc torch --after-unmap barrier --free empty &&
run own_none_vary --alloc own --after-unmap none &&
run own_bar_vary --alloc own --after-unmap barrier &&
run own_none_fixed --alloc own --after-unmap none --sizes fixed &&
run own_bar_fixed --alloc own --after-unmap barrier --sizes fixed &&
timeout -k 10 120 rocprofv3 --memory-copy-trace --kernel-trace --stats --output-format csv -d $O/dma/trace -o legs -- \
  python3 tools/probe_dma_legs.py --legs 7 --mib 64 --out $O/dma/legs.json > $O/dma/legs.out 2> $O/dma/legs.err &&
cat $O/dma/legs.json
mkdir -p $O/rows &&
for c in ns c2; do
  timeout -k 10 300 python3 tools/tune_rows.py --config $c --reps 4 --alloc clones --only lt > $O/rows/${c}_clones.jsonl 2> $O/rows/${c}_clones.err || exit 1
done
echo rows-done
