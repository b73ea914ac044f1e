#!/bin/bash
# tools/gpu_run.sh RECIPE [OUT] [ARGS...] — every GPU pass of this repo, one recipe each.  Run on the
# MI355X box through gpurun, e.g.
#   gpurun --timeout 1200 -- 'bash tools/gpu_run.sh suite r06x'
# Outputs go to gpurun_out/OUT (default: the recipe's name).  Every GPU step runs under its own
# time limit and the steps are chained: the first failure ends the call (no retries).
#
#   suite          pytest -m gpu (whole suite), smoke(), the default bench line   (the driver's round end)
#   bench          the default bench line (ARGS are passed to bench.py)
#   rehearsal      bench.py's N>1 path: ranks sharing the GPU over gloo (ARGS: config ranks [bench flags],
#                  default ns 2)
#   profile        per config (ARGS: tag:config[:flags] ..., default ns:ns): bench line, bench under
#                  rocprofv3 --kernel-trace --stats, separate --pmc FETCH_SIZE / WRITE_SIZE passes
#                  (then tools/refresh_profiles.sh gpurun_out/OUT profiles/<round> <tags>)
#   push_order     tests/push_order_probe.py at world 8 (ARGS are passed to it)
#   event_chain    tools/probe_event_chain (single-process cross-stream ordering)
#   slab_pmc       slab uploads vs the packed stack (tools/slab_pmc.py): kernel stats + counter passes
#   rows_pmc       the row-pointer kernel vs the stack kernel (tools/rows_pmc.py), counter passes
#                  (ARGS: config:alloc ..., default ns:clones ns:stack c3:clones)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
R=$PWD
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
RECIPE=${1:?recipe}
shift
O=$R/gpurun_out/${1:-$RECIPE}
[ $# -gt 0 ] && shift
mkdir -p "$O"

# counter groups that fit one pass each (MI355X_MICROARCH.md slot limits)
PASSES=(
  "fetch:FETCH_SIZE"
  "write:WRITE_SIZE"
  "utcl1:TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum"
  "busy:TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
  "sq:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY"
)

suite() {
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$O/pytest_gpu.log" 2>&1 || { echo "suite failed"; grep -E "FAILED|Error|passed|failed" "$O/pytest_gpu.log" | tail -20; return 1; }
  tail -1 "$O/pytest_gpu.log"
  timeout -k 10 180 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" \
    > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail "$O/smoke.log"; return 1; }
  tail -1 "$O/smoke.log"
  bench
}

bench() {
  timeout -k 10 300 python3 bench.py "$@" > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail "$O/bench.err"; return 1; }
  cat "$O/bench.json"
}

rehearsal() {
  local cfg=${1:-ns} g=${2:-2}
  if [ $# -ge 2 ]; then shift 2; else set --; fi
  FLEARN_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node="$g" --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus "$g" --steps 5 --warmup 2 \
    --config "$cfg" "$@" > "$O/rehearsal_${cfg}_g$g.json" 2> "$O/rehearsal_${cfg}_g$g.err" \
    || { echo "rehearsal failed"; tail "$O/rehearsal_${cfg}_g$g.err"; return 1; }
  echo "rehearsal $cfg g$g ok"
}

profile() {
  local entries=("$@")
  [ ${#entries[@]} -eq 0 ] && entries=(ns:ns)
  local e tag cfg flags
  for e in "${entries[@]}"; do
    IFS=: read -r tag cfg flags <<< "$e"
    flags=${flags//,/ }
    timeout -k 10 300 python3 bench.py --config "$cfg" $flags > "$O/bench_$tag.json" 2> "$O/bench_$tag.err" || return 1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$tag" -o "$tag" -- \
      python3 "$R/bench.py" --config "$cfg" $flags --no-cpu-baseline --no-verify > "$O/trace_${tag}_bench.json" 2> "$O/trace_$tag.err" || return 1
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch_$tag" -o "$tag" -- \
      python3 "$R/bench.py" --config "$cfg" $flags --no-cpu-baseline --no-verify --steps 5 --warmup 1 > /dev/null 2> "$O/fetch_$tag.err" || return 1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write_$tag" -o "$tag" -- \
      python3 "$R/bench.py" --config "$cfg" $flags --no-cpu-baseline --no-verify --steps 5 --warmup 1 > /dev/null 2> "$O/write_$tag.err" || return 1
    echo "profiled $tag"
  done
}

push_order() {
  timeout -k 10 800 python3 -u tests/push_order_probe.py --world 8 --out "$O/push_order.json" "$@" > "$O/push_order.log" 2>&1 \
    || { echo "push_order failed"; tail "$O/push_order.log"; return 1; }
  echo push-order-ok
}

event_chain() {
  [ -x tools/probe_event_chain ] || { echo "build tools/probe_event_chain first (see its header)"; return 1; }
  timeout -k 10 200 ./tools/probe_event_chain "${1:-30}" > "$O/event_chain.json" 2> "$O/event_chain.err" || return 1
  echo event-chain-ok
}

_counter_passes() {  # tag, then the program and its arguments
  local tag=$1 p name ctrs
  shift
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$tag" -o "$tag" -- "$@" \
    > "$O/trace_$tag.json" 2> "$O/trace_$tag.err" || return 1
  for p in "${PASSES[@]}"; do
    name=${p%%:*}
    ctrs=${p#*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex reduce_kernel --output-format csv -d "$O/${name}_$tag" \
      -o "$tag" -- "$@" > /dev/null 2> "$O/${name}_$tag.err" || return 1
  done
}

slab_pmc() {
  local cfgs=("$@") cfg w
  [ ${#cfgs[@]} -eq 0 ] && cfgs=(ns c3)
  for cfg in "${cfgs[@]}"; do
    timeout -k 10 180 python3 tools/slab_pmc.py --config "$cfg" --which both > "$O/slab_$cfg.json" 2> "$O/slab_$cfg.err" || return 1
    for w in engine stack; do
      _counter_passes "${cfg}_$w" python3 "$R/tools/slab_pmc.py" --config "$cfg" --which "$w" --reps 5 || return 1
    done
    echo "slab $cfg done"
  done
}

rows_pmc() {
  local runs=("$@") run cfg al
  [ ${#runs[@]} -eq 0 ] && runs=(ns:clones ns:stack c3:clones)
  for run in "${runs[@]}"; do
    IFS=: read -r cfg al <<< "$run"
    _counter_passes "${cfg}_$al" python3 "$R/tools/rows_pmc.py" --config "$cfg" --alloc "$al" --reps 5 || return 1
  done
}

case "$RECIPE" in
  suite | bench | rehearsal | profile | push_order | event_chain | slab_pmc | rows_pmc) "$RECIPE" "$@" ;;
  *) echo "unknown recipe $RECIPE"; exit 2 ;;
esac
