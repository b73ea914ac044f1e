# Replicated-tail round: GPU suite (multi-rank ShardedReducer with a tail, bench rehearsal), then
# the emulated per-rank steps (rank 0's stripes + tail on one GPU, a priori gather model).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-tail}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
for g in 2 4 8; do
  for c in ns c5; do
    timeout -k 10 200 python3 $R/bench.py --config $c --emulate-world $g --scaling strong --no-cpu-baseline --steps 20 > $O/emu_${c}_strong_g$g.json 2> $O/emu_${c}_strong_g$g.err
  done
done
echo done
