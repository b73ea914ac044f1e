# Emulated per-rank steps (one GPU) of the 2/4/8-GPU jobs with the current kernels and the
# default stripes: the reduce of rank 0's columns, no gather.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/emu
mkdir -p $O
for g in 2 4 8; do
  timeout -k 10 200 python3 $R/bench.py --emulate-world $g --no-cpu-baseline --steps 30 > $O/emu_weak_g$g.json 2> $O/emu_weak_g$g.err
  timeout -k 10 200 python3 $R/bench.py --config c4 --scaling strong --emulate-world $g --no-cpu-baseline --steps 20 > $O/emu_c4strong_g$g.json 2> $O/emu_c4strong_g$g.err
done
timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --steps 30 > $O/bench_n1.json 2> $O/bench_n1.err
echo done
