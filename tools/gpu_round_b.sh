# Measurement pass B on one MI355X: bench lines with the CPU baseline, end-to-end (host uploads,
# PCIe-inclusive) and HTTP-mode (wire codec) rounds.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rb
mkdir -p $O
lscpu > $O/host_lscpu.txt
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python3 $R/bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
done
for c in c1 c2 c3; do
  timeout -k 10 300 python3 $R/tools/bench_e2e.py --config $c > $O/e2e_$c.json 2> $O/e2e_$c.err
done
timeout -k 10 300 python3 $R/tools/bench_e2e.py --config c2 --output float32 > $O/e2e_c2_f32.json 2> $O/e2e_c2_f32.err
for c in c1 c2; do
  timeout -k 10 600 python3 $R/tools/bench_wire.py --config $c > $O/wire_$c.json 2> $O/wire_$c.err
done
echo done-b
