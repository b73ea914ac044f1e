# Round 4, pass c: C5's whole-line f64 stores at KG = 4 (tools/tune_reduce.hip set xl4, double-
# buffered v_t as in the product), C3's KG = 3 XL kernel after the opaque-lane change (set xl),
# then the product's c3 / c5 / ns bench lines on this box.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04c}
mkdir -p $O
TUNE_V2=1 SET=xl4 OUTSET=r04c/xl4 ROUNDS=5 bash $R/tools/gpu_tune_reduce.sh
TUNE_V2=1 SET=xl OUTSET=r04c/xl ROUNDS=3 bash $R/tools/gpu_tune_reduce.sh
for c in ns c3 c5; do
  timeout -k 10 300 python3 $R/bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
done
echo done
