# Narrow-shard sweep: the per-rank reduce shapes of the multi-GPU runs (weak: 100*G clients x P/G
# columns; strong: 100 clients x P/G), one stripe and four stripes per step.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/narrow
mkdir -p $O
T=$R/tools/tune_reduce
for shape in "200 5849600" "200 1462400" "400 2924800" "400 731200" "800 1462400" "800 365632" "100 1462400" "100 365632" "100 3201280"; do
  set -- $shape
  TUNE_SET=narrow timeout -k 10 120 $T $1 $2 3 > $O/n$1_p$2.txt 2>&1
done
echo done
