# Row-pipelined grid (reduce_kernel_rows) vs the product geometries over the per-rank shard
# shapes of the multi-GPU runs and the full single-GPU configs.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rows
mkdir -p $O
T=$R/tools/tune_reduce
for shape in "800 365632 mean" "800 1462400 mean" "400 731200 mean" "400 2924800 mean" "200 1462400 mean" "200 5849600 mean" "100 365632 mean" "100 1462400 mean" "100 11699136 mean" "100 25610176 avgm" "1000 11699136 mean" "100 86567680 adagrad"; do
  set -- $shape
  TUNE_SET=rows timeout -k 10 150 $T $1 $2 3 $3 > $O/n$1_p$2_$3.txt 2>&1
done
echo done
