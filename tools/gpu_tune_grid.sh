# Persistent row-pipeline grid sweep: resident blocks x piece shape, over the bench configs and
# the multi-GPU per-rank shard shapes.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/grid
mkdir -p $O
T=$R/tools/tune_reduce
for shape in "100 11699136 mean" "100 25610176 avgm" "100 86567680 adagrad" "1000 11699136 mean" "800 1462400 mean" "400 2924800 mean" "200 5849600 mean" "800 365632 mean" "400 731200 mean"; do
  set -- $shape
  TUNE_SET=grid timeout -k 10 200 $T $1 $2 3 $3 > $O/n$1_p$2_$3.txt 2>&1
done
echo done
