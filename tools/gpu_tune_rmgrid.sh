set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rmgrid
mkdir -p $O
T=$R/tools/tune_reduce
for shape in "100 11699136 mean" "1000 11699136 mean" "200 11699136 mean" "100 25610176 avgm" "100 86567680 adagrad" ; do
  set -- $shape
  TUNE_SET=rmgrid timeout -k 10 200 $T $1 $2 3 $3 > $O/n$1_p$2_$3.txt 2>&1
done
echo done
