# In-place vs double-buffered epilogue state (out32 == prev; v_out = a second v), one process per shape.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/inplace
mkdir -p $O
cd $R
for s in 100:25610176:avgm 100:86567680:adagrad 100:11699136:avgm 100:25610176:adagrad; do
  IFS=: read -r n p op <<< "$s"
  TUNE_SET=inplace timeout -k 10 200 tools/tune_reduce $n $p 3 $op > $O/n${n}_p${p}_$op.txt 2>&1
done
echo done
