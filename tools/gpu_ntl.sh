# Cached vs non-temporal epilogue state loads (FA_EPI_LOAD_AUX 0 / 2), each binary's "inplace" set
# (in place vs double-buffered state) on the fused shapes, alternating binaries on one box.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ntl
mkdir -p $O
cd $R
for s in 100:86567680:adagrad 100:25610176:avgm; do
  IFS=: read -r n p op <<< "$s"
  for b in tune_reduce tune_reduce_ntl tune_reduce tune_reduce_ntl; do
    TUNE_SET=inplace timeout -k 10 200 tools/$b $n $p 3 $op >> $O/${b}_n${n}_p${p}_$op.txt 2>&1
  done
done
echo done
