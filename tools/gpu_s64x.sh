# f64 state / result stores: the product's two half-line stores per quad vs whole-line stores
# regrouped through LDS (FA_EPI_STORE64_LDS=1), double-buffered v_t (TUNE_V2=1), alternating
# binaries on one box.  Build: tools/tune_reduce (product) and tools/tune_reduce_s64x
# (-DFA_EPI_STORE64_LDS=1).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s64x
mkdir -p $O
cd $R
for s in 100:86567680:adagrad 100:25610176:avgm 100:11699136:avgm; do
  IFS=: read -r n p op <<< "$s"
  for b in tune_reduce tune_reduce_s64x tune_reduce tune_reduce_s64x; do
    TUNE_V2=1 TUNE_SET=epib4 timeout -k 10 200 tools/$b $n $p 3 $op >> $O/${b}_n${n}_p${p}_$op.txt 2>&1
  done
done
echo done
