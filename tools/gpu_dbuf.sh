# Epilogue batch / geometry re-check with double-buffered v_t (TUNE_V2=1, the product's form).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dbuf
mkdir -p $O
cd $R
for s in 100:86567680:adagrad 100:25610176:avgm 100:11699136:avgm; do
  IFS=: read -r n p op <<< "$s"
  TUNE_V2=1 TUNE_SET=epib16 timeout -k 10 200 tools/tune_reduce $n $p 3 $op > $O/n${n}_p${p}_$op.txt 2>&1
done
timeout -k 10 200 tools/probe_alloc 100 25610176 6 5 > $O/alloc_ns.txt 2>&1
timeout -k 10 200 tools/probe_alloc 100 25610176 6 5 > $O/alloc_ns_b.txt 2>&1
echo done
