# Repeat of gpu_epi_aux.sh for two binaries and two shapes, 5 interleaved passes.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/epiaux2
mkdir -p $O
for pass in 1 2 3 4 5; do
  for s in 100:25610176:mean 100:86567680:adagrad 100:25610176:avgm; do
    IFS=: read -r n p op <<< "$s"
    for b in l0s0 l0s2; do
      TUNE_SET=epinT timeout -k 10 200 $R/tools/tune_reduce_$b $n $p 3 $op > $O/${b}_n${n}_p${p}_${op}_$pass.txt 2>&1
    done
  done
done
echo done
