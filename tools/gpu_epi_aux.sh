# A/B of the epilogue's cache-policy bits (state loads / result stores; 2 = non-temporal): the
# same tune binary built four ways (-DFA_EPI_LOAD_AUX / -DFA_EPI_STORE_AUX), run interleaved.
#   for v in "0 0" "0 2" "2 0" "2 2"; do set -- $v; hipcc ... -DFA_EPI_LOAD_AUX=$1 -DFA_EPI_STORE_AUX=$2 \
#       tools/tune_reduce.hip -o tools/tune_reduce_l$1s$2; done
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/epiaux
mkdir -p $O
for pass in 1 2; do
  for s in 100:25610176:avgm 100:86567680:adagrad 100:11699136:avgm 100:25610176:mean; do
    IFS=: read -r n p op <<< "$s"
    for b in l0s0 l0s2 l2s0 l2s2; do
      TUNE_SET=epinT timeout -k 10 200 $R/tools/tune_reduce_$b $n $p 3 $op > $O/${b}_n${n}_p${p}_${op}_$pass.txt 2>&1
    done
  done
done
echo done
