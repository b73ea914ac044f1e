# Geometry sweeps of tools/tune_reduce.hip behind profiles/r01_rows/tune/<SET>/ (variants
# interleaved in one process, bitwise-checked, bracketed by streaming-read and float4-copy roofs).
#   SET=rm bash tools/gpu_tune_reduce.sh        (build: hipcc -O3 --offload-arch=gfx950 ... tools/tune_reduce.hip)
set -e
R=$GRAFT_REPO_ROOT
SET=${SET:-rm}
O=$R/gpurun_out/${OUTSET:-$SET}
mkdir -p $O
T=$R/tools/tune_reduce
case $SET in
  narrow) SHAPES="200:5849600:mean 200:1462400:mean 400:2924800:mean 400:731200:mean 800:1462400:mean 800:365632:mean 100:1462400:mean 100:365632:mean 100:3201280:mean" ;;
  nsgrid) SHAPES="100:25610176:mean 100:11699136:mean 100:86567680:mean 1000:11699136:mean" ;;
  kgrid) SHAPES="100:25610176:avgm 100:25610176:mean 100:25610176:adagrad" ;;
  timeline) SHAPES="100:25610176:avgm 100:86567680:adagrad" ;;
  epiw) SHAPES="100:25610176:avgm 100:86567680:adagrad 100:11699136:avgm" ;;
  epib) SHAPES="100:25610176:avgm 100:86567680:adagrad 100:11699136:adagrad" ;;
  epi) SHAPES="100:25610176:avgm 100:86567680:adagrad 100:3201280:avgm 800:1462400:avgm 100:11699136:adagrad 400:731200:adagrad" ;;
  grid|inflight|misc) SHAPES="100:11699136:mean 1000:11699136:mean 100:25610176:avgm 100:86567680:adagrad 800:1462400:mean 400:731200:mean 200:5849600:mean" ;;
  stagger) SHAPES="100:11699136:mean 200:11699136:mean 1000:11699136:mean 100:25610176:avgm" ;;
  deep3) SHAPES="1000:177704:mean 800:365632:mean 400:731200:mean 100:1462400:mean 200:5849600:mean 1000:177704:avgm" ;;
  xlg) SHAPES="100:86567680:adagrad 100:86567680:avgm" ;;
  pfg) SHAPES="100:25610176:mean 100:25610176:avgm 100:86567680:adagrad 100:11699136:mean 1000:11699136:mean 100:86567680:mean" ;;
  nostore) SHAPES="100:25610176:mean 100:25610176:mean" ;;
  xl4) SHAPES="100:86567680:adagrad 100:86567680:avgm" ;;
  xl) SHAPES="100:25610176:avgm 100:25610176:adagrad 100:86567680:adagrad 100:11699136:avgm 300:25610176:avgm" ;;
  nlb) SHAPES="1000:44426:mean 2000:44426:mean 400:44426:mean 100:44426:mean 1000:44426:avgm 300:70001:mean 1000:177704:mean" ;;
  deep2) SHAPES="1000:44426:mean 1000:44426:avgm 400:44426:mean 100:44426:mean 2000:44426:mean 300:70001:mean 1000:3:mean" ;;
  lds) SHAPES="1000:44426:mean 400:44426:mean 100:44426:mean 2000:44426:mean 1000:177704:mean 300:70001:mean 1000:44426:avgm" ;;
  epib4) SHAPES="100:25610176:avgm 100:86567680:adagrad 100:25610176:mean 100:11699136:avgm 1000:11699136:mean" ;;
  epib16) SHAPES="100:25610176:avgm 100:86567680:adagrad 100:25610176:mean" ;;
  tail) SHAPES="100:25610176:avgm 100:25610176:mean 100:86567680:adagrad" ;;
  deep) SHAPES="1000:44426:mean 1000:44426:avgm 400:44426:mean 100:44426:mean 2000:44426:mean 1000:177704:mean" ;;
  dfr) SHAPES="100:25610176:avgm 100:25610176:mean 100:86567680:adagrad 100:11699136:avgm" ;;
  one) SHAPES="100:86567680:adagrad 100:25610176:avgm 100:11699136:mean 1000:11699136:mean" ;;
  *) SHAPES="100:11699136:mean 1000:11699136:mean 200:11699136:mean 100:25610176:avgm 100:86567680:adagrad 800:1462400:mean" ;;
esac
for s in $SHAPES; do
  IFS=: read -r n p op <<< "$s"
  TUNE_SET=$SET timeout -k 10 200 $T $n $p ${ROUNDS:-3} $op > $O/n${n}_p${p}_$op.txt 2>&1
done
echo done
