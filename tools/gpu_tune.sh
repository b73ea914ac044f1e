set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
T=$R/tools/tune_reduce
TUNE_SET=blocked timeout -k 10 240 $T 100 11699136 5 > $R/gpurun_out/tune12_c2.txt 2>&1
TUNE_SET=blocked timeout -k 10 240 $T 100 25610176 3 avgm > $R/gpurun_out/tune12_c3.txt 2>&1
TUNE_SET=blocked timeout -k 10 240 $T 1000 11699136 2 > $R/gpurun_out/tune12_c4.txt 2>&1
TUNE_SET=blocked timeout -k 10 240 $T 100 86567680 2 adagrad > $R/gpurun_out/tune12_c5.txt 2>&1
TUNE_SET=blocked timeout -k 10 240 $T 1000 1169920 3 > $R/gpurun_out/tune12_n1000.txt 2>&1
TUNE_SET=blocked timeout -k 10 240 $T 10 44800 3 > $R/gpurun_out/tune12_c1.txt 2>&1
