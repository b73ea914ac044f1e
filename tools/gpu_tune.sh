set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
T=$R/tools/tune_reduce
TUNE_SET=buf timeout -k 10 240 $T 100 11699133 1 > $R/gpurun_out/tune11_ragged.txt 2>&1
TUNE_SET=buf timeout -k 10 240 $T 7 1000003 1 avgm > $R/gpurun_out/tune11_ragged_avgm.txt 2>&1
for nc in 11699136 12582912 25610176; do
  TUNE_SET=buf timeout -k 10 240 $T 100 $nc 5 > $R/gpurun_out/tune11_$nc.txt 2>&1
done
TUNE_SET=buf timeout -k 10 240 $T 100 25610176 3 avgm > $R/gpurun_out/tune11_c3avgm.txt 2>&1
TUNE_SET=buf timeout -k 10 240 $T 100 86567680 2 adagrad > $R/gpurun_out/tune11_c5.txt 2>&1
TUNE_SET=buf timeout -k 10 240 $T 1000 11699136 2 > $R/gpurun_out/tune11_c4.txt 2>&1
TUNE_SET=buf timeout -k 10 240 $T 1000 1169920 3 > $R/gpurun_out/tune11_n1000.txt 2>&1
