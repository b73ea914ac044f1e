# Round 4, pass i: does the NS reduce pay for its own result stores beyond their bytes?
set -e
R=$GRAFT_REPO_ROOT
SET=nostore OUTSET=r04i/nostore ROUNDS=7 bash $R/tools/gpu_tune_reduce.sh
echo done
