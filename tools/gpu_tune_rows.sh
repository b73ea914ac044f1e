# Geometry / work-plan sweep of the row-pointer kernel (tools/tune_rows.py, tools/libtune_rows.so)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-tune_rows2}
mkdir -p $O
for c in ${CONFIGS:-c2 ns}; do
  timeout -k 10 400 python3 $R/tools/tune_rows.py --config $c --reps ${REPS:-4} --alloc ${ALLOC:-views} ${ONLY:+--only $ONLY} > $O/${c}_${ALLOC:-views}.jsonl 2> $O/${c}.err
done
echo done
