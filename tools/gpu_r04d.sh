# Round 4, pass d: translation prefetch in the row-pointer kernel (tools/tune_rows.py rm_*pf*
# variants) against the product plan and the stack kernel, per allocation pattern.
set -e
R=$GRAFT_REPO_ROOT
for al in clones views stack; do
  OUT=r04d ALLOC=$al CONFIGS="ns c2" ONLY="lib,rm_v8w8kg2,rm_v16w4kg2" REPS=4 bash $R/tools/gpu_tune_rows.sh
done
echo done
