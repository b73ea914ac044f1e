# Round 4, pass j: cross-group prefetch (PFG): the next group's first loads issued before this group's
# epilogue stores, so the store drain overlaps the next reads.
set -e
R=$GRAFT_REPO_ROOT
SET=pfg OUTSET=r04j/pfg ROUNDS=7 bash $R/tools/gpu_tune_reduce.sh
echo done
