# Split-N geometry sweep (tools/tune_splitn.py) -> gpurun_out/tune_splitn
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-tune_splitn}
mkdir -p $O
timeout -k 10 400 python3 $R/tools/tune_splitn.py ${SHAPES:+--shapes $SHAPES} > $O/splitn.jsonl 2> $O/splitn.err
echo done
