# Round 4, pass t: contention terms of the one-shot push gather on one GPU — a link-bound push
# kernel (into pinned host memory over PCIe) beside the reduce (the sender's side), and
# rate-limited write-only streams (what the peers' pushes do to the receiver's HBM).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04t}
mkdir -p $O
timeout -k 10 300 python3 $R/tools/overlap_probe.py --grids 0 --copy pushhost4,pushhost8,pushhost16,pushhost32,pushhost64 --copy-mb 64 > $O/overlap_push.json 2> $O/overlap_push.err
echo done
