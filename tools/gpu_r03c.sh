# Round 3: split-N guard tests + timing, C1 host profile, allocation-order A/B of the
# row-pointer kernel.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03c}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python tools/time_splitn_guard.py > $O/time_splitn_guard.jsonl 2>&1
timeout -k 10 200 python tools/prof_host_c1.py > $O/prof_host_c1.txt 2>&1
for alloc in views clones stack; do
  for c in c2 ns; do
    timeout -k 10 300 python tools/tune_rows.py --config $c --alloc $alloc --reps 5 --only lib > $O/rows_${c}_${alloc}.jsonl 2> $O/rows_${c}_${alloc}.err
  done
done
echo done
