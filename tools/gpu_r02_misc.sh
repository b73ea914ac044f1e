set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r02_misc}
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "client_side or group_mode" > $O/pytest_misc.log 2>&1
timeout -k 10 400 python3 $R/tools/tune_splitn.py --shapes ${SHAPES:-1000:44416,1000:44426,4000:44416} > $O/splitn.jsonl 2> $O/splitn.err
echo done
