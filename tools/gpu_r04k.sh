# Round 4, pass k: client update host overheads (exact-type key classification, views made while
# the GPU finishes, pool-wide pack of the head chunks).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04k}
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q -k "client_receive or client_side" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_client.log 2>&1
timeout -k 10 300 python3 $R/tools/bench_client_update.py --rounds 12 --phases > $O/cu_default.json 2> $O/cu_default.err
timeout -k 10 300 python3 $R/tools/bench_client_update.py --rounds 12 --phases > $O/cu_default2.json 2> $O/cu_default2.err
timeout -k 10 300 python3 $R/tools/bench_client_update.py --device-model --layout resnet50 --rounds 8 > $O/devmodel_r50.json 2> $O/devmodel_r50.err
echo done
