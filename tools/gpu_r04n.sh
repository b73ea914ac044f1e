# Round 4, pass n: client update packed by native threads (fa_py_pack_start) vs the Python pool,
# medians over calls, interleaved; device-model path; client tests.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04n}
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_pack_async.py -x -q -k "client_receive or client_side or pack" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_client.log 2>&1
for i in 1 2 3; do
  for p in 1 0; do
    timeout -k 10 300 python3 $R/tools/bench_client_update.py --rounds 16 --ref-rounds 1 --phases --native-pack $p > $O/cu_np${p}_$i.json 2> $O/cu_np${p}_$i.err
  done
done
timeout -k 10 300 python3 $R/tools/bench_client_update.py --device-model --layout resnet50 --rounds 8 > $O/devmodel_r50.json 2> $O/devmodel_r50.err
timeout -k 10 300 python3 $R/tools/bench_client_update.py --device-model --layout vit_b_16 --rounds 6 > $O/devmodel_vit.json 2> $O/devmodel_vit.err
echo done
