# Round 4, pass h: client_receive on a CUDA model (tests + device-model bench on ViT-B/16 and a
# counter-free ResNet-50), and the overlap probe's read-only / write-only / low-rate stand-ins.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04h}
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q -k "client_receive or client_side" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_client.log 2>&1
timeout -k 10 300 python3 $R/tools/bench_client_update.py --device-model --layout vit_b_16 --rounds 5 > $O/devmodel_vit.json 2> $O/devmodel_vit.err
timeout -k 10 300 python3 $R/tools/bench_client_update.py --device-model --layout resnet50 --rounds 5 > $O/devmodel_r50.json 2> $O/devmodel_r50.err
timeout -k 10 300 python3 $R/tools/overlap_probe.py --grids 0 --copy 2,4,8,16,rd8,rd16,rd64,wr8,wr16,wr64 > $O/overlap_rw.json 2> $O/overlap_rw.err
echo done
