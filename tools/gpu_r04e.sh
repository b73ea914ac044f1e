# Round 4, pass e: client-side update (pipelined pack, vectorised BN counters): parity tests,
# per-chunk phases and the A/B against the copy-engine path.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04e}
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q -k "client_side" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_client.log 2>&1
timeout -k 10 300 python3 $R/tools/bench_client_update.py --phases --rounds 6 > $O/client_update.json 2> $O/client_update.err
timeout -k 10 300 python3 $R/tools/bench_client_update.py --ab --phases --rounds 4 > $O/client_update_ab.json 2> $O/client_update_ab.err
timeout -k 10 300 python3 $R/tools/bench_client_update.py --phases --rounds 6 --transfer kernel > $O/client_update_kernel.json 2> $O/client_update_kernel.err
echo done
