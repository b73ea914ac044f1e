# Round 3: the GPU suite on the current tree, then the profile pass of every config
# (tools/gpu_profile.sh: bench line, rocprofv3 --kernel-trace --stats, --pmc FETCH_SIZE / WRITE_SIZE).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03d}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
OUT=${OUT:-r03d}/prof ENTRIES="${ENTRIES:-ns:ns c3:c3 c5:c5 c2:c2 c4:c4 c1k:c1k c1k_reorder:c1k:--reorder}" bash tools/gpu_profile.sh
echo done
