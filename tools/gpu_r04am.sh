# Round 4, pass am: row-pitch padding of the client stack across the BASELINE shapes (interleaved).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04am}
mkdir -p $O
timeout -k 10 300 python3 $R/tools/probe_stride_variance.py 0,64,320,576 3 resnet18 100 > $O/c2.json 2> $O/c2.err
timeout -k 10 300 python3 $R/tools/probe_stride_variance.py 0,64,320,576 3 resnet50 100 > $O/ns.json 2> $O/ns.err
timeout -k 10 300 python3 $R/tools/probe_stride_variance.py 0,64,320,576 2 resnet18 1000 > $O/c4.json 2> $O/c4.err
timeout -k 10 300 python3 $R/tools/probe_stride_variance.py 0,64,320,576 2 vit_b_16 100 > $O/c5.json 2> $O/c5.err
echo done
