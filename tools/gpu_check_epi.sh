set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/chkepi
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
for c in c2 c3 c4 c5; do timeout -k 10 200 python3 $R/bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err; done
for g in 2 4 8; do timeout -k 10 200 python3 $R/bench.py --emulate-world $g --scaling strong --config c3 --no-cpu-baseline > $O/emu_c3strong_g$g.json 2>> $O/emu.err; done
echo done
