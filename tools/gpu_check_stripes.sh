set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stripes
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python3 $R/bench.py > $O/bench_default.json 2> $O/bench.err
for g in 2 4 8; do
  timeout -k 10 200 python3 $R/bench.py --emulate-world $g --no-cpu-baseline > $O/emu_weak_g${g}_w31.json 2>> $O/emu.err
  timeout -k 10 200 python3 $R/bench.py --emulate-world $g --stripe-weights equal --no-cpu-baseline > $O/emu_weak_g${g}_eq.json 2>> $O/emu.err
  timeout -k 10 200 python3 $R/bench.py --emulate-world $g --config c4 --scaling strong --no-cpu-baseline > $O/emu_c4strong_g${g}_w31.json 2>> $O/emu.err
done
echo done
