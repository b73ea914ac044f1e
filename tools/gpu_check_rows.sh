# Parity suite + bench lines for every config + emulated per-rank multi-GPU shards.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/chk
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python $R/bench.py > $O/bench_default.json 2> $O/bench_default.err
for c in c3 c4 c5; do timeout -k 10 200 python $R/bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err; done
for g in 2 4 8; do
  for st in 1 2 4; do
    timeout -k 10 200 python $R/bench.py --emulate-world $g --stripes $st --no-cpu-baseline > $O/emu_c2_g${g}_s${st}.json 2> $O/emu.err
  done
  timeout -k 10 200 python $R/bench.py --emulate-world $g --scaling strong --config c3 --stripes 2 --no-cpu-baseline > $O/emu_c3strong_g${g}.json 2>> $O/emu.err
done
echo done
