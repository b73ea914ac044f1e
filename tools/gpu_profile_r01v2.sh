# Round-1 measurement pass for the row-pipelined kernel: parity suite, smoke, rocprofv3 kernel
# traces and HBM counters (separate --pmc passes) for every config, plain bench runs.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01v2
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp
for c in c2 c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o $c -- python3 $R/bench.py --config $c --no-cpu-baseline > $O/trace_${c}_bench.json 2> $O/trace_$c.err
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$c -o $c -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2> $O/fetch_$c.err
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$c -o $c -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2> $O/write_$c.err
done
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python3 $R/bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
done
for g in 2 4 8; do
  for st in 1 2 4; do
    timeout -k 10 200 python3 $R/bench.py --emulate-world $g --stripes $st --no-cpu-baseline > $O/emu_c2_weak_g${g}_s${st}.json 2>> $O/emu.err
  done
  timeout -k 10 200 python3 $R/bench.py --emulate-world $g --scaling strong --stripes 2 --no-cpu-baseline > $O/emu_c2_strong_g${g}_s2.json 2>> $O/emu.err
  timeout -k 10 200 python3 $R/bench.py --emulate-world $g --scaling strong --config c3 --stripes 2 --no-cpu-baseline > $O/emu_c3_strong_g${g}_s2.json 2>> $O/emu.err
done
for c in c1 c2 c3; do timeout -k 10 300 python3 $R/tools/bench_e2e.py --config $c > $O/e2e_$c.json 2> $O/e2e_$c.err; done
echo done
