# Round-2 measurement pass for the north-star shape (ns: FedAVG 100 x ResNet-50) and the
# small-P / deep-N shape (c1k: 1000 x LeNet5): plain bench lines, rocprofv3 kernel stats and
# separate FETCH_SIZE / WRITE_SIZE passes; plus the launcher's refusal on a 1-GPU box.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r02_ns}
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
for c in ${CONFIGS:-ns c1k}; do
  timeout -k 10 300 python3 $R/bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
done
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-ns c1k}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o $c -- python3 $R/bench.py --config $c --no-cpu-baseline > $O/trace_${c}_bench.json 2> $O/trace_$c.err
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$c -o $c -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2> $O/fetch_$c.err
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$c -o $c -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2> $O/write_$c.err
done
if timeout -k 10 120 python3 $R/bench.py --gpus 2 --steps 2 --warmup 1 > $O/gpus2.out 2> $O/gpus2.err; then
  echo "gpus2 rc=0 (unexpected on a 1-GPU box)" >> $O/gpus2.err
else
  echo "gpus2 rc=$? (expected non-zero on a 1-GPU box)" >> $O/gpus2.err
fi
echo done
