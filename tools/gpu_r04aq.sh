# push tests (kernel + dma, worlds 2/3/4) repeated with the receive pool; stops at the first run
# that ends in anything but pass (0) or a test failure (1)
mkdir -p gpurun_out/r04aq
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_multirank.py -x -q -k "push_gather" --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04aq/run$i.log 2>&1
  rc=$?
  echo "run $i: $(tail -1 gpurun_out/r04aq/run$i.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "run $i rc $rc: stopping"; exit $rc; fi
done
