# world-3 push tests repeated (stale IPC imports: receive pool + token check); stops at the first
# run that ends in anything but pass (0) or a test failure (1): a timeout or a crash ends the call
mkdir -p gpurun_out/r04ap
for i in 1 2 3 4 5 6; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_multirank.py -x -q -k "push_gather and 3" --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04ap/run$i.log 2>&1
  rc=$?
  tail -1 gpurun_out/r04ap/run$i.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "run $i rc $rc: stopping"; exit $rc; fi
done
