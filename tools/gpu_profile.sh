# Measurement pass behind profiles/<round>/<tag>/: for every TAG:CONFIG[:FLAGS] entry, a plain
# bench line, the same command under rocprofv3 --kernel-trace --stats, and separate --pmc
# FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md: one TCC counter group per pass).
#   OUT=r02_prof ENTRIES="ns:ns c3:c3 c1k_reorder:c1k:--reorder" bash tools/gpu_profile.sh
# then: tools/refresh_profiles.sh gpurun_out/$OUT profiles/<round> <tags...>
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-prof}
mkdir -p $O
for e in ${ENTRIES:-ns:ns}; do
  IFS=: read -r tag cfg flags <<< "$e"
  flags=${flags//,/ }
  timeout -k 10 300 python3 $R/bench.py --config $cfg $flags > $O/bench_$tag.json 2> $O/bench_$tag.err
done
cd /tmp && export TMPDIR=/tmp
for e in ${ENTRIES:-ns:ns}; do
  IFS=: read -r tag cfg flags <<< "$e"
  flags=${flags//,/ }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$tag -o $tag -- python3 $R/bench.py --config $cfg $flags --no-cpu-baseline --no-verify > $O/trace_${tag}_bench.json 2> $O/trace_$tag.err
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$tag -o $tag -- python3 $R/bench.py --config $cfg $flags --no-cpu-baseline --no-verify --steps 5 --warmup 1 > /dev/null 2> $O/fetch_$tag.err
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$tag -o $tag -- python3 $R/bench.py --config $cfg $flags --no-cpu-baseline --no-verify --steps 5 --warmup 1 > /dev/null 2> $O/write_$tag.err
done
echo done
