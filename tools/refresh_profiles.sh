# Copy one gpu_profile_r01v2.sh pass (gpurun_out/r01v2) into profiles/r01_rows and recompute
# profiles/traffic.json; prints the numbers DESIGN.md §5/§6 quote.
set -e
S=gpurun_out/r01v2
D=profiles/r01_rows
for c in c2 c3 c4 c5; do
  mkdir -p $D/$c
  cp $S/bench_$c.json $D/$c/bench_$c.json
  cp $S/trace_${c}_bench.json $D/$c/bench_${c}_under_rocprof.json
  cp $S/trace_$c/${c}_kernel_stats.csv $D/$c/${c}_kernel_stats.csv
  cp $S/trace_$c/${c}_kernel_trace.csv $D/$c/${c}_kernel_trace.csv
  cp $S/fetch_$c/${c}_counter_collection.csv $D/$c/${c}_pmc_FETCH_SIZE.csv
  cp $S/write_$c/${c}_counter_collection.csv $D/$c/${c}_pmc_WRITE_SIZE.csv
  B=$(python -c "import json; print(json.load(open('$S/bench_$c.json'))['roofline']['bytes_per_launch'])")
  python tools/pmc_traffic.py --config $c --stats $D/$c/${c}_kernel_stats.csv --fetch $D/$c/${c}_pmc_FETCH_SIZE.csv \
    --write $D/$c/${c}_pmc_WRITE_SIZE.csv --bytes-per-launch $B --out profiles/traffic.json \
    --source "$D/$c/${c}_pmc_{FETCH,WRITE}_SIZE.csv (rocprofv3 --pmc, separate passes)" > /dev/null
done
rm -f $D/scaling_emulated/emu_*.json
cp $S/emu_*.json $D/scaling_emulated/
cp $S/e2e_*.json $D/e2e/
cp $S/pytest_gpu.log $S/smoke.log $D/
for c in c2 c3 c4 c5; do python -c "
import json
d=json.load(open('$D/$c/bench_$c.json')); t=json.load(open('profiles/traffic.json'))['$c']; u=json.load(open('$D/$c/bench_${c}_under_rocprof.json'))
r=d['roofline']
print('$c', r['launch_us'], round(t['rocprof_kernel_stats']['avg_ns']/1e3,1), u['roofline']['launch_us'], r['achieved'], round(r['frac']*100,1), t['traffic_over_algorithmic'], d['cpu_baseline']['value'], t['rocprof_kernel_stats']['name'][:40])"; done
for f in $D/scaling_emulated/*.json; do python -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], d['ms_per_step'])"; done
for c in c1 c2 c3; do python -c "
import json; d=json.load(open('$D/e2e/e2e_$c.json')); print('$c', d['median_s'], d['e2e_GiB_s_algorithmic'], d['pack_h2d_GB_s'])"; done
