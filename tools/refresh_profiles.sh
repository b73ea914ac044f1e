# Copy one `tools/gpu_run.sh profile` pass into the tracked record and recompute profiles/traffic.json:
#   bash tools/refresh_profiles.sh gpurun_out/<OUT> profiles/<round> tag [tag ...]
set -e
S=$1
D=$2
shift 2
for c in "$@"; do
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
  python -c "
import json
d=json.load(open('$D/$c/bench_$c.json')); t=json.load(open('profiles/traffic.json'))['$c']
r=d['roofline']; ks=t['rocprof_kernel_stats']
print('$c', 'bench_us', r['launch_us'], 'rocprof_us', round(ks['avg_ns']/1e3,1), 'frac_bench', r['frac'],
      'frac_rocprof', round(r['bytes_per_launch']/ks['avg_ns']/8000,4), 'traffic/alg', t['traffic_over_algorithmic'],
      'cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
