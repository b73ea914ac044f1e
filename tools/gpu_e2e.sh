# Host-side numbers behind DESIGN.md §5: loopback rounds (tools/bench_e2e.py), HTTP-mode rounds
# (tools/bench_wire.py), device-resident uploads (tools/bench_rows.py) and the emulated per-rank
# steps of the multi-GPU jobs (bench.py --emulate-world).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-e2e}
mkdir -p $O
for c in c1 c2 c3; do timeout -k 10 300 python3 $R/tools/bench_e2e.py --config $c > $O/e2e_$c.json 2> $O/e2e_$c.err; done
for c in c1 c2; do timeout -k 10 300 python3 $R/tools/bench_wire.py --config $c > $O/wire_$c.json 2> $O/wire_$c.err; done
timeout -k 10 300 python3 $R/tools/bench_wire.py --config c2 --stage > $O/wire_c2_stage.json 2> $O/wire_c2_stage.err
for c in c2 ns c3; do timeout -k 10 300 python3 $R/tools/bench_rows.py --config $c > $O/rows_$c.json 2> $O/rows_$c.err; done
for g in 2 4 8; do
  timeout -k 10 200 python3 $R/bench.py --emulate-world $g --scaling weak --no-cpu-baseline --steps 30 > $O/emu_ns_weak_g$g.json 2> $O/emu_ns_weak_g$g.err
  timeout -k 10 200 python3 $R/bench.py --emulate-world $g --scaling strong --no-cpu-baseline --steps 30 > $O/emu_ns_strong_g$g.json 2> $O/emu_ns_strong_g$g.err
  timeout -k 10 200 python3 $R/bench.py --config c4 --scaling strong --emulate-world $g --no-cpu-baseline --steps 20 > $O/emu_c4strong_g$g.json 2> $O/emu_c4strong_g$g.err
  timeout -k 10 200 python3 $R/bench.py --config c5 --scaling strong --emulate-world $g --no-cpu-baseline --steps 20 > $O/emu_c5strong_g$g.json 2> $O/emu_c5strong_g$g.err
done
echo done
