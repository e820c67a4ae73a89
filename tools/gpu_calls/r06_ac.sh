#!/bin/bash
# Round 6, call AC: the teapot lines at HEAD with the roofline priced from the timed regime's own PMC records
# (kernels unchanged since 80cb38a): the full frame (bench.py defaults) and the driver's --steps 20 --warmup 5.
export TMPDIR=/tmp
O=gpurun_out/r06ac; mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench_teapot.json 2> $O/bench_teapot.err || { tail $O/bench_teapot.err; exit 1; }
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_teapot_steps20.json 2> $O/bench_teapot_steps20.err || { tail $O/bench_teapot_steps20.err; exit 1; }
for f in bench_teapot bench_teapot_steps20; do
  python3 -c "import json; j=json.load(open('$O/$f.json')); r=j['roofline']; print('$f', j['value'], j['ms_per_step'], j['render_wall_ms'], j['bit_exact_vs_oracle'], r['frac'], r['traffic_frac'], r['timed']['wave_cycle_share'], r['timed']['one_pass'])"
done
