# Round 3 closing bench lines after the shaped staggered start (every BASELINE config + the driver-style line)
export TMPDIR=/tmp
OUT=gpurun_out/r3fin2
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_teapot.json 2> $OUT/bench_teapot.err || { tail $OUT/bench_teapot.err; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_teapot_steps20.json 2> $OUT/bench_teapot_steps20.err || { tail $OUT/bench_teapot_steps20.err; exit 1; }
for cfg in cornell_plus spheres lamp teapot:--no-sort lamp:--no-sort cornell; do
  args=$(echo $cfg | tr ':' ' '); name=$(echo $cfg | tr -d ':-')
  timeout -k 10 400 python bench.py --scene $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail $OUT/bench_$name.err; exit 1; }
done
for f in $OUT/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1],d['value'],d['ms_per_step'],d.get('render_wall_ms'),d.get('bit_exact_vs_oracle'))"; done
echo done
