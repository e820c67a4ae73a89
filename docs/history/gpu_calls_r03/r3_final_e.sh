# Round 3 closing measurement with the root step at refill: part A (tests, smoke, PMC records of teapot, teapot lines, kernel trace),
# then every other config's bench line
export TMPDIR=/tmp
bash tools/round_measure.sh r3fin4 A || exit 1
OUT=gpurun_out/r3fin4
for cfg in cornell_plus spheres lamp teapot:--no-sort lamp:--no-sort cornell; do
  args=$(echo $cfg | tr ':' ' '); name=$(echo $cfg | tr -d ':-')
  timeout -k 10 400 python bench.py --scene $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail $OUT/bench_$name.err; exit 1; }
done
for f in $OUT/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1],d['value'],d['ms_per_step'],d.get('render_wall_ms'),d.get('bit_exact_vs_oracle'))"; done
echo done-final
