# Round 3 measurement, part B (GPU box): PMC records of the other configs, then their bench lines
TAG=$1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/pmc_configs.sh ${TAG}_pmc > $OUT/pmc_configs.log 2>&1 || { tail -20 $OUT/pmc_configs.log; exit 1; }
cp profiles/pmc_traffic.json profiles/pmc_issue.json $OUT/
for cfg in cornell_plus spheres lamp teapot:--no-sort lamp:--no-sort cornell; do
  args=$(echo $cfg | tr ':' ' '); name=$(echo $cfg | tr -d ':-'); echo "== bench $args $(date +%T)"
  timeout -k 10 400 python bench.py --scene $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail $OUT/bench_$name.err; exit 1; }
  cut -c1-160 $OUT/bench_$name.json
done
echo done-b
