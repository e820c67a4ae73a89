#!/bin/bash
# Round measurement on the GPU box: GPU test suite, PMC traffic of one profiled pass (summarised
# into profiles/pmc_traffic.json, which the bench reads for roofline.traffic), bench lines for the
# BASELINE configs, and the rocprofv3 kernel-trace summary of the headline bench command.
# Every GPU step has its own time limit; the script stops at the first failure.
# usage: tools/round_measure.sh TAG [skip-tests] [configs...]     (outputs under gpurun_out/TAG/)
TAG=$1; shift
SKIP_TESTS=0
if [ "$1" = "skip-tests" ]; then SKIP_TESTS=1; shift; fi
CONFIGS=${*:-"cornell_plus spheres lamp teapot_--no-sort lamp_--no-sort cornell"}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
REV=$(cat .rev 2>/dev/null || echo unknown)
step() { echo "== $* $(date +%T)"; }
if [ $SKIP_TESTS = 0 ]; then
  step tests
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
fi
step pmc traffic teapot
bash tools/pmc.sh ${TAG}_tf tools/pmc_groups/traffic.txt > $OUT/pmc_tf.log 2>&1 || { cat $OUT/pmc_tf.log; exit 1; }
python3 tools/pmc_summary.py ${TAG}_tf --json profiles/pmc_traffic.json \
    --workload "teapot.scene 1920x1080 2048spp 16 bounces sort=on" \
    --run "rev $REV: python3 bench.py --steps 1 --warmup 0 --no-extras (tools/pmc.sh ${TAG}_tf)" > $OUT/pmc_summary_teapot.txt || exit 1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
step bench teapot
timeout -k 10 400 python bench.py > $OUT/bench_teapot.json 2> $OUT/bench_teapot.err || { tail $OUT/bench_teapot.err; exit 1; }
cat $OUT/bench_teapot.json
step rocprof kernel trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-counters > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
for cfg in $CONFIGS; do
  args=$(echo $cfg | tr '_' ' '); name=$(echo $cfg | tr -d '_-'); step bench $args
  timeout -k 10 400 python bench.py --scene $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail $OUT/bench_$name.err; exit 1; }
done
echo done
