#!/bin/bash
# Round measurement on the GPU box: GPU test suite, bench lines for the BASELINE configs, the
# rocprofv3 kernel-trace summary of the headline bench command and the PMC traffic passes.
# Every GPU step has its own time limit; the script stops at the first failure.
# usage: tools/round_measure.sh TAG          (outputs under gpurun_out/TAG/)
TAG=$1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() { echo "== $*"; }
step tests
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
step bench teapot
timeout -k 10 400 python bench.py > $OUT/bench_teapot.json 2> $OUT/bench_teapot.err || { tail $OUT/bench_teapot.err; exit 1; }
for cfg in "cornell_plus" "spheres" "lamp" "teapot --no-sort" "lamp --no-sort"; do
  name=$(echo $cfg | tr -d ' -'); step bench $cfg
  timeout -k 10 400 python bench.py --scene $cfg --no-cpu-baseline > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail $OUT/bench_$name.err; exit 1; }
done
step rocprof kernel trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-counters > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
step pmc traffic
bash tools/pmc.sh ${TAG}_tf tools/pmc_groups/traffic.txt || exit 1
step pmc trace
bash tools/pmc.sh ${TAG}_tr tools/pmc_groups/trace.txt || exit 1
step strong-scaling probe
bash tools/scaling_probe.sh $TAG/scaling || exit 1
echo done
