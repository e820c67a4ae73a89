#!/bin/bash
# First half of a round measurement (GPU box): GPU tests, bench lines for every BASELINE config,
# rocprofv3 kernel-trace summary of the headline bench.  usage: tools/measure_a.sh TAG
TAG=$1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
echo "== tests"
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "== bench teapot"
timeout -k 10 400 python bench.py > $OUT/bench_teapot.json 2> $OUT/bench_teapot.err || { tail $OUT/bench_teapot.err; exit 1; }
for cfg in "cornell_plus" "spheres" "lamp" "teapot --no-sort" "lamp --no-sort"; do
  name=$(echo $cfg | tr -d ' -'); echo "== bench $cfg"
  timeout -k 10 400 python bench.py --scene $cfg --no-cpu-baseline > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail $OUT/bench_$name.err; exit 1; }
done
echo "== rocprof kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-counters > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
echo done
