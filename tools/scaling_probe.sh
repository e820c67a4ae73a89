#!/bin/bash
# Strong-scaling probe on one GPU: ms per pass when a rank renders only its share of the
# teapot frame (103 passes over N GPUs -> 52 / 26 / 13 passes), plus the dist path at N=1.
# usage: tools/scaling_probe.sh TAG [extra bench args]   (outputs under gpurun_out/TAG/)
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for n in 13 26 52; do
  timeout -k 10 300 python bench.py --steps $n --no-counters --no-cpu-baseline "$@" > $OUT/steps$n.json 2> $OUT/steps$n.err || { tail $OUT/steps$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/steps$n.json'));print($n,d['ms_per_step'],d['value'])"
done
timeout -k 10 300 python bench.py --no-counters --no-cpu-baseline "$@" > $OUT/full.json 2> $OUT/full.err || { tail $OUT/full.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/full.json'));print('full',d['ms_per_step'],d['value'])"
timeout -k 10 300 python bench.py --dist --no-counters --no-cpu-baseline "$@" > $OUT/dist.json 2> $OUT/dist.err || { tail $OUT/dist.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/dist.json'));print('dist',d['ms_per_step'],d['value'])"
