#!/bin/bash
# Strong-scaling probe on one GPU: ms per pass when a rank renders only its share of the
# teapot frame (103 passes over N GPUs -> 52 / 26 / 13 passes, through the RCCL path), plus the
# full frame alone and through the dist path at N=1.
# usage: tools/scaling_probe.sh TAG [extra bench args]   (outputs under gpurun_out/TAG/)
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for n in 13 26 52; do
  # a rank's share through the torch.distributed (RCCL) path, as the driver's N>1 runs render it
  timeout -k 10 300 python bench.py --steps $n --dist --no-extras "$@" > $OUT/steps$n.json 2> $OUT/steps$n.err || { tail $OUT/steps$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/steps$n.json'));print($n,d['ms_per_step'],d['value'])"
done
timeout -k 10 300 python bench.py --no-extras "$@" > $OUT/full.json 2> $OUT/full.err || { tail $OUT/full.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/full.json'));print('full',d['ms_per_step'],d['value'])"
timeout -k 10 300 python bench.py --dist --no-extras "$@" > $OUT/dist.json 2> $OUT/dist.err || { tail $OUT/dist.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/dist.json'));print('dist',d['ms_per_step'],d['value'])"
