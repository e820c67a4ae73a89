#!/bin/bash
# Round 6, call AI: the one-GPU strong-scaling probe at the round's end, both multi-GPU paths on one box: a rank's share
# (13 / 26 / 52 passes) through torch.distributed (tools/scaling_probe.sh) and through the in-library path (--inlib).
export TMPDIR=/tmp
O=gpurun_out/r06ai; mkdir -p $O
bash tools/scaling_probe.sh r06ai/dist > $O/scaling_probe.log 2>&1 || { cat $O/scaling_probe.log; exit 1; }
for n in 13 26 52; do
  timeout -k 10 300 python bench.py --steps $n --warmup 2 --inlib --no-extras > $O/inlib$n.json 2> $O/inlib$n.err || { tail $O/inlib$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/inlib$n.json'));print('inlib', $n, d['ms_per_step'], d['value'])" >> $O/scaling_probe.log
done
cat $O/scaling_probe.log
