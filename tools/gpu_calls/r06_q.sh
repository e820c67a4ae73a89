#!/bin/bash
# Round 6, call Q: a rank's 13 / 26-pass share through the in-library path (rt_multi at N = 1, RCCL communicator,
# 16 passes in flight) beside the torch.distributed path.
export TMPDIR=/tmp
O=gpurun_out/r06q; mkdir -p $O
for n in 13 26; do
  timeout -k 10 300 python bench.py --steps $n --warmup 2 --inlib --no-extras > $O/inlib$n.json 2> $O/inlib$n.err || { tail $O/inlib$n.err; exit 1; }
  timeout -k 10 300 python bench.py --steps $n --warmup 2 --dist --no-extras > $O/dist$n.json 2> $O/dist$n.err || { tail $O/dist$n.err; exit 1; }
  python3 -c "import json;a=json.load(open('$O/inlib$n.json'));b=json.load(open('$O/dist$n.json'));print($n,'inlib',a['ms_per_step'],a['config']['launch'],'| dist',b['ms_per_step'])"
done
