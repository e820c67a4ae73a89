#!/bin/bash
# r05: passes in flight x hardware queues, through the torch.distributed (RCCL) path at N=1 and the plain path:
# is the "20 in flight next to RCCL" cliff a queue-count effect?
export TMPDIR=/tmp
OUT=gpurun_out/r5_q1; mkdir -p $OUT
for cfg in 16:28 20:28 20:24 20:20 20:16 16:16 16:20 20:12; do
  inf=${cfg%%:*}; q=${cfg##*:}
  RTAMD_INFLIGHT=$inf RTAMD_HW_QUEUES=$q timeout -k 10 200 python bench.py --dist --steps 20 --warmup 5 --no-extras > $OUT/dist_${inf}_$q.json 2> $OUT/dist_${inf}_$q.err || { tail $OUT/dist_${inf}_$q.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/dist_${inf}_$q.json'));print('dist inflight $inf queues $q:',d['ms_per_step'])"
done
for cfg in 20:24 20:32 24:32 20:16; do
  inf=${cfg%%:*}; q=${cfg##*:}
  RTAMD_INFLIGHT=$inf RTAMD_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras > $OUT/plain_${inf}_$q.json 2> $OUT/plain_${inf}_$q.err || { tail $OUT/plain_${inf}_$q.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/plain_${inf}_$q.json'));print('plain inflight $inf queues $q:',d['ms_per_step'])"
done
