#!/bin/bash
# r05: the dist path's 20-in-flight cliff: overlap off / stagger off / group size
export TMPDIR=/tmp
OUT=gpurun_out/r5_q2; mkdir -p $OUT
run() { name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --dist --steps 20 --warmup 5 --no-extras > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name',d['ms_per_step'])"
}
run if20_base RTAMD_INFLIGHT=20
run if20_nooverlap RTAMD_INFLIGHT=20 RTAMD_XCHG_OVERLAP=0
run if20_nostagger RTAMD_INFLIGHT=20 RTAMD_STAGGER_US=0
run if20_none RTAMD_INFLIGHT=20 RTAMD_XCHG_OVERLAP=0 RTAMD_STAGGER_US=0
run if19_base RTAMD_INFLIGHT=19
run if16_nooverlap RTAMD_INFLIGHT=16 RTAMD_XCHG_OVERLAP=0
run if20_timing RTAMD_INFLIGHT=20 RTAMD_TIMING=1
grep -i "rt_renderer run" $OUT/if20_timing.err | tail -3
