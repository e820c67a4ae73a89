#!/bin/bash
# r05: the remaining dist-path cliff at 20 in flight (framebuffer add chain already off)
export TMPDIR=/tmp
OUT=gpurun_out/r5_q5; mkdir -p $OUT
run() { name=$1; shift
  a=(); e=(); for x in "$@"; do case $x in --*) a+=($x);; *) e+=($x);; esac; done
  env "${e[@]}" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras "${a[@]}" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name',d['ms_per_step'])"
}
run dist20_noov --dist RTAMD_INFLIGHT=20 RTAMD_XCHG_OVERLAP=0
run dist20_nostag --dist RTAMD_INFLIGHT=20 RTAMD_STAGGER_US=0
run dist18_18 --dist --steps=18 RTAMD_INFLIGHT=18
run plain18_18 --steps=18 RTAMD_INFLIGHT=18
run dist17_17 --dist --steps=17 RTAMD_INFLIGHT=17
run dist20_20b --dist RTAMD_INFLIGHT=20 NCCL_LAUNCH_MODE=GROUP
run dist20_q8 --dist RTAMD_INFLIGHT=20 RTAMD_HW_QUEUES=8
