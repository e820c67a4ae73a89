#!/bin/bash
# r05: passes in flight next to RCCL: the largest count with every pass stream on its own hardware queue
export TMPDIR=/tmp
OUT=gpurun_out/r5_q6; mkdir -p $OUT
run() { name=$1; shift
  a=(); e=(); for x in "$@"; do case $x in --*) a+=($x);; *) e+=($x);; esac; done
  env "${e[@]}" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras "${a[@]}" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name',d['ms_per_step'])"
}
run dist19_19 --dist --steps=19 RTAMD_INFLIGHT=19
run dist17_20 --dist RTAMD_INFLIGHT=17
run dist18_20 --dist RTAMD_INFLIGHT=18
run dist16_20 --dist RTAMD_INFLIGHT=16
run plain20_20
echo "== in-library, 26 and 52 passes"
timeout -k 10 400 python tools/share_probe.py 26 > $OUT/share26.txt 2>&1 || { tail $OUT/share26.txt; exit 1; }
cat $OUT/share26.txt
RTAMD_INFLIGHT=16 timeout -k 10 400 python tools/share_probe.py 26 > $OUT/share26_if16.txt 2>&1 || { tail $OUT/share26_if16.txt; exit 1; }
grep rt_render $OUT/share26_if16.txt
