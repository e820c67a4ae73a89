#!/bin/bash
# r05: dist path without the renderer's framebuffer add chain: 20 passes in flight next to RCCL
export TMPDIR=/tmp
OUT=gpurun_out/r5_q4; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_dist_rccl.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() { name=$1; shift
  a=(); e=(); for x in "$@"; do case $x in --*) a+=($x);; *) e+=($x);; esac; done
  env "${e[@]}" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras "${a[@]}" > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name',d['ms_per_step'])"
}
for i in 1 2; do
run dist16_$i --dist
run dist20_$i --dist RTAMD_INFLIGHT=20
run plain20_$i
done
run dist20_q16 --dist RTAMD_INFLIGHT=20 RTAMD_HW_QUEUES=16
run dist20_13 --dist --steps=13 RTAMD_INFLIGHT=20
run dist16_13 --dist --steps=13
timeout -k 10 300 python tools/share_probe.py 13 > $OUT/share13.txt 2>&1 || { tail $OUT/share13.txt; exit 1; }
cat $OUT/share13.txt
