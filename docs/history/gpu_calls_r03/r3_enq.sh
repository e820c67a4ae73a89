# Round 3: is the host's pass enqueue on the critical path of a 20-pass batch?
export TMPDIR=/tmp
OUT=gpurun_out/r3_enq
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 4 default default@RTAMD_ENQ_DELAY_US=250 default@RTAMD_ENQ_DELAY_US=1000 > $OUT/ab_20.txt 2>&1; tail -4 $OUT/ab_20.txt
RTAMD_TIMING=1 timeout -k 10 200 python bench.py --no-extras --steps 20 --warmup 5 2>&1 >/dev/null | grep enqueued | tail -2
echo done
