# Round 3: staggered pass starts in a 20-pass batch (host delay per enqueued pass)
export TMPDIR=/tmp
OUT=gpurun_out/r3_enq2
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 800 python tools/ab.py 5 default default@RTAMD_ENQ_DELAY_US=1000 default@RTAMD_ENQ_DELAY_US=2000 default@RTAMD_ENQ_DELAY_US=3000 default@RTAMD_ENQ_DELAY_US=500 > $OUT/ab_20.txt 2>&1; tail -6 $OUT/ab_20.txt
echo done
