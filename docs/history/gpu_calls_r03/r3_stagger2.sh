# Round 3: staggered start, host-side enqueue delay vs device-side delay kernel vs none (20-pass batch)
export TMPDIR=/tmp
OUT=gpurun_out/r3_stagger2
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 1000 python tools/ab.py 7 default@RTAMD_STAGGER_US=0 default@RTAMD_STAGGER_US=0,RTAMD_ENQ_DELAY_US=1000 default default@RTAMD_STAGGER_US=0,RTAMD_ENQ_DELAY_US=2000 > $OUT/ab_20.txt 2>&1; tail -5 $OUT/ab_20.txt
echo done
