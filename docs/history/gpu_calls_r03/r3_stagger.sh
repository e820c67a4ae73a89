# Round 3: staggered start of the first passes in flight (delay kernel), sweep
export TMPDIR=/tmp
OUT=gpurun_out/r3_stagger
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 800 python tools/ab.py 5 default@RTAMD_STAGGER_US=0 default@RTAMD_STAGGER_US=1000 default default@RTAMD_STAGGER_US=2500 > $OUT/ab_20.txt 2>&1; tail -5 $OUT/ab_20.txt
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 3 default@RTAMD_STAGGER_US=0 default > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 13 --dist" timeout -k 10 500 python tools/ab.py 4 default@RTAMD_STAGGER_US=0 default default@RTAMD_STAGGER_US=2500 > $OUT/ab_13.txt 2>&1; tail -4 $OUT/ab_13.txt
AB_ARGS="--no-extras --scene lamp --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 3 default@RTAMD_STAGGER_US=0 default > $OUT/ab_lamp20.txt 2>&1; tail -3 $OUT/ab_lamp20.txt
echo done
