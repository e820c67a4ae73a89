# Round 3: stagger shape, final candidates against the current default; frame, lamp and dist checks
export TMPDIR=/tmp
OUT=gpurun_out/r3_stagger8
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 1000 python tools/ab.py 6 default default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=4000 default@RTAMD_STAGGER_GROUP=6,RTAMD_STAGGER_US=3000 default@RTAMD_STAGGER_GROUP=6,RTAMD_STAGGER_US=4000 > $OUT/ab_20.txt 2>&1; tail -5 $OUT/ab_20.txt
AB_ARGS="--no-extras --steps 20 --warmup 5 --dist" timeout -k 10 600 python tools/ab.py 4 default default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=4000 default@RTAMD_STAGGER_GROUP=6,RTAMD_STAGGER_US=3000 > $OUT/ab_20dist.txt 2>&1; tail -4 $OUT/ab_20dist.txt
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 2 default default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=4000 > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 2 default default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=4000 > $OUT/ab_lamp20.txt 2>&1; tail -3 $OUT/ab_lamp20.txt
echo done
