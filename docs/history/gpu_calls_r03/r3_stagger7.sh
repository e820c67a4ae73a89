# Round 3: stagger shape sweep, second pass
export TMPDIR=/tmp
OUT=gpurun_out/r3_stagger7
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 1150 python tools/ab.py 6 default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=4000 default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=5000 default@RTAMD_STAGGER_GROUP=6,RTAMD_STAGGER_US=4000 default@RTAMD_STAGGER_GROUP=8,RTAMD_STAGGER_US=4000 default@RTAMD_STAGGER_GROUP=6,RTAMD_STAGGER_US=5000 > $OUT/ab_20.txt 2>&1; tail -6 $OUT/ab_20.txt
echo done
