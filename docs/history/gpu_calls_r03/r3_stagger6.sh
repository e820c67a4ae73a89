# Round 3: stagger shape sweep around g=4, delta=3 ms
export TMPDIR=/tmp
OUT=gpurun_out/r3_stagger6
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 1150 python tools/ab.py 6 default default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=3000 default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=4000 default@RTAMD_STAGGER_GROUP=6,RTAMD_STAGGER_US=3000 default@RTAMD_STAGGER_GROUP=2,RTAMD_STAGGER_US=3000 > $OUT/ab_20.txt 2>&1; tail -6 $OUT/ab_20.txt
echo done
