# Round 3: stagger shape, tie-break between g6/3 ms, g4/4 ms and g5/3.5 ms (20-pass batch, 8 rounds)
export TMPDIR=/tmp
OUT=gpurun_out/r3_stagger9
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 1150 python tools/ab.py 8 default@RTAMD_STAGGER_GROUP=6,RTAMD_STAGGER_US=3000 default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=4000 default@RTAMD_STAGGER_GROUP=5,RTAMD_STAGGER_US=3500 > $OUT/ab_20.txt 2>&1; tail -4 $OUT/ab_20.txt
echo done
