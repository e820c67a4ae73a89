# Round 3: stagger shape: the first g passes together, then one every delta
export TMPDIR=/tmp
OUT=gpurun_out/r3_stagger5
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 1100 python tools/ab.py 6 default default@RTAMD_STAGGER_GROUP=4 default@RTAMD_STAGGER_GROUP=8 default@RTAMD_STAGGER_GROUP=4,RTAMD_STAGGER_US=3000 > $OUT/ab_20.txt 2>&1; tail -5 $OUT/ab_20.txt
echo done
