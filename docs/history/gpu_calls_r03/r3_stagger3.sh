# Round 3: staggered start sweep (device delay kernel), 20-pass batch
export TMPDIR=/tmp
OUT=gpurun_out/r3_stagger3
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 1100 python tools/ab.py 6 default@RTAMD_STAGGER_US=0 default@RTAMD_STAGGER_US=2000 default@RTAMD_STAGGER_US=3000 default@RTAMD_STAGGER_US=4000 default@RTAMD_STAGGER_US=0,RTAMD_ENQ_DELAY_US=2000 > $OUT/ab_20.txt 2>&1; tail -6 $OUT/ab_20.txt
echo done
