# Round 3: the staggered start limited to renders that fill every pass context: short configs and teapot
export TMPDIR=/tmp
OUT=gpurun_out/r3_cfgstag2
mkdir -p $OUT
AB_ARGS="--no-extras --scene cornell_plus" timeout -k 10 600 python tools/ab.py 3 default@RTAMD_STAGGER_US=0 default > $OUT/ab_cornell_plus.txt 2>&1; tail -3 $OUT/ab_cornell_plus.txt
AB_ARGS="--no-extras --scene cornell" timeout -k 10 600 python tools/ab.py 3 default@RTAMD_STAGGER_US=0 default > $OUT/ab_cornell.txt 2>&1; tail -3 $OUT/ab_cornell.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 600 python tools/ab.py 3 default@RTAMD_STAGGER_US=0 default > $OUT/ab_20.txt 2>&1; tail -3 $OUT/ab_20.txt
echo done
