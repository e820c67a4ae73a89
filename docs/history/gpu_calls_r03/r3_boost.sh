# Round 3: larger trace grid for the first bounces of a staggered batch's first passes
export TMPDIR=/tmp
OUT=gpurun_out/r3_boost
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 900 python tools/ab.py 6 default default@RTAMD_BOOST=1 default@RTAMD_BOOST=2 default@RTAMD_BOOST=4 > $OUT/ab_20.txt 2>&1; tail -5 $OUT/ab_20.txt
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 2 default default@RTAMD_BOOST=1 default@RTAMD_BOOST=2 > $OUT/ab_frame.txt 2>&1; tail -4 $OUT/ab_frame.txt
echo done
