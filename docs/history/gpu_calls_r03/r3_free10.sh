# Round 3: order-free trace: leaf fill while descending, masked record loads at 7 waves
export TMPDIR=/tmp
OUT=gpurun_out/r3_free10
mkdir -p $OUT
AB_ARGS="--no-extras" timeout -k 10 700 python tools/ab.py 2 default@RTAMD_EXACT_TRACE=1 default fill m7 > $OUT/ab_frame.txt 2>&1; tail -5 $OUT/ab_frame.txt
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/fillprof/librtamd.so timeout -k 10 300 python bench.py --no-extras > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep -E "RT_FPROFILE" $OUT/prof.err | tail -2
echo done
