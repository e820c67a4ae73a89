# Round 3: which rays run long in the order-free kernel (lamp full frame, profiling build)
export TMPDIR=/tmp
OUT=gpurun_out/r3_free8
mkdir -p $OUT
RTAMD_TIMING=1 RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/prof/librtamd.so timeout -k 10 600 python bench.py --no-extras --scene lamp > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep -E "RT_FDEBUG|RT_FPROFILE" $OUT/prof.err | head -24
echo done
