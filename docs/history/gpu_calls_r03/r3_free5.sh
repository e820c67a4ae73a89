# Round 3: order-free trace on lamp: step composition and kernel split
export TMPDIR=/tmp
OUT=gpurun_out/r3_free5
mkdir -p $OUT
RTAMD_TIMING=1 RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/prof/librtamd.so timeout -k 10 300 python bench.py --no-extras --scene lamp --steps 3 --warmup 1 > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep -E "RT_FPROFILE|re-traced" $OUT/prof.err | tail -3
RTAMD_TIMING=1 RTAMD_EXACT_TRACE=1 RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/prof/librtamd.so timeout -k 10 300 python bench.py --no-extras --scene lamp --steps 3 --warmup 1 > $OUT/prof_exact.json 2> $OUT/prof_exact.err || { tail $OUT/prof_exact.err; exit 1; }
grep -E "RT_PROFILE" $OUT/prof_exact.err | tail -2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-extras --scene lamp --steps 3 --warmup 1 > $OUT/rocprof.log 2>&1 || { tail $OUT/rocprof.log; exit 1; }
echo done
