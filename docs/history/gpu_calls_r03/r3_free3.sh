# Round 3: order-free trace: step composition per policy, and a policy A/B
export TMPDIR=/tmp
OUT=gpurun_out/r3_free3
mkdir -p $OUT
for v in prof fprof1; do
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so timeout -k 10 200 python bench.py --no-extras > $OUT/$v.json 2> $OUT/$v.err || { tail $OUT/$v.err; exit 1; }
grep RT_FPROFILE $OUT/$v.err | tail -2
done
AB_ARGS="--no-extras" timeout -k 10 700 python tools/ab.py 2 default@RTAMD_EXACT_TRACE=1 default pol32 pol48 pol64 > $OUT/ab_frame.txt 2>&1; tail -6 $OUT/ab_frame.txt
echo done
