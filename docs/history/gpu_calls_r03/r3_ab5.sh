# Round 3: trace record loads from one scalar base (RT_SADDR) and select-based leaf entry (RT_UBIG):
# parity of the combined variant at full size, the traversal profile, interleaved A/B
export TMPDIR=/tmp
OUT=gpurun_out/r3_ab5
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/both/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_both.log 2>&1; rc=$?
tail -2 $OUT/gpu_tests_both.log
[ $rc -eq 0 ] || exit $rc
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/prof/librtamd.so timeout -k 10 200 python bench.py --no-extras > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep RT_PROFILE $OUT/prof.err | tail -2
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 4 default saddr ubig both > $OUT/ab_frame.txt 2>&1; tail -5 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 400 python tools/ab.py 3 default both > $OUT/ab_20.txt 2>&1; tail -3 $OUT/ab_20.txt
echo done
