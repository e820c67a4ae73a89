# Round 3: trace-step flattening A/B + parity of the candidate + tile-probe kernel profile (GPU box)
export TMPDIR=/tmp
OUT=gpurun_out/r3_ab1
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/popmtd/librtamd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_popmtd.log 2>&1; rc=$?
tail -3 $OUT/gpu_tests_popmtd.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 700 python tools/ab.py 5 default mtflat popmt popmtd > $OUT/ab_frame.txt 2>&1; tail -6 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 5 default popmt popmtd > $OUT/ab_20.txt 2>&1; tail -5 $OUT/ab_20.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_tile_on -o run --output-format csv -- python3 bench.py --tile-share 8 --no-extras --no-cpu-baseline > $OUT/prof_tile_on.log 2>&1 || { tail $OUT/prof_tile_on.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_tile_off -o run --output-format csv -- python3 bench.py --tile-share 8 --no-sort --no-extras --no-cpu-baseline > $OUT/prof_tile_off.log 2>&1 || { tail $OUT/prof_tile_off.log; exit 1; }
echo done
