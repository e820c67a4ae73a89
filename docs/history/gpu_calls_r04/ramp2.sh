# Round 4: larger trace grids for the first passes of a run while fewer passes share the chip
# (RT_OCC_RAMP, build_var/ramp) -- parity, interleaved A/B at 20 steps, full frame, lamp 20 steps
export TMPDIR=/tmp
OUT=gpurun_out/r4_ramp2
mkdir -p $OUT
RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/ramp/librtamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 200 --timeout-method thread > $OUT/parity_ramp.log 2>&1 || { tail -30 $OUT/parity_ramp.log; exit 1; }
tail -1 $OUT/parity_ramp.log
timeout -k 10 600 python tools/ab.py 5 default ramp -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -3 $OUT/ab_steps20.txt
timeout -k 10 400 python tools/ab.py 3 default ramp > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 3 default ramp -- --steps 20 --warmup 5 > $OUT/ab_lamp.txt 2>&1 || { tail -20 $OUT/ab_lamp.txt; exit 1; }
tail -3 $OUT/ab_lamp.txt
echo done
