# Round 3: adaptive reorder tiles + vector framebuffer add (GPU box): parity, A/B vs the previous build
export TMPDIR=/tmp
OUT=gpurun_out/r3_ab4
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-extras" timeout -k 10 500 python tools/ab.py 4 prev default > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 400 python tools/ab.py 4 prev default > $OUT/ab_20.txt 2>&1; tail -3 $OUT/ab_20.txt
AB_ARGS="--no-extras --steps 13 --dist" timeout -k 10 400 python tools/ab.py 4 prev default > $OUT/ab_13dist.txt 2>&1; tail -3 $OUT/ab_13dist.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 400 python tools/ab.py 2 prev default > $OUT/ab_lamp.txt 2>&1; tail -3 $OUT/ab_lamp.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_ramp13 -o run --output-format csv -- python3 bench.py --steps 13 --dist --no-extras > $OUT/prof_ramp13.log 2>&1 || { tail $OUT/prof_ramp13.log; exit 1; }
echo done
