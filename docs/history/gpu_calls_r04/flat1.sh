# Round 4: node step and pop loop with the rare cases (overflow push, big leaf) behind wave-uniform
# tests (RT_NODE_FLAT / RT_POP_FLAT, default on; nf0 = both off = the previous kernel, pf0 = pop off):
# the GPU suite at the new default, interleaved A/B at 20 steps, full frame, lamp
export TMPDIR=/tmp
OUT=gpurun_out/r4_flat1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python tools/ab.py 5 default nf0 pf0 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -4 $OUT/ab_steps20.txt
timeout -k 10 400 python tools/ab.py 3 default nf0 pf0 > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -4 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 3 default nf0 pf0 -- --steps 20 --warmup 5 > $OUT/ab_lamp.txt 2>&1 || { tail -20 $OUT/ab_lamp.txt; exit 1; }
tail -4 $OUT/ab_lamp.txt
echo done
