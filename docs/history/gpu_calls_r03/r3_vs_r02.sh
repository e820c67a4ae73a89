# Round 3 against round 2's library (c8df27e) on one box: full frame, driver-style 20 steps, lamp
export TMPDIR=/tmp
OUT=gpurun_out/r3_vs_r02
mkdir -p $OUT
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 700 python tools/ab.py 4 r02 default > $OUT/ab_20.txt 2>&1; tail -3 $OUT/ab_20.txt
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 3 r02 default > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 600 python tools/ab.py 2 r02 default > $OUT/ab_lamp.txt 2>&1; tail -3 $OUT/ab_lamp.txt
AB_ARGS="--no-extras --scene cornell_plus" timeout -k 10 400 python tools/ab.py 3 r02 default > $OUT/ab_cp.txt 2>&1; tail -3 $OUT/ab_cp.txt
echo done
