# Round 4: trace grid floor 10 / 12 % of resident workgroups (15) -- interleaved A/B, full frame and 20 steps, teapot and lamp
export TMPDIR=/tmp
OUT=gpurun_out/r4_knob3
mkdir -p $OUT
timeout -k 10 500 python tools/ab.py 4 default occ10 occ12 > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -4 $OUT/ab_frame.txt
timeout -k 10 500 python tools/ab.py 4 default occ10 occ12 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -4 $OUT/ab_steps20.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 2 default occ10 occ12 > $OUT/ab_lamp.txt 2>&1 || { tail -20 $OUT/ab_lamp.txt; exit 1; }
tail -4 $OUT/ab_lamp.txt
echo done
