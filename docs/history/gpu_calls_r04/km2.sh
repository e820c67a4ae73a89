# Round 4: leaf lanes without the child-ref load (RT_KIDS_MASK=1, build_var/km1) against the default:
# driver-style 20 steps (5 rounds), teapot full frame and lamp full frame (3 rounds each)
export TMPDIR=/tmp
OUT=gpurun_out/r4_km2
mkdir -p $OUT
timeout -k 10 600 python tools/ab.py 5 default km1 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -3 $OUT/ab_steps20.txt
timeout -k 10 400 python tools/ab.py 3 default km1 > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --scene lamp" timeout -k 10 500 python tools/ab.py 3 default km1 > $OUT/ab_lamp.txt 2>&1 || { tail -20 $OUT/ab_lamp.txt; exit 1; }
tail -3 $OUT/ab_lamp.txt
echo done
