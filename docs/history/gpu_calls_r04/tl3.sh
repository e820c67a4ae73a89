# Round 4: device-clock pass timelines of lamp's 20-pass batch and of teapot's full frame (next round's planning)
export TMPDIR=/tmp
OUT=gpurun_out/r4_tl3
mkdir -p $OUT
RTAMD_TIMELINE=1 timeout -k 10 300 python3 bench.py --scene lamp --steps 20 --warmup 5 --no-cpu-baseline --no-counters > $OUT/tl_lamp.json 2> $OUT/tl_lamp.err || { tail $OUT/tl_lamp.err; exit 1; }
cut -c1-160 $OUT/tl_lamp.json
RTAMD_TIMELINE=1 timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-counters > $OUT/tl_frame.json 2> $OUT/tl_frame.err || { tail $OUT/tl_frame.err; exit 1; }
cut -c1-160 $OUT/tl_frame.json
echo done
