# Round 4: trace knobs re-tuned after the memory-side changes -- refill threshold 16 / 32 idle lanes (24),
# trace grid floor 12 / 20 % of resident workgroups (15) -- interleaved A/B at 20 steps and full frame
export TMPDIR=/tmp
OUT=gpurun_out/r4_knob2
mkdir -p $OUT
timeout -k 10 700 python tools/ab.py 4 default rf16 rf32 occ12 occ20 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -6 $OUT/ab_steps20.txt
timeout -k 10 500 python tools/ab.py 2 default rf16 rf32 occ12 occ20 > $OUT/ab_frame.txt 2>&1 || { tail -20 $OUT/ab_frame.txt; exit 1; }
tail -6 $OUT/ab_frame.txt
echo done
