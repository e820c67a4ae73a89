# Round 4: pass stagger for the driver-style 20-pass batch -- 0 / 1 / 3 ms (default 4) -- interleaved A/B
export TMPDIR=/tmp
OUT=gpurun_out/r4_knob4
mkdir -p $OUT
timeout -k 10 600 python tools/ab.py 5 default default@RTAMD_STAGGER_US=0 default@RTAMD_STAGGER_US=1000 default@RTAMD_STAGGER_US=3000 -- --steps 20 --warmup 5 > $OUT/ab_steps20.txt 2>&1 || { tail -20 $OUT/ab_steps20.txt; exit 1; }
tail -5 $OUT/ab_steps20.txt
echo done
