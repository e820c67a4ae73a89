# Round 4: kernel trace of the driver-style run (20 timed passes after 5 warmup passes) for the ramp analysis
export TMPDIR=/tmp
OUT=gpurun_out/r4_ramp1
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extras > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log | cut -c1-200
echo done
