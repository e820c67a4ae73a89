# Round 4: kernel timeline of the driver-style 20-pass batch (for the ramp-up / ramp-down occupancy study)
export TMPDIR=/tmp
OUT=gpurun_out/r4_tl1
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extras > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cut -c1-200 $OUT/bench.json
echo done
