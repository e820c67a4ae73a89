# Round 3: order-free trace diagnostics: re-traced rays by cause, kernel split
export TMPDIR=/tmp
OUT=gpurun_out/r3_free2
mkdir -p $OUT
RTAMD_TIMING=1 timeout -k 10 300 python bench.py --no-extras --scene lamp > $OUT/lamp.json 2> $OUT/lamp.err || { tail $OUT/lamp.err; exit 1; }
grep -E "re-traced" $OUT/lamp.err | tail -3
RTAMD_TIMING=1 timeout -k 10 300 python bench.py --no-extras > $OUT/teapot.json 2> $OUT/teapot.err || { tail $OUT/teapot.err; exit 1; }
grep -E "re-traced" $OUT/teapot.err | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-extras > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -12 $OUT/kernel_stats.csv | cut -c1-200
echo done
