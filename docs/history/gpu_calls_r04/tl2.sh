# Round 4: device-clock timeline of the driver-style 20-pass batch without a profiler (RTAMD_TIMELINE:
# every pass's trace launch spans from the event-timed re-run of the timed steps)
export TMPDIR=/tmp
OUT=gpurun_out/r4_tl2
mkdir -p $OUT
for i in 1 2; do
RTAMD_TIMELINE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-counters > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail $OUT/bench_$i.err; exit 1; }
RTAMD_TIMELINE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-counters --dist > $OUT/bench_dist_$i.json 2> $OUT/bench_dist_$i.err || { tail $OUT/bench_dist_$i.err; exit 1; }
done
cut -c1-200 $OUT/bench_1.json
grep -c timeline $OUT/bench_1.err
echo done
