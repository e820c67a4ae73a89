# Round 3: per-launch durations of one pass alone, tail traces by trace_kernel vs trace_group_kernel
export TMPDIR=/tmp
OUT=gpurun_out/r3_group2
mkdir -p $OUT
for gb in 0 32768 2000000000; do
RTAMD_GROUP_BELOW=$gb RTAMD_INFLIGHT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/p$gb -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-extras > $OUT/p$gb.log 2>&1 || { tail $OUT/p$gb.log; exit 1; }
done
echo done
