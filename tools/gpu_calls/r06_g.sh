#!/bin/bash
# Round 6, call G: kernel-trace timelines of a 20-pass and a 13-pass batch (ramp shapes), REPORT.pdf Table 1 again.
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extras > $O/p20.log 2>&1 || { tail $O/p20.log; exit 1; }
python3 tools/timeline_occupancy.py $O/p20/run_kernel_trace.csv 20 4 > $O/timeline20.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p13 -o run --output-format csv -- python3 bench.py --steps 13 --warmup 2 --no-extras --dist > $O/p13.log 2>&1 || { tail $O/p13.log; exit 1; }
python3 tools/timeline_occupancy.py $O/p13/run_kernel_trace.csv 13 4 > $O/timeline13.txt || exit 1
rm -rf $O/p20 $O/p13
cat $O/timeline20.txt; cat $O/timeline13.txt
RTAMD_TIMING=1 bash tools/table1.sh $O/table1.txt > /dev/null || exit 1
cat $O/table1.txt
