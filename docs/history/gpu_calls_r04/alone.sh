# Round 4: the end-of-batch "alone" phase of a 13-pass rank share (tools/ramp_breakdown.py), kernel trace
export TMPDIR=/tmp
OUT=gpurun_out/r4_alone
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 13 --warmup 2 --dist --no-extras > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/ramp_breakdown.py $OUT/prof/run_kernel_trace.csv > $OUT/ramp_breakdown_share13.json || exit 1
python3 -c "import json; d=json.load(open('$OUT/ramp_breakdown_share13.json')); print({k: v for k, v in d.items() if k != 'bounces'})"
echo done
