# Round 3: the trace launch's start time published at exit (no start atomic): the whole GPU suite, the probe
# (event timing on vs off, profiler durations), A/B against af1f23b (build_var/prev), the closing teapot lines
export TMPDIR=/tmp
OUT=gpurun_out/r3_tspan
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_probe -o run --output-format csv -- python3 tools/excl_probe.py > $OUT/probe.log 2>&1 || { tail $OUT/probe.log; exit 1; }
grep "events" $OUT/probe.log
python3 - $OUT/prof_probe/run_kernel_trace.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "trace_kernel" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
for k in range(0, len(d), 16):
    g = d[k:k + 16]
    print("profiler pass %d: %.3f ms over %d launches = %.4f ms/launch" % (k // 16, sum(g), len(g), sum(g) / len(g)))
PY
AB_ARGS="--no-extras" timeout -k 10 600 python tools/ab.py 3 prev default > $OUT/ab_frame.txt 2>&1; tail -3 $OUT/ab_frame.txt
AB_ARGS="--no-extras --steps 20 --warmup 5" timeout -k 10 500 python tools/ab.py 3 prev default > $OUT/ab_20.txt 2>&1; tail -3 $OUT/ab_20.txt
timeout -k 10 400 python bench.py > $OUT/bench_teapot.json 2> $OUT/bench_teapot.err || { tail $OUT/bench_teapot.err; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_teapot_steps20.json 2> $OUT/bench_teapot_steps20.err || { tail $OUT/bench_teapot_steps20.err; exit 1; }
for f in bench_teapot bench_teapot_steps20; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],d['bit_exact_vs_oracle'],r['ms_per_launch'],r['pmc_run']['ms_per_launch'])"; done
echo done
