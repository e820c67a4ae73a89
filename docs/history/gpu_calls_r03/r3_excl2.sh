# Round 3: why the bench's exclusive trace launch (device wall clock) reads 0.75 ms against the profiler's 0.64
# since the root step: both measures of the same launches in one process (tools/excl_probe.py), for the
# default build and the pre-root-step kernel (build_var/head); then the bounce-0 depth-1 step A/B
export TMPDIR=/tmp
OUT=gpurun_out/r3_excl2
mkdir -p $OUT
for v in default head; do
  lib=$PWD/cuda-raytracer_amd/build/librtamd.so; [ $v = head ] && lib=$PWD/cuda-raytracer_amd/build_var/head/librtamd.so
  RTAMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 tools/excl_probe.py > $OUT/probe_$v.log 2>&1 || { tail $OUT/probe_$v.log; exit 1; }
  grep "events" $OUT/probe_$v.log
  python3 - $OUT/prof_$v/run_kernel_trace.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "trace_kernel" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
for k in range(0, len(d), 16):
    g = d[k:k + 16]
    print("profiler pass %d: %.3f ms over %d launches = %.4f ms/launch" % (k // 16, sum(g), len(g), sum(g) / len(g)))
PY
done
bash tools/gpu_calls/r03/r3_r2f.sh
