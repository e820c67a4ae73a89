export TMPDIR=/tmp
for q in 16 24 32; do
  for m in "--dist" ""; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-counters --no-cpu-baseline $m > gpurun_out/q.json 2> gpurun_out/q.err || { tail gpurun_out/q.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/q.json'));print('queues $q', '$m', d['ms_per_step'])"
  done
done
