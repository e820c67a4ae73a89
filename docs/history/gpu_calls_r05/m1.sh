#!/bin/bash
# r05: GPU suite (queue-sharing test), in-library 13-pass share probe, PMC stall+traffic records at HEAD,
# driver-style bench line with roofline.timed.
export TMPDIR=/tmp
OUT=gpurun_out/r5_m1; mkdir -p $OUT
REV=$(cat .rev 2>/dev/null || echo unknown)
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "== share probe $(date +%T)"
timeout -k 10 300 python tools/share_probe.py 13 > $OUT/share13.txt 2>&1 || { tail $OUT/share13.txt; exit 1; }
cat $OUT/share13.txt
RTAMD_INFLIGHT=16 timeout -k 10 300 python tools/share_probe.py 13 > $OUT/share13_if16.txt 2>&1 || { tail $OUT/share13_if16.txt; exit 1; }
cat $OUT/share13_if16.txt
RTAMD_XCHG_OVERLAP=0 timeout -k 10 300 python tools/share_probe.py 13 > $OUT/share13_sync.txt 2>&1 || { tail $OUT/share13_sync.txt; exit 1; }
grep rt_render $OUT/share13_sync.txt
echo "== pmc $(date +%T)"
W="teapot.scene 1920x1080 2048spp 16 bounces sort=on"
bash tools/pmc.sh r5m1_st tools/pmc_groups/stall.txt > $OUT/pmc_st.log 2>&1 || { cat $OUT/pmc_st.log; exit 1; }
python3 tools/stall_summary.py r5m1_st --json profiles/pmc_issue.json --workload "$W" --run "rev $REV: python3 bench.py --steps 1 --warmup 0 --no-extras (tools/pmc.sh r5m1_st)" > $OUT/pmc_stall_teapot.txt || exit 1
bash tools/pmc.sh r5m1_tf tools/pmc_groups/traffic.txt > $OUT/pmc_tf.log 2>&1 || { cat $OUT/pmc_tf.log; exit 1; }
python3 tools/pmc_summary.py r5m1_tf --json profiles/pmc_traffic.json --workload "$W" --run "rev $REV: python3 bench.py --steps 1 --warmup 0 --no-extras (tools/pmc.sh r5m1_tf)" > $OUT/pmc_summary_teapot.txt || exit 1
cp profiles/pmc_issue.json profiles/pmc_traffic.json $OUT/
echo "== bench $(date +%T)"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_steps20.json 2> $OUT/bench_steps20.err || { tail $OUT/bench_steps20.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_steps20.json'));print(d['value'],d['ms_per_step']);print(json.dumps(d['roofline'].get('timed')));print(json.dumps(d['cpu_baseline']))"
