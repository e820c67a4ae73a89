#!/bin/bash
# Round measurement on the GPU box, in two parts (each GPU step under its own time limit; stops at
# the first failure).  Outputs under gpurun_out/TAG/; copy what is judged into profiles/rNN/.
#   part A: GPU test suite, smoke(), PMC passes of one profiled teapot pass (traffic -> summarised into
#           profiles/pmc_traffic.json, which the bench reads for roofline.traffic; stall -> instruction
#           counts in profiles/pmc_issue.json, read for roofline.valu; the same two over the driver's 20
#           concurrent passes, keyed "... | timed 20 passes", read for the roofline headline; trace), the
#           headline bench line, the driver-style --steps 20 line, rocprofv3 kernel-trace summary.
#   part B: bench lines of the other BASELINE configs, the strong-scaling probe, REPORT.pdf Table 1
#           (their PMC records come from tools/pmc_configs.sh, run before part B).
# usage: tools/round_measure.sh TAG A|B
TAG=$1; PART=$2
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
REV=$(cat .rev 2>/dev/null || echo unknown)
step() { echo "== $* $(date +%T)"; }
if [ "$PART" = A ]; then
  step tests
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  step pmc traffic
  bash tools/pmc.sh ${TAG}_tf tools/pmc_groups/traffic.txt > $OUT/pmc_tf.log 2>&1 || { cat $OUT/pmc_tf.log; exit 1; }
  python3 tools/pmc_summary.py ${TAG}_tf --json profiles/pmc_traffic.json \
      --workload "teapot.scene 1920x1080 2048spp 16 bounces sort=on" \
      --run "rev $REV: python3 bench.py --steps 1 --warmup 0 --no-extras (tools/pmc.sh ${TAG}_tf)" > $OUT/pmc_summary_teapot.txt || exit 1
  cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
  step pmc stall + trace
  bash tools/pmc.sh ${TAG}_st tools/pmc_groups/stall.txt > $OUT/pmc_st.log 2>&1 || { cat $OUT/pmc_st.log; exit 1; }
  python3 tools/stall_summary.py ${TAG}_st --json profiles/pmc_issue.json \
      --workload "teapot.scene 1920x1080 2048spp 16 bounces sort=on" \
      --run "rev $REV: python3 bench.py --steps 1 --warmup 0 --no-extras (tools/pmc.sh ${TAG}_st)" > $OUT/pmc_stall_teapot.txt || exit 1
  cp profiles/pmc_issue.json $OUT/pmc_issue.json
  step pmc of the timed regime, 20 concurrent passes
  W20="teapot.scene 1920x1080 2048spp 16 bounces sort=on | timed 20 passes"
  bash tools/pmc.sh ${TAG}_t20st tools/pmc_groups/stall.txt --steps 20 > $OUT/pmc_t20st.log 2>&1 || { cat $OUT/pmc_t20st.log; exit 1; }
  python3 tools/stall_summary.py ${TAG}_t20st --json profiles/pmc_issue.json --workload "$W20" \
      --run "rev $REV: python3 bench.py --steps 20 --warmup 0 --no-extras (tools/pmc.sh ${TAG}_t20st)" > $OUT/pmc_stall_t20.txt || exit 1
  bash tools/pmc.sh ${TAG}_t20tf tools/pmc_groups/traffic.txt --steps 20 > $OUT/pmc_t20tf.log 2>&1 || { cat $OUT/pmc_t20tf.log; exit 1; }
  python3 tools/pmc_summary.py ${TAG}_t20tf --json profiles/pmc_traffic.json --workload "$W20" \
      --run "rev $REV: python3 bench.py --steps 20 --warmup 0 --no-extras (tools/pmc.sh ${TAG}_t20tf)" > /dev/null || exit 1
  cp profiles/pmc_issue.json profiles/pmc_traffic.json $OUT/
  bash tools/pmc.sh ${TAG}_tr tools/pmc_groups/trace.txt > $OUT/pmc_trc.log 2>&1 || { cat $OUT/pmc_trc.log; exit 1; }
  python3 tools/pmc_summary.py ${TAG}_tr > $OUT/pmc_trace_teapot.txt || exit 1
  step bench teapot
  timeout -k 10 400 python bench.py > $OUT/bench_teapot.json 2> $OUT/bench_teapot.err || { tail $OUT/bench_teapot.err; exit 1; }
  cut -c1-300 $OUT/bench_teapot.json
  step bench teapot driver-style
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_teapot_steps20.json 2> $OUT/bench_teapot_steps20.err || { tail $OUT/bench_teapot_steps20.err; exit 1; }
  step rocprof kernel trace
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-counters > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
  python3 tools/trace_summary.py trace $OUT/prof/run_kernel_trace.csv > $OUT/kernel_trace_summary_teapot.txt || exit 1
else
  for cfg in cornell_plus spheres lamp teapot:--no-sort lamp:--no-sort cornell; do
    args=$(echo $cfg | tr ':' ' '); name=$(echo $cfg | tr -d ':-'); step bench $args
    timeout -k 10 400 python bench.py --scene $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail $OUT/bench_$name.err; exit 1; }
  done
  step strong-scaling probe
  bash tools/scaling_probe.sh $TAG/scaling > $OUT/scaling_probe.log 2>&1 || { cat $OUT/scaling_probe.log; exit 1; }
  cat $OUT/scaling_probe.log
  step table1
  RTAMD_TIMING=1 bash tools/table1.sh $OUT/table1.txt > /dev/null || exit 1
fi
echo done
