#!/bin/bash
# Round 6, call B: two-level trace (trace2_kernel) parity at every bounce, then exclusive per-launch and
# 20-step A/B against the one-level kernel.
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
RTAMD_TRACE2=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trace_rays.py \
  tests/test_gpu_edge_scenes.py tests/test_gpu_baseline_sizes.py tests/test_gpu_bounce0_dielectric.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > $O/trace2_parity.log 2>&1 || { tail -40 $O/trace2_parity.log; exit 1; }
tail -1 $O/trace2_parity.log
timeout -k 10 500 python tools/launch_ab.py 2 default default@RTAMD_TRACE2=0 default@RTAMD_TRACE2=1 default@RTAMD_TRACE2=2 \
  w5@RTAMD_TRACE2=0 w6@RTAMD_TRACE2=0 > $O/launch_ab.txt 2>&1 || { tail -20 $O/launch_ab.txt; exit 1; }
tail -8 $O/launch_ab.txt
timeout -k 10 700 python tools/ab.py 3 default default@RTAMD_TRACE2=1 default@RTAMD_TRACE2=2 w5@RTAMD_TRACE2=1 \
  -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail -20 $O/ab20.txt; exit 1; }
tail -6 $O/ab20.txt
timeout -k 10 500 python tools/ab.py 3 default default@RTAMD_PREFAULT=1 -- --steps 20 --warmup 5 > $O/ab_prefault.txt 2>&1 || { tail -20 $O/ab_prefault.txt; exit 1; }
tail -3 $O/ab_prefault.txt
