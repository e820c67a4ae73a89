#!/bin/bash
# Round 6, call A: the new GPU tests first (rt_multi, bench --gpus 2 without torchrun, the C++ ABI host), then
# the whole GPU suite, then the driver-style bench line.
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi_renderer.py tests/test_gpu_abi_host.py -m gpu -x -v -s \
  --timeout 240 --timeout-method thread > $O/new_tests.log 2>&1 || { tail -40 $O/new_tests.log; exit 1; }
grep -E "passed|failed|ms_per_pass|value" $O/new_tests.log | tail -8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || { tail $O/bench_steps20.err; exit 1; }
cut -c1-400 $O/bench_steps20.json
