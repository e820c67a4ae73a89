#!/bin/bash
# One GPU iteration: parity tests, bench line, rocprofv3 kernel trace (run on the GPU box).
# usage: tools/gpu_iter.sh TAG [extra bench args]
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { cat gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --no-cpu-baseline --no-counters "$@" > gpurun_out/prof_$TAG.log 2>&1 || exit 1
python3 tools/trace_summary.py trace gpurun_out/prof_$TAG/run_kernel_trace.csv
