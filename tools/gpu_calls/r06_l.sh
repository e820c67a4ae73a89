#!/bin/bash
# Round 6, call L: concurrent tails vs the number of streams / hardware queues that exist.
export TMPDIR=/tmp
O=gpurun_out/r06l; mkdir -p $O
run() { timeout -k 10 300 env "$@" python tools/tail_probe.py 1 6 >> $O/tail_probe.json 2>> $O/tail_probe.err || { tail $O/tail_probe.err; exit 1; }; }
run PROBE_TAG=inflight20_q24 GPU_MAX_HW_QUEUES=24
run PROBE_TAG=inflight6_q24 RTAMD_INFLIGHT=6 GPU_MAX_HW_QUEUES=24
run PROBE_TAG=inflight6_q8 RTAMD_INFLIGHT=6 GPU_MAX_HW_QUEUES=8
run PROBE_TAG=inflight20_q32 GPU_MAX_HW_QUEUES=32
cut -c1-120 $O/tail_probe.json; python3 -c "
import json
for l in open('$O/tail_probe.json'):
    d=json.loads(l); print(d['tag'], d['passes'], d['kernel_ms'], 'tail_trace', d['pass0_tail_trace_ms'], 'proc', d['process_ms'], 'sort', d['sort_ms'], 'trace', d['trace_ms'])"
