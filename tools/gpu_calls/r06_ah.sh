#!/bin/bash
# Round 6, call AH: rt_multi runs of fewer passes than devices (1 and 0) through the loopback transport.
export TMPDIR=/tmp
O=gpurun_out/r06ah; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_multi_renderer.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
