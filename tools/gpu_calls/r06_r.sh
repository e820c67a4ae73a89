#!/bin/bash
# Round 6, call R: the new GPU tests (random configs, --inlib), then the whole GPU suite and smoke at HEAD.
export TMPDIR=/tmp
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_random_configs.py tests/test_gpu_multi_renderer.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > $O/new_tests.log 2>&1 || { tail -30 $O/new_tests.log; exit 1; }
tail -1 $O/new_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
