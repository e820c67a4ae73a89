#!/bin/bash
# r05: in-library multi-device path -- identity exchange at N = 1, one renderer call per share, no per-bounce events;
# parity of the multi tests, the exchange-group timeline of a 13-pass share, then the share probe
export TMPDIR=/tmp
OUT=gpurun_out/r5_mx1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "multi or cli" --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
RTAMD_TIMING=1 GPU_MAX_HW_QUEUES=24 timeout -k 10 200 python -c "
import os, sys
sys.path[:0] = ['cuda-raytracer_amd', 'tools']
import make_envmap, rtamd as R
make_envmap.ensure_envmap('assets/teapot/textures/envmap.pfm')
psc = R.Scene(os.path.join(R.ASSETS, 'teapot.scene'), image=(1920, 1080, 260, 16))
for k in range(3):
    R.render(psc, sort=True, devices=[0])
" > $OUT/timeline.log 2>&1 || { tail $OUT/timeline.log; exit 1; }
grep "rt_multi" $OUT/timeline.log
timeout -k 10 600 python tools/share_probe.py 13 26 52 > $OUT/share_probe.txt 2>&1 || { tail $OUT/share_probe.txt; exit 1; }
cat $OUT/share_probe.txt
