#!/bin/bash
# Round 6, call P: bounce 0 on camera-relative records -- parity, exclusive launches, 20 steps, full frame.
export TMPDIR=/tmp
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_edge_scenes.py \
  tests/test_gpu_tiles.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 400 python tools/launch_ab.py 3 default nocam > $O/launch_ab.txt 2>&1 || { tail $O/launch_ab.txt; exit 1; }
tail -3 $O/launch_ab.txt
timeout -k 10 600 python tools/ab.py 4 default nocam -- --steps 20 --warmup 5 > $O/ab20.txt 2>&1 || { tail $O/ab20.txt; exit 1; }
tail -3 $O/ab20.txt
timeout -k 10 600 python tools/ab.py 2 default nocam > $O/abfull.txt 2>&1 || { tail $O/abfull.txt; exit 1; }
tail -3 $O/abfull.txt
