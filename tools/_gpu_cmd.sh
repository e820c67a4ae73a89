export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
timeout -k 10 600 python tools/ab.py 2 cur_if1 prev_if1 -- --steps 24 --warmup 2
timeout -k 10 600 python tools/ab.py 2 default prev -- --steps 48 --warmup 4
