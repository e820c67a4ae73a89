export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
timeout -k 10 600 python tools/ab.py 2 default prev -- --steps 48 --warmup 4 --no-sort
timeout -k 10 600 python tools/ab.py 1 default prev -- --steps 48 --warmup 4
