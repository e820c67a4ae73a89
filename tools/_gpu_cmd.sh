export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
timeout -k 10 1000 python tools/ab.py 2 default o35 o40i16 o40i8 o40r8 o40r24 -- --steps 48 --warmup 4
