export TMPDIR=/tmp
timeout -k 10 700 python tools/ab.py 3 default kidsel -- --steps 40 > gpurun_out/ab_kid.log 2>&1; tail -3 gpurun_out/ab_kid.log
