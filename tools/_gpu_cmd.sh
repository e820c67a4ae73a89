export TMPDIR=/tmp
timeout -k 10 900 python tools/ab.py 2 default lds6 lds12 ch256 ch64 q16 if20 -- --steps 40 > gpurun_out/ab_knobs.log 2>&1; tail -8 gpurun_out/ab_knobs.log
