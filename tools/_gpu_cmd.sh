export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
RTAMD_LIB=cuda-raytracer_amd/build_var/if1/librtamd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_if1_nosort -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-counters --no-sort > gpurun_out/prof_if1.log 2>&1 || exit 1
timeout -k 10 600 python tools/ab.py 2 default prev -- --steps 48 --warmup 4 --no-sort
