export TMPDIR=/tmp
RTAMD_LIB=cuda-raytracer_amd/build_var/pair/librtamd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trace_rays.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t4.log 2>&1; tail -2 gpurun_out/t4.log
timeout -k 10 700 python tools/ab.py 3 default pair -- --steps 40 > gpurun_out/ab_pair.log 2>&1; tail -3 gpurun_out/ab_pair.log
