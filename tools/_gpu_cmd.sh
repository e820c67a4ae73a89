export TMPDIR=/tmp
RTAMD_LIB=cuda-raytracer_amd/build_var/tri36/librtamd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_scenes.py tests/test_gpu_trace_rays.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t8.log 2>&1; tail -1 gpurun_out/t8.log
timeout -k 10 900 python tools/ab.py 3 default tri36 -- --steps 40 > gpurun_out/ab_t36.log 2>&1; tail -3 gpurun_out/ab_t36.log
timeout -k 10 900 python tools/ab.py 2 default tri36 -- --scene lamp --steps 40 > gpurun_out/ab_t36l.log 2>&1; tail -3 gpurun_out/ab_t36l.log
