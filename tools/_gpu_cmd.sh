export TMPDIR=/tmp
RTAMD_LIB=cuda-raytracer_amd/build_var/wpe8/librtamd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_scenes.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t6.log 2>&1; tail -1 gpurun_out/t6.log
timeout -k 10 900 python tools/ab.py 3 default wpe8 wpe8o35 wpe8o50 -- --steps 40 > gpurun_out/ab_wpe.log 2>&1; tail -5 gpurun_out/ab_wpe.log
