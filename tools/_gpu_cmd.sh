export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bvh_build.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t10.log 2>&1; tail -3 gpurun_out/t10.log
