export TMPDIR=/tmp
RTAMD_TIMING=1 timeout -k 10 200 python tools/experiments/cli_overhead.py
cd assets && RTAMD_TIMING=1 ../cuda-raytracer_amd/build/raytracing teapot.scene --image 1000 1000 100 10 1 --out /tmp/x.png
