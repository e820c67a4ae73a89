export TMPDIR=/tmp
for t in 1 4 16; do for sc in teapot lamp_available; do RTAMD_LIB=${LIBV:-cuda-raytracer_amd/build/librtamd.so} RT_BVH_THREADS=$t timeout -k 10 120 python3 -c "
import sys, time; sys.path.insert(0,'cuda-raytracer_amd'); import rtamd as R
best=1e9
for k in range(3):
    s=R.Scene('assets/$sc.scene', quiet=True); best=min(best, s.bvh_ms)
print('threads $t $sc bvh_ms %.1f' % best)
" || exit 1; done; done
LIBV=cuda-raytracer_amd/build_var/prev/librtamd.so; for sc in teapot lamp_available; do RTAMD_LIB=$LIBV timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,\"cuda-raytracer_amd\"); import rtamd as R
print(\"prev $sc bvh_ms %.1f\" % min(R.Scene(\"assets/$sc.scene\").bvh_ms for k in range(3)))
"; done
