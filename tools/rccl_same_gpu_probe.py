"""Probe: can two processes on ONE GPU join one RCCL communicator (rt_renderer_set_exchange_rccl)
and render pixel tiles with sort on through the library's in-place ncclAllReduce?  Prints the
outcome; exit 0 if the owners' images add up to the oracle's render bit for bit."""
import multiprocessing as mp
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "cuda-raytracer_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "tools")]
IMAGE = (48, 30, 45, 8)
SCENE = os.path.join(REPO, "assets", "teapot.scene")


def owner(rank, owners, q_id, q_out):
    try:
        os.environ.setdefault("NCCL_DEBUG", "WARN")
        import numpy as np
        import rtamd as R
        sc = R.Scene(SCENE, image=IMAGE)
        r = R.Renderer(sc, sort=True, tiles=(owners, rank, 4))
        if rank == 0:
            uid = R.rccl_unique_id()
            for _ in range(owners - 1):
                q_id.put(uid)
        else:
            uid = q_id.get(timeout=60)
        r.set_exchange_rccl(uid, owners, rank)
        st = r.run(0, -1)
        q_out.put((rank, r.framebuffer().tobytes(), st["live_segments"], None))
        r.close()
    except Exception:
        q_out.put((rank, None, 0, traceback.format_exc()))


def main():
    owners = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    q_id, q_out = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=owner, args=(k, owners, q_id, q_out)) for k in range(owners)]
    for p in ps:
        p.start()
    res = [q_out.get(timeout=240) for _ in range(owners)]
    for p in ps:
        p.join(timeout=60)
    errs = [r for r in res if r[3]]
    if errs:
        for r in errs:
            print("rank %d failed:\n%s" % (r[0], r[3]))
        sys.exit(1)
    import numpy as np
    import oracle_lib as O
    fb = sum(np.frombuffer(r[1], np.float32) for r in res)
    ref, rst = O.OracleScene(SCENE, image=IMAGE).render(sort=True)
    ok = np.array_equal(fb, ref) and sum(r[2] for r in res) == rst["live_segments"]
    print("rccl same-gpu tiles (%d owners): %s" % (owners, "bit-exact" if ok else "MISMATCH"))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
