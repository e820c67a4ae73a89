#!/usr/bin/env python3
"""Benchmark of the MI355X path tracer (BASELINE.json metric: Mrays/s per scene at 1/2/4/8 GPUs).

Workload (default): teapot.scene at 1920x1080, 2048 spp, 16 bounces, sort on (BASELINE.json
configs[3], the config the north star's roofline target is stated on).  A step is one 20-spp
pass of the hot path on every GPU: ray generation, 16 x (BVH traversal + shading + reorder
key, stable reorder), ordered accumulation.  Multi-GPU runs shard whole passes round-robin
over ranks (rank r renders pass r + N*k); the pass framebuffers are exchanged as pixel slices
(one RCCL all-to-all: rank j owns slice j and adds the slices in pass order, bit-identical to
1 GPU) and the finished slices are gathered to rank 0.  By default the timed region is one
full frame (strong scaling); `--steps K` times K passes per GPU (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scene teapot] [--no-sort]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  `value` = live ray segments (process_ray calls on live slots)
per second over all GPUs, inputs resident in HBM.  `roofline` prices the dominant kernel
(process_kernel) with SURVEY.md §8(d)'s logical byte model; `cpu_baseline` times the
oracle's restatement of the reference `cpu` path on a bounded sample on the host cores.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
# The renderer keeps up to 20 passes in flight on their own streams; HIP's default of 4 hardware
# queues would make them share queues (20 in flight: 24 queues beat 16 by 1.5 % on teapot, 3.4 %
# on lamp).  With torch.distributed (RCCL) in the process its streams need queues too (16 passes
# and 16 queues cost the 1-GPU --dist run 11 %).  Set before HIP initialises.
_DIST = int(os.environ.get("WORLD_SIZE", "1")) > 1 or "--dist" in sys.argv
_QUEUES = 28 if _DIST else 24
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _QUEUES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_QUEUES)
# Next to RCCL, 16 passes in flight beat 20 (1-GPU --dist: 7.63 vs 7.76 ms/pass for a frame, 8.10
# vs 9.0-12.7 for a 13-pass share); alone, 20 are faster.
if _DIST:
    os.environ.setdefault("RTAMD_INFLIGHT", "16")
sys.path.insert(0, os.path.join(REPO, "cuda-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402

import rtamd  # noqa: E402

CONFIGS = {
    # name: (scene file, W, H, spp, bounces, sort, use_bvh)
    "teapot": ("teapot.scene", 1920, 1080, 2048, 16, True, True),
    "cornell_plus": ("cornell_plus.scene", 512, 512, 256, 8, True, True),
    "spheres": ("spheres.scene", 1024, 1024, 1024, 8, True, False),
    "lamp": ("lamp_available.scene", 1920, 1080, 4096, 32, True, True),
    "cornell": ("cornell.scene", 256, 256, 64, 4, True, True),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
TILE_ROWS = 8          # pixel-tile stripe height (--shard tiles; SURVEY §8e: interleaved 8-row stripes)


def segment_bytes(st, spheres):
    """SURVEY.md §8(d) logical bytes of the process kernel, summed over the counted launches."""
    live = st["live_segments"]
    hits, hs = st["hits"], st["hits_sphere"]
    b = live * (8 + 48 + 48 + 4 + 16 * spheres)
    b += 32 * st["nodes_popped"] + 64 * st["internal_visits"] + 48 * st["triangle_tests"]
    b += hits * (2 + 48) + (hits - hs) * 48 + hs * 16 + st["misses"] * 12
    # §8(d) also charges 8 B per terminated slot; this kernel never touches those slots when the
    # reorder is on (it walks only the live prefix), and reads a 1-B bucket per slot when off.
    b += st.get("dead_slot_bytes", 0)
    return b


def load_pmc(workload):
    """HBM traffic per process_kernel launch from the committed rocprofv3 PMC summary."""
    path = os.path.join(REPO, "profiles", "pmc_process_kernel.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("workload") != workload:
        return None
    return d.get("hbm_bytes_per_launch")


def cpu_baseline(cfg, args):
    """Times the oracle's restatement of cpu_raytrace (raytracing.cu:122-163) on a bounded
    sample of the same scene: full resolution, `--cpu-spp` rays/pixel, same bounces."""
    exe = os.path.join(REPO, "oracle", "build", "cpu_baseline")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    scene, w, h, _, bounces = cfg[:5]
    cmd = [exe, os.path.join(rtamd.ASSETS, scene), rtamd.ASSETS, str(w), str(h), str(args.cpu_spp),
           str(bounces), "1", str(threads)]
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, env=env).stdout
    rec = json.loads(out.strip().splitlines()[-1])
    return {
        "value": round(rec["live_segments"] / rec["seconds"] / 1e6, 3),
        "unit": "Mrays/s",
        "cores": rec["threads"],
        "kind": "port",
        "sample": "%s %dx%d, %d spp (one pass), %d bounces: %d live segments in %.2f s "
                  "(oracle cpu_raytrace restatement, -O3 -ffast-math -fopenmp)" % (
                      scene, w, h, args.cpu_spp, bounces, rec["live_segments"], rec["seconds"]),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="passes per GPU to time (default: one full frame, ceil(passes/N) per GPU)")
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--scene", default="teapot", choices=sorted(CONFIGS))
    ap.add_argument("--no-sort", action="store_true")
    ap.add_argument("--cpu-spp", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-counters", action="store_true", help="skip the byte-model counting rerun")
    ap.add_argument("--dist", action="store_true", help="use the torch.distributed path even at N=1")
    ap.add_argument("--shard", choices=("passes", "tiles"), default="passes",
                    help="multi-GPU decomposition: whole passes per GPU (exact in both sort modes) or "
                         "8-row pixel stripes per GPU over every pass (exact with --no-sort only)")
    ap.add_argument("--tile-share", type=int, default=0, metavar="N",
                    help="1-GPU probe of --shard tiles: render only rank 0's stripes of an N-GPU split")
    args = ap.parse_args()
    # The JSON line is the only thing on stdout: native libraries (RCCL prints a version banner)
    # write to stdout too, so fd 1 is pointed at stderr and the line goes to a saved copy of it.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    torch = None
    use_dist = world > 1 or args.dist
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    cfg = CONFIGS[args.scene]
    scene_file, W, H, spp, bounces, sort, use_bvh = cfg
    if args.no_sort:
        sort = False
    tiles = args.shard == "tiles" or args.tile_share > 1
    if tiles and sort:
        ap.error("--shard tiles needs --no-sort: with the reorder on, process seeds follow the global "
                 "post-sort slot (raytracing.cu:89), which a pixel tile cannot know")
    import make_envmap
    make_envmap.ensure_envmap(os.path.join(REPO, "assets", "teapot", "textures", "envmap.pfm"))
    t_load = time.perf_counter()
    scene = rtamd.Scene(os.path.join(rtamd.ASSETS, scene_file), use_bvh=use_bvh, image=(W, H, spp, bounces))
    load_s = time.perf_counter() - t_load
    P = scene.passes
    tile_split = (args.tile_share, 0) if args.tile_share > 1 else (world, rank)
    ren = rtamd.Renderer(scene, sort=sort, device=local, tiles=tile_split + (TILE_ROWS,) if tiles else None)

    px3 = W * H * 3
    frame = None
    stats_acc = {}

    def accumulate_stats(st):
        for k, v in st.items():
            if isinstance(v, (int, float)):
                stats_acc[k] = stats_acc.get(k, 0) + v

    def render_passes(passes, out):
        # passes are r, r+N, r+2N, ...: one renderer call keeps several of them in flight
        stride = passes[1] - passes[0] if len(passes) > 1 else 1
        accumulate_stats(ren.run(pass_begin=passes[0], count=len(passes), stride=stride,
                                 d_pass_sums=out.data_ptr()))

    # rounds (one pass per GPU each) per frame; pixel tiles: every GPU renders every pass
    R = P if tiles else -(-P // world)
    full_frame = args.steps is None
    steps = R if full_frame else args.steps
    if use_dist:
        import rtamd_dist
        if tiles:
            frame = rtamd_dist.TileShardedFrame(dist, torch, W, H, torch.device("cuda", local),
                                                lambda out: ren.copy_framebuffer(out.data_ptr()), rows=TILE_ROWS)
        else:
            frame = rtamd_dist.PassShardedFrame(dist, torch, px3, P, torch.device("cuda", local), render_passes)

    def barrier_sync():
        if use_dist:
            dist.barrier()
            torch.cuda.synchronize()

    def run_steps(k, stats):
        """k steps from the first pass of the frame, wrapping at its end; one pass per GPU per
        step (rank r renders passes r, r+N, ...).  Returns the passes this rank rendered."""
        stats_acc.clear()
        done = mine = 0
        while done < k:
            m = min(k - done, R)
            if tiles:
                # every pass over this GPU's row stripes, then one RCCL gather of the owned rows
                # to rank 0 (rtamd_dist.TileShardedFrame)
                ren.clear()
                accumulate_stats(ren.run(pass_begin=0, count=m, stride=1))
                if use_dist:
                    frame.run_all()
                mine += m
            elif use_dist:
                # this rank's passes of those rounds in one renderer call, then one RCCL all-to-all
                # of pixel slices to their owners, which add them in pass order, and a gather of the
                # finished slices to rank 0 (rtamd_dist.PassShardedFrame)
                frame.reset()
                mine += frame.run_rounds(0, m)
                frame.collect()
            else:
                accumulate_stats(ren.run(pass_begin=0, count=m, stride=1))
                mine += m
            done += m
        for key, v in stats_acc.items():
            stats[key] = stats.get(key, 0) + v
        return mine

    # No per-bounce HIP events in the timed steps (four marker packets per bounce in every pass's
    # stream cost ~2 %); the kernel-time split comes from an untimed re-run below.
    ren.set_event_timing(False)
    warm = {}
    run_steps(args.warmup, warm)
    barrier_sync()
    timed = {}
    t0 = time.perf_counter()
    my_passes = run_steps(steps, timed)
    barrier_sync()
    elapsed = time.perf_counter() - t0

    live = timed.get("live_segments", 0)
    # Kernel-time split (process / reorder launches, HIP events on each pass's stream): the same
    # steps again, untimed, with events on.
    ren.set_event_timing(True)
    evrun = {}
    run_steps(steps, evrun)
    ren.set_event_timing(False)
    proc_ms = evrun.get("process_ms", 0.0)
    if use_dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        t = torch.tensor([live], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        live = int(t.item())

    # Byte model: recount the timed passes with the counting kernel variant (untimed).
    counted = None
    if not args.no_counters and steps > 0:
        ren.set_counters(True)
        counted = {}
        run_steps(steps, counted)
        counted = {k: int(v) for k, v in counted.items() if isinstance(v, int)}
        counted["dead_slot_bytes"] = 0   # terminated slots are never visited (reorder or live list)
        ren.set_counters(False)
    bytes_total = segment_bytes(counted, scene.view.sphere_count) if counted else 0.0
    launches = my_passes * bounces
    if use_dist:
        t = torch.tensor([bytes_total, launches], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        bytes_total, launches = float(t[0].item()), int(t[1].item())

    if rank == 0:
        workload = "%s %dx%d %dspp %d bounces sort=%s" % (scene_file, W, H, spp, bounces, "on" if sort else "off")
        ms_launch = proc_ms / (my_passes * bounces) if my_passes else 0.0
        roof = None
        if counted:
            bytes_launch = bytes_total / launches
            # Up to 20 passes are in flight, so process launches of different passes overlap and a
            # launch's own duration overstates its share of the GPU: `achieved` is the process
            # kernels' algorithmic bytes over the wall time of the timed steps (conservative: the
            # wall also covers reorder/accumulate); the per-launch figure is reported too.
            achieved = bytes_total / elapsed / 1e9 if elapsed > 0 else 0.0
            per_launch = bytes_launch / (ms_launch / 1e3) / 1e9 if ms_launch > 0 else 0.0
            traffic = load_pmc(workload)
            # measured HBM-side bytes (rocprofv3 PMC, per trace+shade launch) over the same launches
            hbm_gbs = traffic * launches / elapsed / 1e9 if traffic and elapsed > 0 else None
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "hbm_measured_gbs": round(hbm_gbs, 1) if hbm_gbs else None,
                    "hbm_measured_frac": round(hbm_gbs / HBM_PEAK_GBS, 4) if hbm_gbs else None,
                    "note": "achieved/frac: SURVEY.md 8(d) logical bytes (every BVH node and triangle fetch counted, "
                            "cache-inclusive) over the render wall; frac > 1 means the traversal working set is "
                            "served by L2/Infinity Cache. traffic: measured L2->fabric bytes per trace+shade launch "
                            "(profiles/pmc_process_kernel.json); hbm_measured_*: that traffic over the same wall",
                    "kernel": "process (trace_kernel + shade_kernel per bounce)",
                    "bytes_per_launch": int(bytes_launch), "ms_per_launch": round(ms_launch, 4),
                    "achieved_per_launch_events": round(per_launch, 1),
                    "per_launch_events_from": "untimed re-run of the timed steps with per-bounce HIP events "
                                              "(the timed steps record none)",
                    "model": "SURVEY.md 8(d): per live segment 108+16S + 32*Pn + 64*Iv + 48*Tt + hit(98|66)/miss(12); "
                             "dead slots: 0 B with sort (never visited), 1 B without; counts from the device "
                             "counters of the same passes; achieved = bytes of all process launches / timed wall"}
        value = live / elapsed / 1e6 if elapsed > 0 else 0.0
        gen = timed.get("generated_rays", 0)
        if use_dist:
            t = torch.tensor([gen], dtype=torch.float64, device="cuda")
            dist.all_reduce(t)
            gen = int(t.item())
        nominal = gen * bounces / elapsed / 1e6 if elapsed > 0 else 0.0
        ms_step = elapsed / steps * 1e3 if steps else 0.0
        out = {
            "metric": "Mrays/s (live ray segments/s, %s)" % args.scene,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if full_frame or tiles else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: reference scene + assets, procedural stand-in env map (assets missing upstream)",
            "config": {
                "workload": workload,
                "step": ("one 20-spp pass (%d rays x %d bounces) over this GPU's %d-row pixel stripes; "
                         "every GPU renders every pass" % (20 * W * H, bounces, TILE_ROWS)) if tiles else
                        ("one 20-spp pass (%d rays x %d bounces) per GPU; pass-sharded over GPUs" % (20 * W * H, bounces)),
                "timed": ("one full frame (%d passes)" % P) if full_frame else ("%d passes per GPU" % steps),
                "parallelism": ("pixel-tile x%d (%d-row stripes) + RCCL gather" % (world, TILE_ROWS) if tiles else
                                "pass-shard x%d + RCCL all-to-all/gather" % world) if world > 1 else "single GPU",
                "nominal_mrays_per_s": round(nominal, 2),
                "render_wall_ms": round(elapsed * 1e3, 1) if full_frame else None,
                "render_wall_ms_projected": round(ms_step * R, 1),
                "passes_per_frame": P,
                "process_ms_per_step": round(proc_ms / max(my_passes, 1), 3),
                "sort_ms_per_step": round(evrun.get("sort_ms", 0.0) / max(my_passes, 1), 3),
                "scene_load_s": round(load_s, 3),
                "bvh_ms": round(scene.bvh_ms, 1),
                **({"tile_share_probe": "rank 0's %d-row stripes of a %d-GPU split, on one GPU"
                    % (TILE_ROWS, args.tile_share)} if args.tile_share > 1 else {}),
            },
            "roofline": roof,
            "cpu_baseline": None,
        }
        if counted:
            out["config"]["counters"] = {k: counted[k] for k in ("live_segments", "nodes_popped", "internal_visits",
                                                                 "triangle_tests", "hits", "misses", "dead_slots")}
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(cfg, args)
            except Exception as e:  # reported, never fatal for the GPU numbers
                out["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(out), file=json_out, flush=True)
    ren.close()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
