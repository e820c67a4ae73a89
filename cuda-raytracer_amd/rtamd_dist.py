"""Multi-GPU pass sharding over torch.distributed (RCCL on ROCm, gloo on CPU for tests).

The render is a sequence of independent 20-spp passes (raytracing.cu:222-254): each pass has
its own generate seed (`remaining`), its own per-bounce process seeds and its own stable
reorder, so a pass renders identically on any GPU.  Rank r renders passes r, r+N, r+2N, ...
(round-robin keeps the load balanced: passes cost the same, except a shorter last pass).

Accumulation is owned per pixel slice: the framebuffer (W*H*3 floats) is cut into N equal
slices and rank j owns slice j.  After a chunk of rounds every rank sends slice j of each of
its pass framebuffers to rank j in one all-to-all (RCCL over xGMI: every link carries 1/N of
the data, nothing converges on one GPU), and each owner adds the pass slices it received in
pass order: fb_j = ((0 + S_0,j) + S_1,j) + ... exactly as one GPU adds whole passes, so the
N-GPU image is bit-identical to the 1-GPU image.  `collect()` gathers the N finished slices to
rank 0 (one framebuffer, 24.9 MB at 1080p).  There is no per-bounce collective.  With an
asynchronous renderer (rtamd.Renderer.run_async) the exchange of each group of rounds overlaps the
rendering of the later ones: torch's stream waits on the renderer's per-pass events only.
"""
from typing import Callable, List, Optional


def pass_schedule(rank: int, world: int, passes: int) -> List[int]:
    """Passes rendered by `rank` (round-robin over `world` ranks)."""
    return list(range(rank, passes, world))


def rounds(world: int, passes: int) -> int:
    return -(-passes // world)


def slice_len(pixels3: int, world: int) -> int:
    """Floats per owner slice (the last slice is padded)."""
    return -(-pixels3 // world)


class PassShardedFrame:
    """Accumulates a frame rendered pass-sharded over the ranks of a process group.

    render_passes(passes, out) must write pass passes[j]'s per-pixel sum (W*H*3 float32) into
    out[j], a 2-D tensor on `device`; handing several passes to one call lets the renderer keep
    several passes in flight (the default chunk is the whole frame, one call per rank).
    After `collect()`, rank 0 holds the accumulated framebuffer in `fb`.
    """

    def __init__(self, dist, torch, pixels3: int, passes: int, device, render_passes: Callable,
                 max_rounds_per_call: Optional[int] = None, async_render=None, exchange_rounds: int = 4):
        self.dist, self.torch = dist, torch
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.pixels3 = pixels3
        self.passes = passes
        self.render_passes = render_passes
        self.chunk = max(1, min(max_rounds_per_call or rounds(self.world, passes), rounds(self.world, passes)))
        self.sl = slice_len(pixels3, self.world)
        f32 = torch.float32
        # pass framebuffers, row stride padded to N slices so a row splits into N equal pieces
        self.buf = torch.zeros((self.chunk, self.world * self.sl), dtype=f32, device=device)
        self.slice = torch.zeros(self.sl, dtype=f32, device=device)   # this rank's owned slice
        # the renderer writes contiguous W*H*3 rows; when N does not divide that, it renders into
        # a staging buffer that is copied into the padded rows
        self.stage = None if self.world * self.sl == pixels3 else \
            torch.zeros((self.chunk, pixels3), dtype=f32, device=device)
        self.fb: Optional[object] = None
        # Overlapped exchange: async_render.start(passes, out) enqueues the passes and returns,
        # async_render.wait(j) makes torch's current stream wait until the j-th of them has written its
        # sums, async_render.finish() waits for the rest.  The slices of every `exchange_rounds` rounds
        # then go to their owners while later passes still render (rtamd.Renderer.run_async /
        # wait_pass / finish); without it, one exchange after the chunk's render call.
        self.async_render = async_render
        self.xrounds = max(1, exchange_rounds)

    def reset(self):
        self.slice.zero_()
        self.fb = None

    def _sync(self):
        if getattr(self.buf, "is_cuda", False):
            self.torch.cuda.current_stream().synchronize()

    def run_rounds(self, k0: int, nrounds: int) -> int:
        """Rounds k0 .. k0+nrounds-1: rank r renders passes r + N*k (those that exist) in one
        renderer call per chunk; the pass slices go to their owners, which add them in pass
        order (with async_render: every `exchange_rounds` rounds, as soon as this rank's passes of
        those rounds are done, while its later passes render).  Returns the number of passes this
        rank rendered."""
        done = 0
        N, sl = self.world, self.sl
        for c0 in range(k0, k0 + nrounds, self.chunk):
            ks = list(range(c0, min(c0 + self.chunk, k0 + nrounds)))
            m = len(ks)
            # this rank's passes of those rounds: a prefix of them (pass rank + N*k exists up to some k),
            # so the j-th of `mine` is round ks[j]'s
            mine = [self.rank + N * k for k in ks if self.rank + N * k < self.passes]
            out = self.buf if self.stage is None else self.stage
            if mine:
                # The renderer writes the pass sums on its own streams, which do not wait for torch's:
                # torch work queued earlier that still reads these buffers (the last chunk's
                # all_to_all send copy, the stage -> buf copy) must finish first.
                self._sync()
                if self.async_render is not None:
                    self.async_render.start(mine, out[:len(mine)])
                else:
                    self.render_passes(mine, out[:len(mine)])
            started = bool(mine) and self.async_render is not None
            try:
                self._exchange(ks, mine, m)
            except BaseException:
                if started:
                    # drain the run even though its stats are lost: the renderer must not be left
                    # with a run pending (every later start() would fail) or with passes still
                    # writing into buf / stage while the caller handles the error
                    try:
                        self.async_render.finish()
                    except Exception:
                        pass
                raise
            if started:
                self.async_render.finish()
            done += len(mine)
        return done

    def _exchange(self, ks, mine, m):
        """The exchange of one chunk: slices of the passes of rounds ks go to their owners, which add
        them in pass order (every `exchange_rounds` rounds with async_render)."""
        N, sl = self.world, self.sl
        step = self.xrounds if self.async_render is not None else m
        for s0 in range(0, m, step):
            s1 = min(s0 + step, m)
            mine_here = [j for j in range(s0, s1) if j < len(mine)]
            if self.async_render is not None:
                for j in mine_here:         # passes in flight finish in any order: wait for each
                    self.async_render.wait(j)
            if mine_here and self.stage is not None:
                self.buf[mine_here[0]:mine_here[-1] + 1, :self.pixels3].copy_(
                    self.stage[mine_here[0]:mine_here[-1] + 1])
            n = s1 - s0
            if N > 1:
                # send[d, j] = slice d of this rank's pass framebuffer of round ks[s0 + j]; every rank
                # issues the same sequence of exchanges (it depends only on m and the step)
                send = self.buf[s0:s1].view(n, N, sl).transpose(0, 1).contiguous()
                recv = self.torch.empty_like(send)
                self.dist.all_to_all_single(recv, send)
            else:
                recv = self.buf[s0:s1].view(1, n, sl)
            for j in range(n):
                for src in range(N):            # pass src + N*k: ascending pass order
                    if src + N * ks[s0 + j] < self.passes:
                        self.slice.add_(recv[src, j])

    def collect(self):
        """Gathers the owned slices to rank 0 (collective); returns rank 0's framebuffer."""
        if self.world > 1:
            parts = [self.torch.empty_like(self.slice) for _ in range(self.world)] if self.rank == 0 else None
            self.dist.gather(self.slice, gather_list=parts, dst=0)
            if self.rank == 0:
                self.fb = self.torch.cat(parts)[:self.pixels3]
        else:
            self.fb = self.slice[:self.pixels3]
        return self.fb

    def run_all(self) -> int:
        n = self.run_rounds(0, rounds(self.world, self.passes))
        self.collect()
        return n


def tile_rows(height: int, world: int, rank: int, rows: int = 8) -> List[int]:
    """Image rows owned by `rank` under pixel-tile sharding: stripes of `rows` rows dealt
    round-robin (rt_opts.tile_*; the image's last stripe may be short)."""
    out: List[int] = []
    for k in range(rank, -(-height // rows), world):
        out.extend(range(k * rows, min((k + 1) * rows, height)))
    return out


class TileShardedFrame:
    """Pixel-tile sharding, exact with sort on and off.

    Every rank renders every pass, but only the rays of its own row stripes (stripes of `rows`
    rows dealt round-robin, so sky rows and geometry rows spread over the ranks), with their
    global ray indices: each of its pixels gets the 1-GPU per-pixel add sequence
    ((0 + S_0) + S_1) + ..., bit for bit.  `render_tile(out)` renders the rank's share of the
    frame and writes the rank's framebuffer (W*H*3 float32, other ranks' rows 0) into `out`.
    `collect()` packs the owned rows and gathers them to rank 0 over RCCL (one gather of the
    framebuffer, 24.9 MB at 1080p); rank 0 puts them back in place.  With sort off there is no
    per-bounce collective.  With sort on the process seeds follow the global post-sort slot
    (raytracing.cu:89): the renderer needs the per-bounce bucket-byte exchange first
    (`join_tile_exchange`, an in-place RCCL all-reduce on the device inside the library; the gloo
    tests use `bucket_exchange` with the oracle's restatement).
    """

    def __init__(self, dist, torch, width: int, height: int, device, render_tile: Callable, rows: int = 8):
        self.dist, self.torch = dist, torch
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.W, self.H = width, height
        self.render_tile = render_tile
        self.rows = [tile_rows(height, self.world, r, rows) for r in range(self.world)]
        self.mine = torch.tensor(self.rows[self.rank], dtype=torch.long, device=device)
        self.maxrows = max(len(r) for r in self.rows)
        f32 = torch.float32
        self.local = torch.zeros((height, width * 3), dtype=f32, device=device)
        self.pack = torch.zeros((self.maxrows, width * 3), dtype=f32, device=device)
        self.fb: Optional[object] = None

    def render(self):
        # the renderer's streams do not wait for torch's: the last collect's index_select of
        # `local` must have read it before the renderer overwrites it
        if getattr(self.local, "is_cuda", False):
            self.torch.cuda.current_stream().synchronize()
        self.render_tile(self.local)

    def collect(self):
        """Gathers every rank's rows to rank 0 (collective); returns rank 0's framebuffer."""
        n = len(self.rows[self.rank])
        if self.world == 1:
            self.fb = self.local.reshape(-1)
            return self.fb
        if n:
            self.pack[:n].copy_(self.local.index_select(0, self.mine))
        parts = [self.torch.empty_like(self.pack) for _ in range(self.world)] if self.rank == 0 else None
        self.dist.gather(self.pack, gather_list=parts, dst=0)
        if self.rank == 0:
            full = self.torch.zeros_like(self.local)
            for r, rows in enumerate(self.rows):
                if rows:
                    idx = self.torch.tensor(rows, dtype=self.torch.long, device=full.device)
                    full.index_copy_(0, idx, parts[r][:len(rows)])
            self.fb = full.reshape(-1)
        return self.fb

    def run_all(self):
        self.render()
        return self.collect()


def join_tile_exchange(dist, renderer, rtamd):
    """Pixel tiles with the reorder on, one process per GPU: the renderer joins an RCCL communicator
    of its own over the process group's ranks (rank 0 makes the id, a torch.distributed broadcast
    hands it to the others) and sums the bucket bytes with an in-place ncclAllReduce on each pass's
    stream (rt_renderer_set_exchange_rccl): no byte leaves the device, no Python per bounce."""
    holder = [rtamd.rccl_unique_id() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(holder, src=0)
    renderer.set_exchange_rccl(holder[0], dist.get_world_size(), dist.get_rank())


def bucket_exchange(dist, torch):
    """The per-bounce exchange of pixel-tile sharding with the reorder on: every
    owner writes bucket + 1 at the global slot of each of its live rays into a zeroed byte array;
    the sum over owners (one all-reduce, uint8: each slot has exactly one owner, so no byte
    exceeds 65) gives every owner the whole bucket array, from which it ranks its own rays.
    Returns exchange(arr): in-place sum of a numpy uint8 array over the process group (host
    memory: the gloo tests of the oracle's restatement; GPU renderers use join_tile_exchange)."""
    def exchange(arr):
        t = torch.from_numpy(arr)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        if t.data_ptr() != arr.ctypes.data:
            arr[:] = t.numpy()
    return exchange
