"""Multi-GPU pass sharding over torch.distributed (RCCL on ROCm, gloo on CPU for tests).

The render is a sequence of independent 20-spp passes (raytracing.cu:222-254): each pass has
its own generate seed (`remaining`), its own per-bounce process seeds and its own stable
reorder, so a pass renders identically on any GPU.  Rank r renders passes r, r+N, r+2N, ...
(round-robin keeps the load balanced: passes cost the same, except a shorter last pass).
After every round of N passes the per-pass framebuffers are gathered to rank 0, which adds them
in pass order: fb = ((0 + S_0) + S_1) + ... exactly as one GPU does, so the N-GPU image is
bit-identical to the 1-GPU image.  This is the only exchange (24.9 MB per pass at 1080p);
there is no per-bounce collective.
"""
from typing import Callable, List, Optional


def pass_schedule(rank: int, world: int, passes: int) -> List[int]:
    """Passes rendered by `rank` (round-robin over `world` ranks)."""
    return list(range(rank, passes, world))


def rounds(world: int, passes: int) -> int:
    return -(-passes // world)


class PassShardedFrame:
    """Accumulates a frame rendered pass-sharded over the ranks of a process group.

    render_passes(passes, out) must write pass passes[j]'s per-pixel sum (W*H*3 float32) into
    out[j], a 2-D tensor on `device`; handing several passes to one call lets the renderer keep
    several passes in flight.  Rank 0 owns the accumulated framebuffer `fb`.
    """

    def __init__(self, dist, torch, pixels3: int, passes: int, device, render_passes: Callable,
                 max_rounds_per_call: int = 8):
        self.dist, self.torch = dist, torch
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.passes = passes
        self.render_passes = render_passes
        self.chunk = max_rounds_per_call
        f32 = torch.float32
        self.buf = torch.zeros((self.chunk, pixels3), dtype=f32, device=device)
        self.gather = [torch.zeros(pixels3, dtype=f32, device=device) for _ in range(self.world)] \
            if self.rank == 0 else None
        self.fb: Optional[object] = torch.zeros(pixels3, dtype=f32, device=device) if self.rank == 0 else None

    def run_rounds(self, k0: int, nrounds: int) -> int:
        """Rounds k0 .. k0+nrounds-1: rank r renders passes r + N*k (those that exist) in one
        renderer call per chunk, then each round is gathered to rank 0 and added in pass order.
        Returns the number of passes this rank rendered."""
        done = 0
        for c0 in range(k0, k0 + nrounds, self.chunk):
            ks = list(range(c0, min(c0 + self.chunk, k0 + nrounds)))
            mine = [self.rank + self.world * k for k in ks if self.rank + self.world * k < self.passes]
            if mine:
                self.render_passes(mine, self.buf[:len(mine)])
            for j, k in enumerate(ks):
                src = self.buf[j] if j < len(mine) else self.buf[-1].zero_()
                if self.world > 1:
                    self.dist.gather(src, gather_list=self.gather, dst=0)
                elif self.rank == 0:
                    self.gather = [src]
                if self.rank == 0:
                    for r in range(self.world):
                        if r + self.world * k < self.passes:
                            self.fb.add_(self.gather[r])
            done += len(mine)
        return done

    def run_round(self, k: int) -> int:
        return self.run_rounds(k, 1)

    def run_all(self) -> int:
        return self.run_rounds(0, rounds(self.world, self.passes))
