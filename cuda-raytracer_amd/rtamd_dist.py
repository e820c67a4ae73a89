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

    render_pass(p, out) must write pass p's per-pixel sum (W*H*3 float32) into `out`, a
    tensor on `device`.  Rank 0 owns the accumulated framebuffer `fb`.
    """

    def __init__(self, dist, torch, pixels3: int, passes: int, device, render_pass: Callable):
        self.dist, self.torch = dist, torch
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.passes = passes
        self.render_pass = render_pass
        f32 = torch.float32
        self.buf = torch.zeros(pixels3, dtype=f32, device=device)
        self.gather = [torch.zeros(pixels3, dtype=f32, device=device) for _ in range(self.world)] \
            if self.rank == 0 else None
        self.fb: Optional[object] = torch.zeros(pixels3, dtype=f32, device=device) if self.rank == 0 else None

    def run_round(self, k: int) -> int:
        """Round k: rank r renders pass r + N*k (if it exists), then the ordered gather.
        Returns the number of passes this rank rendered (0 or 1)."""
        p = self.rank + self.world * k
        mine = p < self.passes
        if mine:
            self.render_pass(p, self.buf)
        else:
            self.buf.zero_()
        if self.world > 1:
            self.dist.gather(self.buf, gather_list=self.gather, dst=0)
        elif self.rank == 0:
            self.gather = [self.buf]
        if self.rank == 0:
            for r in range(self.world):
                if r + self.world * k < self.passes:
                    self.fb.add_(self.gather[r])
        return 1 if mine else 0

    def run_all(self) -> int:
        n = 0
        for k in range(rounds(self.world, self.passes)):
            n += self.run_round(k)
        return n
