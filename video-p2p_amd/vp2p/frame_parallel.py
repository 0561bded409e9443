"""Frame-sharded execution of one clip over G ranks; one process per GPU.

Each rank holds frames [rank*f/G, (rank+1)*f/G) of every batch row.  Only three couplings in the
UNet cross frames, and each gets exactly one collective:

=============================  ==========================================  ===============================
reference site                 coupling                                    collective
=============================  ==========================================  ===============================
attention.py:296-302           FrameAttention reads frame 0's K/V          broadcast of (B, N, 2C) from rank 0
resnet.py:142,158; unet.py:206 5-D GroupNorm statistics over (c/G, f, h, w) all-reduce of (sum x, sum x^2)
attention.py:262-268           attn_temp attends over all f frames         all-to-all frames <-> tokens,
                                                                           before and after the kernel
=============================  ==========================================  ===============================

Cross-attention, FF, convs, the P2P edit (source/edit pairs are on the same rank), LocalBlend
(strictly per frame, SURVEY finding 6) and the DDIM step stay rank-local.  With the NCCL (RCCL)
backend tensors stay on the device; with gloo (CPU rehearsal / tests) they are staged through host
memory.
"""
from __future__ import annotations

import contextlib
from typing import Optional

import torch
import torch.distributed as dist

_ACTIVE: Optional["FrameShard"] = None


def active() -> Optional["FrameShard"]:
    return _ACTIVE


@contextlib.contextmanager
def frame_parallel(shard: Optional["FrameShard"]):
    global _ACTIVE
    prev, _ACTIVE = _ACTIVE, shard
    try:
        yield shard
    finally:
        _ACTIVE = prev


class FrameShard:
    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("FrameShard needs torch.distributed initialised (one process per GPU)")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.src0 = dist.get_global_rank(group, 0) if group is not None else 0
        self.staged = dist.get_backend(group) == "gloo"

    # -- helpers ------------------------------------------------------------------------------
    def _run(self, fn, t: torch.Tensor) -> torch.Tensor:
        if self.staged and t.is_cuda:
            h = t.detach().cpu()
            fn(h)
            t.copy_(h)
            return t
        fn(t)
        return t

    def frames_local(self, frames: int) -> int:
        if frames % self.world:
            raise ValueError(f"{frames} frames do not split over {self.world} ranks")
        return frames // self.world

    # -- collectives --------------------------------------------------------------------------
    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        return self._run(lambda x: dist.all_reduce(x, group=self.group), t)

    def broadcast_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place broadcast from group rank 0 (the owner of frame 0)."""
        return self._run(lambda x: dist.broadcast(x, src=self.src0, group=self.group), t)

    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor):
        if self.staged and inp.is_cuda:
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, group=self.group)

    def to_tokens(self, x: torch.Tensor, batch: int) -> torch.Tensor:
        """(B*fl, N, C) local frames -> (B*f, N/G, C): all frames of this rank's token slice."""
        G = self.world
        Bfl, N, C = x.shape
        fl = Bfl // batch
        if N % G:
            raise ValueError(f"{N} tokens do not split over {G} ranks")
        Nl = N // G
        # send chunk j = token slice j of every local frame, laid out (j, b, fl, Nl, C)
        send = x.reshape(batch, fl, G, Nl, C).permute(2, 0, 1, 3, 4).contiguous()
        recv = torch.empty_like(send)                       # (src, b, fl, Nl, C)
        self._all_to_all(recv, send)
        return recv.permute(1, 0, 2, 3, 4).reshape(batch * G * fl, Nl, C)

    def to_frames(self, y: torch.Tensor, batch: int) -> torch.Tensor:
        """Inverse of ``to_tokens``: (B*f, N/G, C) -> (B*fl, N, C)."""
        G = self.world
        Bf, Nl, C = y.shape
        fl = Bf // (batch * G)
        send = y.reshape(batch, G, fl, Nl, C).permute(1, 0, 2, 3, 4).contiguous()   # (dst, b, fl, Nl, C)
        recv = torch.empty_like(send)                                              # (src slice, b, fl, Nl, C)
        self._all_to_all(recv, send)
        return recv.permute(1, 2, 0, 3, 4).reshape(batch * fl, G * Nl, C)

    def local(self, x: torch.Tensor, dim: int = 2) -> torch.Tensor:
        """This rank's frames of a full-clip tensor (frame axis ``dim``)."""
        fl = self.frames_local(x.shape[dim])
        return x.narrow(dim, self.rank * fl, fl).contiguous()

    def gather(self, x: torch.Tensor, dim: int = 2) -> torch.Tensor:
        """All ranks' frames concatenated along ``dim`` (every rank gets the full clip)."""
        src = x.detach().cpu().contiguous() if (self.staged and x.is_cuda) else x.contiguous()
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src, group=self.group)
        return torch.cat(parts, dim=dim).to(x.device)

    def all_gather_flat(self, t: torch.Tensor) -> torch.Tensor:
        """Every rank's copy of the 1-D tensor ``t`` concatenated in rank order (on t's device):
        the per-chunk GroupNorm partials (count, mean, M2) of K7, merged by the apply kernel."""
        src = t.detach().cpu() if (self.staged and t.is_cuda) else t
        out = torch.empty(self.world * src.numel(), dtype=src.dtype, device=src.device)
        dist.all_gather_into_tensor(out, src.contiguous(), group=self.group)
        return out.to(t.device)

    def group_norm_stats(self, xv: torch.Tensor, n_local: int):
        """Global (mean, var) per (b, group) of xv (B, L, G, Cg) fp32 summed over dims (1, 3)."""
        s = torch.stack([xv.sum(dim=(1, 3)), (xv * xv).sum(dim=(1, 3))])          # (2, B, G)
        self.all_reduce_(s)
        n = n_local * self.world
        mean = s[0] / n
        var = (s[1] / n - mean * mean).clamp_min_(0.0)
        return mean, var
