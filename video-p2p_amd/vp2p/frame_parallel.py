"""Frame-sharded (and CFG-split) execution of one clip over G ranks; one process
per GPU.

``EditLayout`` decides the decomposition: with an even G >= 2 the CFG batch is split first (ranks
[0, G/2) run the unconditional half, ranks [G/2, G) the conditional half -- both prompts, so the
P2P source/edit pairing stays rank-local), then frames are sharded over the G/2 ranks of each half
(``FrameShard``).  The halves meet once per denoising step, where the reference combines them
(pipeline_tuneavideo.py:409-411, ``u + g (t - u)``): one 2-rank all-gather of the UNet outputs, plus
a broadcast of the LocalBlend sum from the conditional rank once the blend is active.

Each rank holds frames [rank*f/G, (rank+1)*f/G) of every batch row.  Only three couplings in the
UNet cross frames, and each gets exactly one collective:

=============================  ==========================================  =================================
reference site                 coupling                                    collective
=============================  ==========================================  =================================
attention.py:296-302           FrameAttention reads frame 0's K/V          frame 0's NORMED hidden state
                                                                           (B, N, C) from rank 0: scatter +
                                                                           all-gather (world >= 4) or
                                                                           broadcast; every rank projects K|V
resnet.py:142,158; unet.py:206 5-D GroupNorm statistics over (c/G, f, h, w) all-gather of the K7 per-chunk
                                                                           (count, mean, M2) partials
attention.py:262-268           attn_temp attends over all f frames         all-to-all frames <-> tokens of
                                                                           the normed hidden state (C per
                                                                           token; q|k|v projected after it)
                                                                           and of the output, in token
                                                                           pieces overlapped with the kernel
=============================  ==========================================  =================================

Backward (the null-text optimisation, run_videop2p.py:580-612, frame-sharded): each collective has
its adjoint -- the frame-0 hidden state's gradient is summed onto rank 0 (all-reduce), the GroupNorm
backward all-gathers its (sum dy, sum dy x^) partials the same way, the all-to-alls swap direction --
and the embedding gradient is all-reduced before the (replicated) Adam step.

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
_LAYOUT: Optional["EditLayout"] = None


def active() -> Optional["FrameShard"]:
    """The frame group of the running edit (None: all frames are local)."""
    return _ACTIVE


def active_layout() -> Optional["EditLayout"]:
    """The full decomposition of the running edit (None: single rank / frames only)."""
    return _LAYOUT


@contextlib.contextmanager
def frame_parallel(shard):
    """Run the enclosed UNet / pipeline calls under ``shard``: a FrameShard, an EditLayout or None."""
    global _ACTIVE, _LAYOUT
    prev = _ACTIVE, _LAYOUT
    if isinstance(shard, EditLayout):
        _ACTIVE, _LAYOUT = shard.frames, shard
    else:
        _ACTIVE, _LAYOUT = shard, None
    try:
        yield shard
    finally:
        _ACTIVE, _LAYOUT = prev


class _Done:
    def wait(self):
        return True


class _Both:
    """wait() on two collective handles (issued in order on the group's stream)."""

    def __init__(self, *works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        return True


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

    def broadcast_async(self, t: torch.Tensor):
        """Start an in-place broadcast of ``t`` from group rank 0; returns a handle whose ``wait()``
        orders the current stream after it (RCCL: the collectives run on their own stream, so work
        enqueued before ``wait()`` overlaps them; gloo staging completes it immediately).

        With 4+ ranks it is a scatter of 1/G slices from rank 0 followed by an in-place all-gather:
        on point-to-point xGMI the root then sends (G-1)/G of the bytes over G-1 links at once instead
        of pushing every byte down one ring, and the all-gather's traffic is spread over all ranks."""
        if self.staged and t.is_cuda:
            self.broadcast_(t)
            return _Done()
        flat = t.view(-1)
        if self.world < 4 or flat.numel() % self.world:
            return dist.broadcast(t, src=self.src0, group=self.group, async_op=True)
        n = flat.numel() // self.world
        mine = flat[self.rank * n:(self.rank + 1) * n]
        # the root already holds its slice in place: its scatter output is a scratch buffer, so no
        # scatter source aliases a destination (the all-gather below is NCCL's in-place form:
        # sendbuff = recvbuff + rank * count)
        out = torch.empty_like(mine) if self.rank == 0 else mine
        w1 = dist.scatter(out, list(flat.split(n)) if self.rank == 0 else None, src=self.src0, group=self.group,
                          async_op=True)
        if self.staged:          # gloo runs async ops on worker threads, unordered: finish the scatter
            w1.wait()
        w2 = dist.all_gather_into_tensor(flat, mine, group=self.group, async_op=True)
        return _Both(w1, w2)     # RCCL: both on the group's stream, in issue order

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

    def _a2a_start(self, out: torch.Tensor, inp: torch.Tensor):
        """Start an all-to-all of ``inp`` (dim 0 = destination rank) into ``out`` (dim 0 = source);
        returns a handle.  RCCL: the exchange runs on the group's stream and ``wait()`` orders the
        current stream after it; gloo (host-staged) completes it here."""
        if self.staged and inp.is_cuda:
            self._all_to_all(out, inp)
            return _Done()
        return dist.all_to_all_single(out, inp, group=self.group, async_op=True)

    def temporal_exchange(self, x: torch.Tensor, batch: int, fn, chunks: int = 1) -> torch.Tensor:
        """attn_temp over sharded frames (attention.py:262-268): ``fn`` maps (batch*f, n, C) -- every
        frame of the clip for n tokens -- to (batch*f, n, Cout), independently per token (the qkv
        projection, the temporal kernel and its P2P edit).  ``x`` is this rank's (batch*fl, N, C)
        frames of the block's normed hidden state; returns this rank's (batch*fl, N, Cout) frames of
        fn's result.

        Only x (C per token) crosses the link, not the projected q|k|v (3C): the projection is per
        token, so it runs after the exchange on the rank's token slice.  The slice is cut into
        ``chunks`` token pieces, each an all-to-all of its own issued up front: piece k+1 moves while
        fn runs on piece k, and piece k's output starts home before piece k+1's fn."""
        G = self.world
        Bfl, N, C = x.shape
        fl = Bfl // batch
        if N % G:
            raise ValueError(f"{N} tokens do not split over {G} ranks")
        Nl = N // G
        if chunks < 1 or Nl % chunks:
            chunks = 1
        Nc = Nl // chunks
        xs = x.reshape(batch, fl, G, Nl, C)
        sends, recvs, works = [], [], []
        for c in range(chunks):
            # to destination j: token piece c of slice j of every local frame, laid out (j, b, fl, Nc, C)
            s = xs[:, :, :, c * Nc:(c + 1) * Nc].permute(2, 0, 1, 3, 4).contiguous()
            r = torch.empty_like(s)                                    # (src, b, fl, Nc, C)
            works.append(self._a2a_start(r, s))
            sends.append(s)
            recvs.append(r)
        out = None
        backs = []
        for c in range(chunks):
            works[c].wait()
            xt = recvs[c].permute(1, 0, 2, 3, 4).reshape(batch * G * fl, Nc, C)     # frames src*fl + i
            y = fn(xt)
            Co = y.shape[-1]
            s = y.reshape(batch, G, fl, Nc, Co).permute(1, 0, 2, 3, 4).contiguous()  # (dst, b, fl, Nc, Co)
            r = torch.empty_like(s)                                                 # (src, b, fl, Nc, Co)
            backs.append((self._a2a_start(r, s), s, r))
            if out is None:
                out = torch.empty(batch, fl, G, Nl, Co, device=x.device, dtype=y.dtype)
        for c, (wk, _, r) in enumerate(backs):
            wk.wait()
            out[:, :, :, c * Nc:(c + 1) * Nc] = r.permute(1, 2, 0, 3, 4)
        del sends
        return out.reshape(batch * fl, N, out.shape[-1])

    def local(self, x: torch.Tensor, dim: int = 2) -> torch.Tensor:
        """This rank's frames of a full-clip tensor (frame axis ``dim``)."""
        fl = self.frames_local(x.shape[dim])
        return x.narrow(dim, self.rank * fl, fl).contiguous()

    def gather(self, x: torch.Tensor, dim: int = 2) -> torch.Tensor:
        """All ranks' frames concatenated along ``dim`` (every rank gets the full clip): one
        all_gather_into_tensor into a rank-major buffer, then one copy into the clip's layout."""
        src = x.detach().cpu().contiguous() if (self.staged and x.is_cuda) else x.contiguous()
        if self.world == 1:
            return src.to(x.device)
        dim = dim % src.dim()
        buf = torch.empty((self.world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        dist.all_gather_into_tensor(buf, src, group=self.group)
        ranks = buf.view((self.world,) + tuple(src.shape))           # (world, *x.shape)
        out = ranks.movedim(0, dim).reshape(src.shape[:dim] + (self.world * src.shape[dim],) + src.shape[dim + 1:])
        return out.to(x.device)

    def all_gather_flat(self, t: torch.Tensor) -> torch.Tensor:
        """Every rank's copy of the 1-D tensor ``t`` concatenated in rank order (on t's device):
        the per-chunk GroupNorm partials (count, mean, M2) of K7, merged by the apply kernel."""
        src = t.detach().cpu() if (self.staged and t.is_cuda) else t
        out = torch.empty(self.world * src.numel(), dtype=src.dtype, device=src.device)
        dist.all_gather_into_tensor(out, src.contiguous(), group=self.group)
        return out.to(t.device)


# -- differentiable exchanges (the frame-sharded null-text backward) -----------------------------------
class _Frame0Hidden(torch.autograd.Function):
    """Forward: rank 0's tensor on every rank (frame 0's normed hidden state, attention.py:296-302).
    Backward: the ranks' gradients summed onto rank 0 (every rank's K|V projection read it)."""

    @staticmethod
    def forward(ctx, x0, shard):
        ctx.shard = shard
        out = x0.detach().clone(memory_format=torch.contiguous_format) if shard.rank == 0 else \
            torch.empty(x0.shape, device=x0.device, dtype=x0.dtype)
        shard.broadcast_async(out).wait()
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        ctx.shard.all_reduce_(g)
        return (g if ctx.shard.rank == 0 else torch.zeros_like(g)), None


class _ToTokens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, shard, batch):
        ctx.shard, ctx.batch = shard, batch
        return shard.to_tokens(x.contiguous(), batch)

    @staticmethod
    def backward(ctx, g):
        return ctx.shard.to_frames(g.contiguous(), ctx.batch), None, None


class _ToFrames(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, shard, batch):
        ctx.shard, ctx.batch = shard, batch
        return shard.to_frames(y.contiguous(), batch)

    @staticmethod
    def backward(ctx, g):
        return ctx.shard.to_tokens(g.contiguous(), ctx.batch), None, None


def frame0_hidden(shard: FrameShard, x0: torch.Tensor) -> torch.Tensor:
    """Rank 0's ``x0`` on every rank; differentiable (gradient all-reduced onto rank 0)."""
    return _Frame0Hidden.apply(x0, shard)


def to_tokens(shard: FrameShard, x: torch.Tensor, batch: int) -> torch.Tensor:
    """Differentiable ``FrameShard.to_tokens`` (its adjoint is ``to_frames``)."""
    return _ToTokens.apply(x, shard, batch)


def to_frames(shard: FrameShard, y: torch.Tensor, batch: int) -> torch.Tensor:
    """Differentiable ``FrameShard.to_frames`` (its adjoint is ``to_tokens``)."""
    return _ToFrames.apply(y, shard, batch)


def _staged_run(group, fn, t: torch.Tensor) -> torch.Tensor:
    if dist.get_backend(group) == "gloo" and t.is_cuda:
        h = t.detach().cpu()
        fn(h)
        t.copy_(h)
        return t
    fn(t)
    return t


class EditLayout:
    """CFG split x frame sharding of one clip over all ranks of the default group.

    ``half``: 0 (unconditional rows), 1 (conditional rows) or None (no CFG split: odd world or
    ``cfg_split=False``).  ``frames``: the FrameShard of this rank's half (None when a half is one
    rank).  Every rank creates every subgroup in the same order, as torch.distributed requires."""

    def __init__(self, cfg_split: bool = True):
        if not dist.is_initialized():
            raise RuntimeError("EditLayout needs torch.distributed initialised (one process per GPU)")
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.cfg_split = bool(cfg_split) and self.world >= 2 and self.world % 2 == 0
        halves = 2 if self.cfg_split else 1
        self.frame_world = self.world // halves
        self.half = self.rank // self.frame_world if self.cfg_split else None
        self.frame_rank = self.rank % self.frame_world
        fgroups = ([dist.new_group(list(range(h * self.frame_world, (h + 1) * self.frame_world)))
                    for h in range(halves)] if self.frame_world > 1 else None)
        pgroups = ([dist.new_group([j, j + self.frame_world]) for j in range(self.frame_world)]
                   if self.cfg_split else None)
        self.frames = FrameShard(fgroups[self.half or 0]) if fgroups else None
        self.pair = pgroups[self.frame_rank] if pgroups else None
        self.cond_src = self.frame_rank + self.frame_world       # global rank of this pair's cond half

    def describe(self) -> str:
        parts = []
        if self.cfg_split:
            parts.append("cfg-split x2")
        if self.frame_world > 1:
            parts.append(f"frame-sharded x{self.frame_world}")
        return " x ".join(parts) or "single rank"

    def frames_local(self, frames: int) -> int:
        return self.frames.frames_local(frames) if self.frames is not None else frames

    def local(self, x: torch.Tensor, dim: int = 2) -> torch.Tensor:
        return self.frames.local(x, dim) if self.frames is not None else x

    def batch_rows(self, emb: torch.Tensor) -> torch.Tensor:
        """This rank's rows of the CFG batch [uncond x P, cond x P] (all rows without a CFG split)."""
        if not self.cfg_split:
            return emb
        P = emb.shape[0] // 2
        return emb[self.half * P:(self.half + 1) * P]

    def gather_cfg(self, noise_half: torch.Tensor) -> torch.Tensor:
        """(P, ...) UNet output of this half -> (2P, ...) [uncond, cond], identical on both ranks of
        the pair (pipeline_tuneavideo.py:410 ``noise_pred.chunk(2)``)."""
        if not self.cfg_split:
            return noise_half
        src = noise_half.contiguous()
        staged = dist.get_backend(self.pair) == "gloo" and src.is_cuda
        s = src.cpu() if staged else src
        out = torch.empty((2 * s.shape[0],) + tuple(s.shape[1:]), dtype=s.dtype, device=s.device)
        dist.all_gather_into_tensor(out, s, group=self.pair)
        return out.to(noise_half.device)

    def share_blend(self, acc: Optional[torch.Tensor], shape, device) -> torch.Tensor:
        """The conditional rank's LocalBlend sum, on both ranks of the pair (the unconditional rank
        never accumulates it: the controller only reads conditional maps, run_videop2p.py:217-218)."""
        if not self.cfg_split:
            return acc
        if self.half == 0:
            acc = torch.empty(shape, device=device, dtype=torch.float32)
        buf = acc.contiguous()
        return _staged_run(self.pair, lambda t: dist.broadcast(t, src=self.cond_src, group=self.pair), buf)
