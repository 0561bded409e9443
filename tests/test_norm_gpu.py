"""K7-K9 parity on the MI355X against plain PyTorch fp32 references of the same ops.

* K7 GroupNorm: nn.GroupNorm applied to the reference's 5-D (b, c, f, h, w) tensor
  (tuneavideo resnet.py:142,158), on x + temb (resnet.py:149-156) when ``add`` is given, then SiLU.
* K8 LayerNorm: F.layer_norm over channels (attention.py:200-216).
* K9 GEGLU gate: a * F.gelu(g) (diffusers 0.11.1 GEGLU).
Tolerances: fp32 1e-5 relative (max|err| / max|ref|), bf16 1e-2 (one bf16 rounding of the output).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
TOL = {torch.float32: 1e-5, torch.bfloat16: 1e-2}


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _rand(shape, seed, dtype, scale=1.0, offset=0.0):
    g = np.random.default_rng(seed)
    return torch.from_numpy((g.standard_normal(shape) * scale + offset).astype(np.float32)).to(dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,f,C,H,G,add,silu,offset", [
    (2, 3, 320, 16, 32, False, True, 0.0),
    (1, 8, 640, 8, 32, True, True, 3.0),     # large common offset: stability of the merged moments
    (4, 8, 1280, 8, 32, True, False, 0.0),
    (2, 1, 64, 4, 32, False, False, 0.0),    # per-frame norm (Transformer3DModel.norm), 2 channels/group
    (1, 2, 960, 8, 32, False, True, 0.0),    # 30 channels per group: vectors straddle groups
    (1, 2, 2560, 4, 32, True, True, 0.0),    # one row per block iteration
])
def test_group_norm(dtype, B, f, C, H, G, add, silu, offset):
    from vp2p import ops
    x = _rand((B * f, C, H, H), 1, dtype, 1.5, offset)
    w = _rand((C,), 2, dtype, 0.3, 1.0)
    b = _rand((C,), 3, dtype, 0.3)
    t = _rand((B * f, C), 4, dtype, 0.7) if add else None
    xin = x if t is None else (x + t[:, :, None, None])          # rounded to dtype, like torch's add
    x5 = xin.float().reshape(B, f, C, H, H).permute(0, 2, 1, 3, 4)
    ref = F.group_norm(x5, G, w.float(), b.float(), 1e-5)
    if silu:
        ref = F.silu(ref)
    ref = ref.permute(0, 2, 1, 3, 4).reshape(B * f, C, H, H)
    xd = x.cuda().to(memory_format=torch.channels_last)
    out = ops.group_norm(xd, G, w.cuda(), b.cuda(), 1e-5, f, silu=silu, add=None if t is None else t.cuda())
    torch.cuda.synchronize()
    assert out.is_contiguous(memory_format=torch.channels_last)
    assert _rel(out.float(), ref) < TOL[dtype], _rel(out.float(), ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,f,C1,C2,H,add,silu", [
    (2, 8, 320, 320, 16, True, True),       # up block res-64: cat(hidden 320, skip 320), 20 ch/group
    (1, 8, 1280, 640, 8, False, True),      # cat(1280, 640) = 1920: groups of 60 straddle the seam
    (2, 4, 640, 320, 8, True, False),       # 960: groups of 30
    (1, 3, 1280, 1280, 16, True, True),     # large: the finalize + apply_stats path
])
def test_group_norm_two_sources(dtype, B, f, C1, C2, H, add, silu):
    """norm1 of an up-block resnet reads torch.cat([hidden, skip], dim=1) from the two tensors: equal
    bit for bit to the norm of the materialised cat (same per-column reads, same sums)."""
    from vp2p import ops
    x1 = _rand((B * f, C1, H, H), 5, dtype).cuda().to(memory_format=torch.channels_last)
    x2 = _rand((B * f, C2, H, H), 6, dtype, 2.0, 0.5).cuda().to(memory_format=torch.channels_last)
    C = C1 + C2
    w, b = _rand((C,), 7, dtype, 0.3, 1.0).cuda(), _rand((C,), 8, dtype, 0.3).cuda()
    t = _rand((B * f, C), 9, dtype, 0.7).cuda() if add else None
    cat = torch.cat([x1, x2], dim=1).contiguous(memory_format=torch.channels_last)
    ref = ops.group_norm(cat, 32, w, b, 1e-5, f, silu=silu, add=t)
    out = ops.group_norm(x1, 32, w, b, 1e-5, f, silu=silu, add=t, x2=x2)
    torch.cuda.synchronize()
    assert out.shape == cat.shape and out.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(out, ref)


def test_group_norm_partials_merge_across_sets():
    """The frame-sharded form: stats of each frame half computed separately, merged by apply."""
    from vp2p import ops, _lib
    import ctypes
    B, f, C, H, G = 2, 4, 320, 8, 32
    x = _rand((B * f, C, H, H), 5, torch.float32, 1.0, 0.5).cuda().to(memory_format=torch.channels_last)
    ref = ops.group_norm(x, G, None, None, 1e-5, f)
    halves = [x.reshape(B, f, C, H, H)[:, i * 2:(i + 1) * 2].reshape(B * 2, C, H, H).contiguous(
        memory_format=torch.channels_last) for i in range(2)]

    # run stats on both halves, then apply with both partial sets
    lib = _lib.load()
    parts = []
    for hx in halves:
        xm = ops._rows_view(hx)
        a = _lib.GroupNormArgs(ops._ptr(xm), None, ops._ptr(xm), None, None, None, B, 2, H * H, C, G, 1e-5, 0,
                               _lib.F32)
        n = lib.vp2p_group_norm_parts(ctypes.byref(a))
        p = torch.empty(B * n * G * 3, device="cuda")
        a.partials = p.data_ptr()
        assert lib.vp2p_group_norm_stats(ctypes.byref(a), ops._stream()) == 0
        parts.append((a, p))
    allp = torch.cat([p for _, p in parts])
    outs = []
    for hx, (a, _) in zip(halves, parts):
        y = torch.empty_like(hx)
        a.y = ops._rows_view(y).data_ptr()
        assert lib.vp2p_group_norm_apply(ctypes.byref(a), ops._ptr(allp), 2, ops._stream()) == 0
        outs.append(y)
    got = torch.cat([o.reshape(B, 2, C, H, H) for o in outs], 1).reshape(B * f, C, H, H)
    torch.cuda.synchronize()
    assert _rel(got, ref) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,C", [(1000, 320), (777, 640), (300, 1280), (64, 64), (5, 2048)])
def test_layer_norm(dtype, rows, C):
    from vp2p import ops
    x = _rand((rows, C), 6, dtype, 2.0, 1.0)
    w = _rand((C,), 7, dtype, 0.2, 1.0)
    b = _rand((C,), 8, dtype, 0.2)
    ref = F.layer_norm(x.float(), (C,), w.float(), b.float(), 1e-5)
    out = ops.layer_norm(x.cuda(), w.cuda(), b.cuda(), 1e-5)
    torch.cuda.synchronize()
    assert _rel(out.float(), ref) < TOL[dtype] * (3 if dtype == torch.float32 else 1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,C", [(1000, 320), (37, 640), (5, 1280)])
def test_add_layer_norm(dtype, rows, C):
    """Residual add fused into LayerNorm: the sum is bit-equal to torch's dtype add, the
    normalised output matches F.layer_norm of that sum."""
    from vp2p import ops
    h = _rand((rows, C), 10, dtype, 2.0, 1.0)
    x = _rand((rows, C), 11, dtype, 2.0)
    w = _rand((C,), 12, dtype, 0.2, 1.0)
    b = _rand((C,), 13, dtype, 0.2)
    s_ref = h + x                                     # torch: one rounding to the dtype
    ref = F.layer_norm(s_ref.float(), (C,), w.float(), b.float(), 1e-5)
    hd = h.cuda()
    s, y = ops.add_layer_norm(hd, x.cuda(), w.cuda(), b.cuda(), 1e-5)
    torch.cuda.synchronize()
    assert s.data_ptr() == hd.data_ptr()
    assert torch.equal(s.cpu(), s_ref)
    assert _rel(y.float(), ref) < TOL[dtype] * (3 if dtype == torch.float32 else 1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,inner", [(1000, 1280), (33, 2560), (7, 5120)])
def test_geglu(dtype, rows, inner):
    from vp2p import ops
    h = _rand((rows, 2 * inner), 9, dtype, 2.0)
    a, g = h.float().chunk(2, dim=-1)
    ge = F.gelu(g).to(dtype).float()                 # torch rounds the gelu result to the dtype
    ref = a * ge
    out = ops.geglu(h.cuda())
    torch.cuda.synchronize()
    assert out.shape == (rows, inner)
    assert _rel(out.float(), ref) < TOL[dtype], _rel(out.float(), ref)
