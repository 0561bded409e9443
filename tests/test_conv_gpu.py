"""K10 implicit-GEMM convolution vs an fp32 reference of the same op (F.conv2d in fp32 on the
bf16-rounded inputs, plus the residual), for the conv shapes of the SD-1.5 UNet3D at reduced
spatial size.  Tolerance: bf16 output rounding, 1e-2 of max|ref| (fp32 accumulation inside)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(n, cin, h, w, cout, k, stride, residual, seed=0):
    from vp2p import ops
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, cin, h, w, generator=g).to(torch.bfloat16)
    wt = (torch.randn(cout, cin, k, k, generator=g) * (1.0 / (cin * k * k) ** 0.5)).to(torch.bfloat16)
    b = (torch.randn(cout, generator=g) * 0.1).to(torch.bfloat16)
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = wt.to(DEV).contiguous(memory_format=torch.channels_last)
    bd = b.to(DEV)
    pad = (k - 1) // 2
    ref = F.conv2d(xd.float(), wd.float(), bd.float(), stride, pad)
    res = None
    if residual:
        res = torch.randn(ref.shape, generator=g).to(torch.bfloat16).to(DEV).contiguous(memory_format=torch.channels_last)
        ref = ref.to(torch.bfloat16).float() + res.float()      # the reference rounds conv, then adds
    assert ops.conv2d_supported(xd, wd, stride, pad)
    out = ops.conv2d(xd, wd, bd, stride, pad, residual=res)
    torch.cuda.synchronize()
    assert out.shape == ref.shape and out.is_contiguous(memory_format=torch.channels_last)
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


@pytest.mark.parametrize("n,cin,h,w,cout,k,stride", [
    (2, 320, 16, 16, 320, 3, 1),      # res-64 resnet conv
    (2, 640, 8, 8, 1280, 3, 1),
    (1, 2560, 4, 4, 1280, 3, 1),      # up-block concat input
    (2, 960, 8, 8, 320, 3, 1),
    (3, 320, 7, 9, 640, 3, 1),        # ragged M (189 pixels), odd sizes
    (2, 320, 16, 16, 320, 3, 2),      # Downsample3D
    (2, 640, 9, 11, 640, 3, 2),       # odd input, stride 2
    (2, 960, 8, 8, 320, 1, 1),        # conv_shortcut 1x1
    (1, 2560, 8, 8, 1280, 1, 1),
    (32, 1280, 8, 8, 1280, 3, 1),     # res-8: 128 tiles -> split-K with fp32 workspace
    (32, 2560, 8, 8, 1280, 1, 1),     # split-K, 1x1
])
def test_conv2d(n, cin, h, w, cout, k, stride):
    _case(n, cin, h, w, cout, k, stride, residual=False)


@pytest.mark.parametrize("n,cin,h,w,cout,k,stride,residual", [
    (8, 320, 64, 64, 320, 3, 1, False),      # res-64 resnet conv: 256 tiles of 256 rows
    (33, 320, 31, 33, 320, 3, 1, True),      # ragged last 256-row tile, odd sizes, residual
    (32, 640, 32, 32, 640, 3, 1, False),     # res-32
    (32, 320, 64, 64, 320, 3, 2, False),     # Downsample3D at res-64
    (32, 960, 32, 32, 640, 1, 1, True),      # conv_shortcut 1x1 + residual
    (8, 1920, 64, 64, 320, 3, 1, False),     # up-block concat input, 90 K-steps
    (32, 320, 64, 64, 320, 3, 1, True),      # the edit's res-64 resnet conv (wide tile)
    (16, 640, 32, 32, 640, 3, 1, False),     # res-32, 32-pixel rows
])
def test_conv2d_large_m(n, cin, h, w, cout, k, stride, residual):
    """The 256-row, three-stage LDS-DMA form (conv_kernel_p: >= 256 tiles of 256 rows) against the
    fp32 reference at the UNet's full-size shapes."""
    _case(n, cin, h, w, cout, k, stride, residual=residual, seed=3)


@pytest.mark.parametrize("n,cin,h,w,cout,k,residual", [
    (4, 320, 64, 64, 320, 3, False),         # 1-frame edit (B 4) res-64: 256 128-row tiles -> 512 64-row
    (8, 640, 32, 32, 640, 3, True),          # 2-frame res-32 + residual
    (4, 960, 64, 64, 320, 1, False),         # conv_shortcut 1x1
    (5, 320, 51, 53, 320, 3, True),          # ragged last 64-row tile
    (4, 320, 32, 32, 640, 3, False),         # 256 short tiles on a short K (45 steps)
])
def test_conv2d_short_tile(n, cin, h, w, cout, k, residual):
    """The 64 x 160 tile (small clips whose 128-row grid leaves CUs idle): one pass, no split-K
    workspace, against the fp32 reference."""
    from vp2p import ops, _lib
    import ctypes
    _case(n, cin, h, w, cout, k, 1, residual=residual, seed=4)
    x = torch.empty(n, cin, h, w, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = torch.empty(cout, cin, k, k, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a, _ = ops._conv_args(x, wt, None, None, None, 1, (k - 1) // 2)
    assert _lib.load().vp2p_conv2d_workspace_bytes(ctypes.byref(a)) == 0


@pytest.mark.parametrize("n,cin,h,cout,residual,ksplit", [
    (12, 320, 64, 320, True, 0),        # 3-frame clip res-64: 256 tiles of 192 x 320 (CF 4)
    (12, 960, 64, 320, False, 0),
    (13, 320, 63, 320, True, 0),        # ragged last 192-row tile (not the CF 4 grid: the auto plan)
    (12, 1280, 16, 1280, True, 4),      # res-16, 180 K-steps: 4 slices of 64 192 x 320 tiles
    (12, 2560, 16, 1280, False, 4),
])
def test_conv2d_small_clip_plans(n, cin, h, cout, residual, ksplit):
    """The 3-frame clip's plans (profiles/r06_k10_plan_sweep.jsonl) vs the fp32 reference; the 192 x 320
    tile bit-equal to the 128 x 160 one (VP2P_K10_PLAN, same K order), and forced CF 4 on a ragged M."""
    import ctypes
    import os
    from vp2p import ops, _lib
    _case(n, cin, h, h, cout, 3, 1, residual=residual, seed=9)
    x = torch.randn(n, cin, h, h, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, 3, 3, device=DEV) * 0.02).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = (torch.randn(cout, device=DEV) * 0.1).to(torch.bfloat16)
    a, _ = ops._conv_args(x, wt, None, None, None, 1, 1)
    M = n * h * h
    assert _lib.load().vp2p_conv2d_workspace_bytes(ctypes.byref(a)) == (ksplit * M * cout * 4 if ksplit else 0)
    if ksplit:
        return
    y = ops.conv2d(x, wt, b, 1, 1)
    old = os.environ.get("VP2P_K10_PLAN")
    try:
        for plan in ("0,1", "4,1"):
            os.environ["VP2P_K10_PLAN"] = plan
            assert torch.equal(ops.conv2d(x, wt, b, 1, 1), y), plan
    finally:
        if old is None:
            os.environ.pop("VP2P_K10_PLAN", None)
        else:
            os.environ["VP2P_K10_PLAN"] = old


@pytest.mark.parametrize("k", [1, 3])
def test_conv2d_residual(k):
    _case(2, 640, 8, 8, 640, k, 1, residual=True, seed=1)


def test_conv2d_splitk_residual():
    from vp2p import ops, _lib
    import ctypes
    _case(32, 1280, 8, 8, 1280, 3, 1, residual=True, seed=2)
    x = torch.empty(32, 1280, 8, 8, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.empty(1280, 1280, 3, 3, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a, _ = ops._conv_args(x, w, None, None, None, 1, 1)
    assert _lib.load().vp2p_conv2d_workspace_bytes(ctypes.byref(a)) > 0     # the split path ran


@pytest.mark.parametrize("n,c1,c2,h,cout,residual", [(32, 320, 320, 16, 320, True), (4, 1280, 640, 8, 640, False),
                                                      (2, 640, 1280, 8, 1280, True), (1, 2560, 1280, 4, 1280, False)])
def test_conv2d_two_sources(n, c1, c2, h, cout, residual):
    """conv_shortcut of an up-block resnet on torch.cat([hidden, skip], dim=1) read from the two
    tensors: bit-equal to K10 on the materialised cat (same K-step order), incl. split-K shapes."""
    from vp2p import ops
    g = torch.Generator().manual_seed(11)
    x1 = torch.randn(n, c1, h, h, generator=g).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
    x2 = torch.randn(n, c2, h, h, generator=g).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
    w = (torch.randn(cout, c1 + c2, 1, 1, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    b = (torch.randn(cout, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    r = (torch.randn(n, cout, h, h, generator=g).to(torch.bfloat16).to(DEV).to(memory_format=torch.channels_last)
         if residual else None)
    cat = torch.cat([x1, x2], dim=1).contiguous(memory_format=torch.channels_last)
    assert ops.conv2d_supported(x1, w, 1, 0, x2=x2)
    ref = ops.conv2d(cat, w, b, 1, 0, residual=r)
    out = ops.conv2d(x1, w, b, 1, 0, residual=r, x2=x2)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert not ops.conv2d_supported(x1, torch.randn(cout, c1 + c2, 3, 3, device=DEV, dtype=torch.bfloat16), 1, 1, x2=x2)


def test_conv2d_unsupported_raises():
    from vp2p import ops, _lib
    x = torch.randn(1, 4, 8, 8, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = torch.randn(320, 4, 3, 3, device=DEV, dtype=torch.bfloat16)
    assert not ops.conv2d_supported(x, wt, 1, 1)
    with pytest.raises(_lib.Vp2pError):
        ops.conv2d(x, wt, None, 1, 1)


@pytest.mark.parametrize("M,K,inner", [(1000, 320, 1280), (257, 640, 2560), (64, 1280, 5120), (65536 + 77, 320, 1280),
                                        (1600, 320, 1280)])
def test_linear_geglu(M, K, inner):
    """K10 with the GEGLU epilogue vs F.linear + diffusers GEGLU in fp32 on the same bf16 inputs
    (projection rounded to bf16, gelu rounded, product rounded -- torch's eager roundings)."""
    from vp2p import ops
    g = torch.Generator().manual_seed(5)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(2 * inner, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    b = (torch.randn(2 * inner, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    h = F.linear(x.float(), w.float(), b.float()).to(torch.bfloat16).float()
    a, gt = h.chunk(2, dim=-1)
    ref = a * F.gelu(gt).to(torch.bfloat16).float()
    assert ops.linear_geglu_supported(x, w)
    wi, bi = ops.geglu_interleave(w, b)
    out = ops.linear_geglu(x, wi, bi)
    torch.cuda.synchronize()
    assert out.shape == (M, inner)
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


@pytest.mark.parametrize("n,cin,h,w,cout", [(2, 1280, 8, 8, 1280), (3, 640, 5, 7, 640), (32, 640, 32, 32, 320),
                                          (12, 1280, 8, 8, 1280)])   # 3-frame clip: 4 slices of 192 x 320
def test_conv2d_fused_upsample(n, cin, h, w, cout):
    """K10 reading a x2 nearest upsample on the fly == F.interpolate then the conv (fp32 reference)."""
    from vp2p import ops
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, cin, h, w, generator=g).to(torch.bfloat16).to(DEV).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5).to(torch.bfloat16).to(DEV)
    wt = wt.contiguous(memory_format=torch.channels_last)
    b = (torch.randn(cout, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    ref = F.conv2d(F.interpolate(x.float(), scale_factor=2.0, mode="nearest"), wt.float(), b.float(), 1, 1)
    assert ops.conv2d_supported(x, wt, 1, 1, upsample=True)
    out = ops.conv2d(x, wt, b, 1, 1, upsample=True)
    torch.cuda.synchronize()
    assert out.shape == ref.shape
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


def test_linear_residual():
    from vp2p import ops
    g = torch.Generator().manual_seed(8)
    x = torch.randn(3, 500, 640, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(640, 640, generator=g) / 640 ** 0.5).to(torch.bfloat16).to(DEV)
    b = (torch.randn(640, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    r = torch.randn(3, 500, 640, generator=g).to(torch.bfloat16).to(DEV)
    ref = F.linear(x.float(), w.float(), b.float()).to(torch.bfloat16).float() + r.float()
    assert ops.linear_residual_supported(x, w, r)
    out = ops.linear_residual(x, w, b, r)
    torch.cuda.synchronize()
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


@pytest.mark.parametrize("M,K,N,alpha", [(1000, 320, 320, 1.0), (70000, 320, 960, 1.0), (4100, 1280, 320, 0.2281),
                                         (131072, 320, 320, 0.2281), (777, 640, 640, -3.5), (8192, 1280, 1280, 1.0)])
def test_linear_k10_alpha(M, K, N, alpha):
    """K10 plain projection alpha * (x W^T + b) (every tile the shape picks: wide 256 x 320, 128 x 160,
    split-K) vs the fp32 GEMM on the same bf16 inputs, one rounding."""
    from vp2p import ops
    g = torch.Generator().manual_seed(11)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    ref = alpha * F.linear(x.float(), w.float(), b.float())
    with torch.no_grad():
        assert ops.linear_k10_ok(x, w, b)
        out = ops.linear_k10(x, w, b, alpha)
    torch.cuda.synchronize()
    assert out.shape == (M, N)
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err
    if alpha == 1.0:       # alpha = 1 (and 0 = unset) is bit-equal to the unscaled epilogue
        a2 = ops.linear_k10(x, w, b)
        assert torch.equal(out, a2)


@pytest.mark.parametrize("mode", ["k10", "library"])
def test_attn_temp_residual_on_output_projection(mode):
    """attn_temp(y, residual=x) (the block's last add riding on to_out, attention.py:268) equals
    attn_temp(y) + x on either branch of the per-shape choice."""
    from vp2p import ops
    from vp2p.attention import CrossAttention
    torch.manual_seed(9)
    attn = CrossAttention(320, heads=8, dim_head=40).to(DEV, torch.bfloat16)
    with torch.no_grad():
        attn.to_out[0].weight.normal_(0, 0.05)
        attn.to_out[0].bias.normal_(0, 0.1)
    f = 8
    y = torch.randn(2 * f, 256, 320, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(2 * f, 256, 320, device=DEV, dtype=torch.bfloat16)
    saved_mode, saved_choice = ops.CONV.mode, dict(ops.CONV.choice)
    ops.CONV.mode, ops.CONV.choice = mode, {}
    try:
        with torch.no_grad():
            ref = (attn(y, video_length=f, temporal_layout="bf") + x).float()
            out = attn(y, video_length=f, temporal_layout="bf", residual=x).float()
        torch.cuda.synchronize()
    finally:
        ops.CONV.mode, ops.CONV.choice = saved_mode, saved_choice
    err = (out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err
    if mode == "library":
        assert torch.equal(out, ref)


@pytest.mark.parametrize("n,frames,c,h,cout,groups", [(8, 4, 320, 64, 320, 32), (8, 8, 640, 32, 640, 32),
                                                      (16, 8, 320, 32, 640, 32), (4, 2, 640, 64, 320, 32),
                                                      (12, 3, 320, 64, 320, 32)])     # the 192 x 320 tile
def test_conv2d_gn_stats(n, frames, c, h, cout, groups):
    """conv1 + temb with norm2's statistics left by K10's epilogue (ops.conv2d_gn): the output equals
    the separate conv + add bit for bit (same tile, same two roundings), and the GroupNorm applied
    from the epilogue's partials matches the GroupNorm with its own statistics pass."""
    from vp2p import ops
    g = torch.Generator().manual_seed(12)
    x = torch.randn(n, c, h, h, generator=g).to(torch.bfloat16).to(DEV).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, c, 3, 3, generator=g) / (c * 9) ** 0.5).to(torch.bfloat16).to(DEV)
    w = w.contiguous(memory_format=torch.channels_last)
    b = (torch.randn(cout, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    t = (torch.randn(n, cout, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    gw = (1 + 0.1 * torch.randn(cout, generator=g)).to(torch.bfloat16).to(DEV)
    gb = (0.1 * torch.randn(cout, generator=g)).to(torch.bfloat16).to(DEV)
    with torch.no_grad():
        r = ops.conv2d_gn(x, w, b, 1, 1, t, groups, frames)
        assert r is not None, "fused statistics unsupported for this shape"
        y, stats = r
        ref = (ops.conv2d(x, w, b, 1, 1).float() + t.float()[:, :, None, None]).to(torch.bfloat16)
        assert torch.equal(y, ref)
        got = ops.group_norm_from_partials(y, groups, gw, gb, 1e-5, frames, stats, silu=True)
        want = ops.group_norm(ref.contiguous(memory_format=torch.channels_last), groups, gw, gb, 1e-5, frames, silu=True)
        f32 = torch.nn.functional.group_norm(ref.float().reshape(n // frames, frames, cout, h, h).transpose(1, 2),
                                             groups, gw.float(), gb.float(), 1e-5)
        f32 = torch.nn.functional.silu(f32.transpose(1, 2).reshape(n, cout, h, h))
    torch.cuda.synchronize()
    err = (got.float() - f32).abs().max().item() / f32.abs().max().item()
    assert err < 1e-2, err
    assert (got.float() - want.float()).abs().max().item() <= 2 * (want.float() - f32).abs().max().item() + 1e-3


@pytest.mark.parametrize("n,c,h,cout", [(32, 1280, 8, 1280),     # split-K: the add in the reduce pass
                                         (8, 320, 64, 320),      # one pass
                                         (4, 640, 32, 640)])     # short tile
def test_conv2d_img_add(n, c, h, cout):
    """K10 conv + a per-image vector (ABI 15 img_add: the resnet's h + temb) equals the conv then the
    add, bit for bit (two roundings), on the one-pass, short and split-K forms."""
    from vp2p import ops
    g = torch.Generator().manual_seed(13)
    x = torch.randn(n, c, h, h, generator=g).to(torch.bfloat16).to(DEV).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, c, 3, 3, generator=g) / (c * 9) ** 0.5).to(torch.bfloat16).to(DEV)
    w = w.contiguous(memory_format=torch.channels_last)
    b = (torch.randn(cout, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    t = (torch.randn(n, cout, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    with torch.no_grad():
        y = ops.conv2d(x, w, b, 1, 1, img_add=t)
        ref = (ops.conv2d(x, w, b, 1, 1).float() + t.float()[:, :, None, None]).to(torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("M,epi", [(131072, "plain"), (131072, "alpha"), (131072, "residual"), (131072, "nobias"),
                                   (393216, "residual"), (32768, "plain"), (98336, "residual")])
def test_k10_stream_k320(M, epi):
    """K10s, the persistent stream for the K = N = 320 projections (M / 32 >= 1024 whole 32-row blocks,
    the 64x64-latent transformer blocks at 8 and 24 frames): bit-equal to the tiled kernels, which the
    same rows take in 16384-row chunks (below the stream's threshold), and within bf16 rounding of the
    fp32 GEMM.  M = 98336 is 3073 blocks: a ragged last round of the persistent grid."""
    from vp2p import ops
    g = torch.Generator().manual_seed(21)
    K = N = 320
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    b = None if epi == "nobias" else (torch.randn(N, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    r = torch.randn(M, N, generator=g).to(torch.bfloat16).to(DEV) if epi == "residual" else None
    alpha = 0.2281 if epi == "alpha" else 1.0

    def run(xs, rs):
        if rs is not None:
            return ops.linear_residual(xs, w, b, rs)
        return ops.linear_k10(xs, w, b, alpha)

    with torch.no_grad():
        full = run(x, r)
        tiled = torch.cat([run(x[i:i + 16384], None if r is None else r[i:i + 16384]) for i in range(0, M, 16384)])
    torch.cuda.synchronize()
    assert torch.equal(full, tiled)
    ref = alpha * F.linear(x[:4096].float(), w.float(), None if b is None else b.float())
    if r is not None:
        ref = ref.to(torch.bfloat16).float() + r[:4096].float()
    err = (full[:4096].float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


@pytest.mark.parametrize("M,N,geglu", [(131072, 960, False), (131072, 2560, True), (393216, 2560, True),
                                       (98336, 960, False), (98336, 2560, True)])
def test_k10_stream_k320_groups(M, N, geglu):
    """K10s over N = 320 NG column groups: attn_temp's q|k|v (N 960) and the GEGLU projection (N 2560,
    interleaved weights, the GEGLU epilogue; 8 and 24 frames) -- bit-equal to the tiled kernels on
    16384-row chunks, and within bf16 rounding of the fp32 reference."""
    from vp2p import ops
    g = torch.Generator().manual_seed(22)
    K = 320
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    with torch.no_grad():
        if geglu:
            w_il, b_il = ops.geglu_interleave(w, b)
            run = lambda xs: ops.linear_geglu(xs, w_il, b_il)           # noqa: E731
        else:
            run = lambda xs: ops.linear_k10(xs, w, b)                    # noqa: E731
        full = run(x)
        tiled = torch.cat([run(x[i:i + 16384]) for i in range(0, M, 16384)])
    torch.cuda.synchronize()
    assert torch.equal(full, tiled)
    h = F.linear(x[:4096].float(), w.float(), b.float())
    if geglu:
        v, gt = h.chunk(2, dim=-1)
        ref = v.to(torch.bfloat16).float() * F.gelu(gt.to(torch.bfloat16).float())
    else:
        ref = h
    err = (full[:4096].float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-2, err


