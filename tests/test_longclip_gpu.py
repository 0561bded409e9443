"""configs[4] at its real size on one GPU: the long synthetic clip, 128 frames at 768^2 (latent 96^2).

* K1 (FrameAttention with first-frame K/V, attention.py:296-302) at the three attention levels of
  the 768^2 UNet -- 9216 / 2304 / 576 tokens, head dims 40 / 80 / 160 -- for 128 frames: a sample
  of query rows (every frame band, both token ends, every head) against float64 numpy over ALL keys.
* One Transformer3DModel (attention.py:90-137: GroupNorm, proj_in, attn1 = K1 over 9216 tokens,
  attn2 = K2, GEGLU FF, attn_temp = K3's long-clip kernel over 128 frames, proj_out + residual) at
  C = 320, 128 frames, 96x96, against ``oracle.unet_ref.transformer_token_slice`` in float64 at a
  set of positions (exact: every cross-position coupling of the block is computed in full there;
  the slice oracle is pinned to the reference's Transformer3DModel in test_oracle_models.py).

Tolerances (BASELINE.json north_star): fp32 1e-4, bf16 2e-2, as max|err| / max|ref| over the sample.
"""
import numpy as np
import pytest
import torch

from oracle import unet_ref

pytestmark = pytest.mark.gpu

F_LONG = 128
TOL = {torch.float32: 1e-4, torch.bfloat16: 2e-2}


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n,d", [(9216, 40), (2304, 80), (576, 160)])
def test_frame_attention_long_clip(n, d, dtype):
    from vp2p import ops
    heads, f = 8, F_LONG
    C = heads * d
    g = torch.Generator(device="cuda").manual_seed(n + d)
    q = torch.randn(f, n, C, device="cuda", generator=g).to(dtype)
    k0 = torch.randn(1, n, C, device="cuda", generator=g).to(dtype)
    v0 = torch.randn(1, n, C, device="cuda", generator=g).to(dtype)
    prescaled = dtype == torch.bfloat16            # the production call (FrameAttention.forward)
    c = ops.frame_query_scale(d)
    qk = (q.double() * c).to(dtype) if prescaled else q
    out = ops.frame_attention(qk, k0, v0, f, heads, q_prescaled=prescaled)
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    rng = np.random.default_rng(n)
    frames = np.concatenate([[0, 1, f // 2, f - 1], rng.integers(0, f, 12)])
    toks = np.concatenate([[0, n - 1, n // 2], rng.integers(0, n, 13)])
    qs = (qk.double() / c if prescaled else qk.double())[frames][:, toks].cpu().numpy()   # (F, T, C)
    K = k0[0].double().cpu().numpy().reshape(n, heads, d)
    V = v0[0].double().cpu().numpy().reshape(n, heads, d)
    got = out[frames][:, toks].double().cpu().numpy()
    ref = np.empty_like(got)
    for h in range(heads):
        sl = slice(h * d, (h + 1) * d)
        s = qs[..., sl] @ K[:, h].T * d ** -0.5                  # (F, T, n): every key
        s = np.exp(s - s.max(-1, keepdims=True))
        ref[..., sl] = (s / s.sum(-1, keepdims=True)) @ V[:, h]
    err = _rel(got, ref)
    assert err < TOL[dtype], err


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_transformer3d_long_clip(dtype):
    import model_spec as MS
    from conftest import model_state
    from vp2p.unet3d import Transformer3DModel
    B, f, H, W, C, D = 1, F_LONG, 96, 96, 320, 768
    fac = lambda: Transformer3DModel(MS.HEADS, C // MS.HEADS, C, D)  # noqa: E731
    sd = model_state(fac, 42)
    m = fac()
    m.load_state_dict(sd, strict=True)
    m = m.to("cuda", dtype).to(memory_format=torch.channels_last).eval()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, C, f, H, W, generator=g).to(dtype)
    ctx = torch.randn(B, 77, D, generator=g).to(dtype)
    xb = x.permute(0, 2, 1, 3, 4).reshape(B * f, C, H, W).cuda().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(xb, ctx.cuda(), f)
    torch.cuda.synchronize()
    tokens = [0, 1, W - 1, W, H * W // 2 + 17, H * W - W, H * W - 1] + list(range(4001, 9216, 1013))
    tok = torch.tensor(tokens)
    got = y.reshape(B, f, C, H * W)[..., tok.cuda()].permute(0, 2, 1, 3).double().cpu().numpy()
    # the oracle sees exactly the operands the GPU saw: dtype-rounded input and weights, float64 math
    sd_r = {k: v.to(dtype).double() for k, v in sd.items()}
    ref = unet_ref.transformer_token_slice(sd_r, "", x, ctx.double(), tokens).numpy()
    err = _rel(got, ref)
    assert np.isfinite(got).all() and err < TOL[dtype], err
