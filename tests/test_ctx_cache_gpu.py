"""The attn2 context K/V (and K2's layout of them) are kept across calls only while the context
tensor is unchanged (vp2p.attention._context_kv, vp2p.unet3d.UNet3DConditionModel._context)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_context_kv_cache_follows_the_context():
    from vp2p.attention import CrossAttention
    torch.manual_seed(0)
    attn = CrossAttention(320, 768, heads=8, dim_head=40).to(DEV, torch.bfloat16).eval()
    x = torch.randn(2 * 4, 256, 320, device=DEV, dtype=torch.bfloat16)      # 2 batch rows x 4 frames
    ctx = torch.randn(2, 77, 768, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        y1 = attn(x, encoder_hidden_states=ctx, video_length=4)
        assert "_ctx_kv" in attn.__dict__
        y2 = attn(x, encoder_hidden_states=ctx, video_length=4)              # served from the cache
        assert torch.equal(y1, y2)
        ctx.mul_(0.5)                                                        # in place: a new version
        y3 = attn(x, encoder_hidden_states=ctx, video_length=4)
        attn.__dict__.pop("_ctx_kv")
        y4 = attn(x, encoder_hidden_states=ctx, video_length=4)              # recomputed from scratch
        assert torch.equal(y3, y4) and not torch.equal(y1, y3)
        other = ctx.clone()                                                  # equal values, new storage
        y5 = attn(x, encoder_hidden_states=other, video_length=4)
        assert torch.equal(y5, y4)
        with torch.no_grad():
            attn.to_k.weight.mul_(2.0)                                       # weights changed: recompute
        y6 = attn(x, encoder_hidden_states=other, video_length=4)
        attn.__dict__.pop("_ctx_kv")
        y7 = attn(x, encoder_hidden_states=other, video_length=4)
        assert torch.equal(y6, y7) and not torch.equal(y6, y5)


def test_unet_context_is_one_tensor_while_unchanged():
    from vp2p.unet3d import UNet3DConditionModel
    unet = UNet3DConditionModel.__new__(UNet3DConditionModel)
    torch.nn.Module.__init__(unet)
    unet.conv_in = torch.nn.Conv2d(4, 8, 3).to(DEV, torch.bfloat16)         # only .dtype is read
    eh = torch.randn(4, 77, 768, device=DEV)
    a = unet._context(eh)
    assert a.dtype == torch.bfloat16 and unet._context(eh) is a
    eh[0].zero_()
    b = unet._context(eh)
    assert b is not a and torch.equal(b, eh.to(torch.bfloat16))
