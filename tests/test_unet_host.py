"""Host-side UNet3D logic that needs no GPU: the batched time-embedding projection
(UNet3DConditionModel._project_temb) equals every resnet's own ``time_emb_proj(silu(temb))``
(resnet.py:185-188), and its weight cache follows in-place weight updates."""
import torch
import torch.nn.functional as F

from test_unet_gpu import CFG
from vp2p.unet3d import ResnetBlock3D, UNet3DConditionModel, init_random_


def test_batched_temb_projection_matches_per_block():
    torch.manual_seed(0)
    u = init_random_(UNet3DConditionModel(**CFG), seed=0, std=0.05)
    for m in u.modules():
        if isinstance(m, ResnetBlock3D):
            m.time_emb_proj.bias.data.normal_()
    emb = torch.randn(2, u.time_embedding.linear_2.out_features)
    with torch.no_grad():
        u._project_temb(emb)
        rs = u._resnets
        assert len(rs) == sum(isinstance(m, ResnetBlock3D) for m in u.modules())
        for r in rs:
            torch.testing.assert_close(r._temb_pre, r.time_emb_proj(F.silu(emb)), rtol=1e-6, atol=1e-6)
        rs[0].time_emb_proj.weight.add_(1.0)       # in-place update -> the concatenated copy is rebuilt
        u._project_temb(emb)
        torch.testing.assert_close(rs[0]._temb_pre, rs[0].time_emb_proj(F.silu(emb)), rtol=1e-6, atol=1e-6)
