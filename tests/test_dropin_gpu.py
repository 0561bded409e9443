"""The drop-in surface on a FOREIGN module tree (not vp2p's classes), on the MI355X.

``ForeignUNet`` is a module tree with exactly the attribute set the reference hook reads
(diffusers-0.11.1 ``CrossAttention``: to_q / to_k / to_v / to_out, heads, scale,
reshape_heads_to_batch_dim / reshape_batch_dim_to_heads; ptp_utils.py:189-208) under down / mid / up
containers -- the shape of the reference's registration target.  The hooked layers are called the
way tuneavideo calls them (attention.py:251-267): attn2 with the per-frame-repeated context on
'(b f) n c', attn_temp on the '(b d) f c' rearrangement, no video_length.

Checked against the oracle (oracle/p2p_oracle.py, pinned to the reference's own controllers by
tests/test_oracle_golden.py) on identical inputs:
* ``vp2p.register_attention_control`` + ``vp2p.make_controller`` (fused kernels) over 12 steps x 32
  layers crossing the cross-attention window (step 10) and the LocalBlend start (counter 11);
* ``store_maps=True``: the AttentionStore maps (post-edit, step-summed, N <= 32^2) and
  ``get_average_attention`` (run_videop2p.py:248-283, 270-272);
* a foreign controller (not a vp2p class): the generic path materialises ``attn`` exactly as the
  reference hook hands it over (ptp_utils.py:217-219) and applies ``attn @ v`` to what it returns.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import p2p_oracle as O

pytestmark = pytest.mark.gpu

HEADS, D = 8, 32
C = HEADS * D
CTX, F_, P = 64, 2, 2
B = 2 * P
LEVELS = [1040, 1040, 144, 144, 256, 256, 16, 256, 256, 256, 144, 144, 144, 1040, 1040, 1040]
PLACES = ["down"] * 6 + ["mid"] + ["up"] * 9
STEPS = 12


def _rng(*k):
    return np.random.default_rng(np.random.SeedSequence(list(k)))


def _weights(block, li, ctx):
    g = _rng(51, block, li)
    return {"to_q": (g.standard_normal((C, C)) * C ** -0.5).astype(np.float32),
            "to_k": (g.standard_normal((C, ctx)) * ctx ** -0.5).astype(np.float32),
            "to_v": (g.standard_normal((C, ctx)) * ctx ** -0.5).astype(np.float32),
            "to_out_w": (g.standard_normal((C, C)) * C ** -0.5).astype(np.float32),
            "to_out_b": (g.standard_normal((C,)) * 0.1).astype(np.float32)}


class CrossAttention(nn.Module):
    """Foreign module with the diffusers-0.11.1 CrossAttention attribute set."""

    def __init__(self, w):
        super().__init__()
        self.heads, self.scale = HEADS, D ** -0.5
        self.to_q = nn.Linear(C, C, bias=False)
        self.to_k = nn.Linear(w["to_k"].shape[1], C, bias=False)
        self.to_v = nn.Linear(w["to_v"].shape[1], C, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(C, C), nn.Dropout(0.0)])
        with torch.no_grad():
            for name, key in (("to_q", "to_q"), ("to_k", "to_k"), ("to_v", "to_v")):
                getattr(self, name).weight.copy_(torch.from_numpy(w[key]))
            self.to_out[0].weight.copy_(torch.from_numpy(w["to_out_w"]))
            self.to_out[0].bias.copy_(torch.from_numpy(w["to_out_b"]))

    def reshape_heads_to_batch_dim(self, t):
        b, n, dim = t.shape
        return t.reshape(b, n, HEADS, dim // HEADS).permute(0, 2, 1, 3).reshape(b * HEADS, n, dim // HEADS)

    def reshape_batch_dim_to_heads(self, t):
        bh, n, d = t.shape
        return t.reshape(bh // HEADS, HEADS, n, d).permute(0, 2, 1, 3).reshape(bh // HEADS, n, HEADS * d)


class FrameAttention(CrossAttention):
    """Foreign attn1: the reference's subclass (attention.py:273-329) -- named ``FrameAttention``,
    with its diffusers attributes group_norm / added_kv_proj_dim unset (as in SD-1.5) and the
    xformers switch the pipeline toggles.  Its own forward must never run once registered."""

    def __init__(self, w):
        super().__init__(w)
        self.group_norm, self.added_kv_proj_dim = None, None
        self._use_memory_efficient_attention_xformers = True

    def forward(self, *a, **k):
        raise AssertionError("the reference FrameAttention.forward ran: attn1 was not routed to K1")


class Block(nn.Module):
    def __init__(self, i):
        super().__init__()
        self.attn1 = FrameAttention(_weights(i, 2, C))
        self.attn2 = CrossAttention(_weights(i, 0, CTX))
        self.attn_temp = CrossAttention(_weights(i, 1, C))


class ForeignUNet(nn.Module):
    def __init__(self):
        super().__init__()
        blocks = [Block(i) for i in range(16)]
        self.down_blocks = nn.ModuleList(blocks[:6])
        self.mid_block = nn.ModuleList(blocks[6:7])
        self.up_blocks = nn.ModuleList(blocks[7:])
        self.blocks = blocks


def _ctx():
    g = _rng(52)
    unc = g.standard_normal((1, 77, CTX)).astype(np.float32)
    cond = g.standard_normal((P, 77, CTX)).astype(np.float32)
    return np.concatenate([np.repeat(unc, P, 0), cond]).astype(np.float32)


def _inputs(step, block):
    g = _rng(53, step, block)
    n = LEVELS[block]
    return (g.standard_normal((B * F_, n, C)).astype(np.float32),
            g.standard_normal((B * n, F_, C)).astype(np.float32))


def _oracle_w(block):
    return _weights(block, 0, CTX), _weights(block, 1, C)


def _controllers(tokenizer, store_maps):
    import spec
    import vp2p
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS["rabbit"]
    bw = ((blend[0],), (blend[1],))
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, bw, eq, tokenizer=tokenizer,
                                store_maps=store_maps)
    octrl = O.EditController(prompts, swap, {"default_": cross}, self_, tokenizer, blend_words=bw, eq_params=eq)
    return ctrl, octrl


def _rel(a, b):
    return float(np.abs(a - b).max() / np.abs(b).max())


@pytest.mark.parametrize("store_maps", [False, True])
def test_register_on_foreign_tree_matches_oracle(tokenizer, store_maps):
    import types
    import vp2p
    net = ForeignUNet().cuda()
    ctrl, octrl = _controllers(tokenizer, store_maps)
    vp2p.register_attention_control(types.SimpleNamespace(unet=net), ctrl)
    assert ctrl.num_att_layers == 32
    ctx = _ctx()
    ctx_f = np.repeat(ctx, F_, axis=0)                     # repeat 'b n c -> (b f) n c' (attention.py:95)
    ctx_t = torch.from_numpy(ctx_f).cuda()
    g = _rng(54)
    worst = 0.0
    with torch.no_grad():
        for step in range(STEPS):
            for bi, blk in enumerate(net.blocks):
                xc, xt = _inputs(step, bi)
                w2, wt = _oracle_w(bi)
                oc = blk.attn2(torch.from_numpy(xc).cuda(), encoder_hidden_states=ctx_t).cpu().numpy()
                ot = blk.attn_temp(torch.from_numpy(xt).cuda()).cpu().numpy()
                rc, _ = O.hooked_forward(xc, ctx_f, w2, HEADS, octrl, PLACES[bi])
                rt, _ = O.hooked_forward(xt, None, wt, HEADS, octrl, PLACES[bi])
                worst = max(worst, _rel(oc, rc), _rel(ot, rt))
            lat = g.standard_normal((P, 4, F_, 64, 64)).astype(np.float32)
            got = ctrl.step_callback(torch.from_numpy(lat).cuda()).cpu().numpy()
            ref = octrl.step_callback(lat)
            # equal wherever the (thresholded) masks agree; count disagreeing pixels
            flips = int((np.abs(got - ref) > 1e-6).any(axis=1).sum())
            assert flips <= 8, (step, flips)
    assert worst < 1e-4, worst
    assert ctrl.cur_step == octrl.cur_step == STEPS and ctrl.local_blend.counter == STEPS
    if store_maps:
        for key, maps in octrl.attention_store.items():
            mine = ctrl.attention_store[key]
            assert len(mine) == len(maps), key
            for a, b in zip(mine, maps):
                assert _rel(a.cpu().numpy(), b) < 1e-4, key
        avg = ctrl.get_average_attention()
        for key, maps in octrl.attention_store.items():
            for a, b in zip(avg[key], maps):
                assert _rel(a.cpu().numpy(), b / STEPS) < 1e-4, key


class ForeignStore:
    """A controller that is NOT a vp2p class: the reference protocol (run_videop2p.py:196-233) with
    an AttentionStore-like sum and a simple edit (cond-half cross maps of word 2 doubled)."""

    def __init__(self):
        self.cur_step, self.cur_att_layer, self.num_att_layers = 0, 0, -1
        self.sums = {}

    def __call__(self, attn, is_cross, place_in_unet):
        h = attn.shape[0]
        if is_cross:
            attn[h // 2:, :, 2] *= 2.0
        key = f"{place_in_unet}_{'cross' if is_cross else 'self'}_{self.cur_att_layer}"
        self.sums[key] = self.sums.get(key, 0) + attn[h // 2:].sum().item()
        self.cur_att_layer += 1
        if self.cur_att_layer == self.num_att_layers:
            self.cur_att_layer = 0
            self.cur_step += 1
        return attn


def test_foreign_controller_generic_path():
    import types
    import vp2p
    net = ForeignUNet().cuda()
    ctrl = ForeignStore()
    vp2p.register_attention_control(types.SimpleNamespace(unet=net), ctrl)
    assert ctrl.num_att_layers == 32

    def oracle_ctrl(attn, is_cross, place):
        h = attn.shape[0]
        attn = attn.copy()
        if is_cross:
            attn[h // 2:, :, 2] *= 2.0
        return attn

    ctx_f = np.repeat(_ctx(), F_, axis=0)
    with torch.no_grad():
        for bi in (0, 4, 6):                             # res-64 (N > 32^2), res-16, mid (res-8)
            blk = net.blocks[bi]
            xc, xt = _inputs(0, bi)
            w2, wt = _oracle_w(bi)
            oc = blk.attn2(torch.from_numpy(xc).cuda(), encoder_hidden_states=torch.from_numpy(ctx_f).cuda())
            ot = blk.attn_temp(torch.from_numpy(xt).cuda())
            rc, _ = O.hooked_forward(xc, ctx_f, w2, HEADS, oracle_ctrl, PLACES[bi])
            rt, _ = O.hooked_forward(xt, None, wt, HEADS, oracle_ctrl, PLACES[bi])
            assert _rel(oc.cpu().numpy(), rc) < 1e-4 and _rel(ot.cpu().numpy(), rt) < 1e-4
    assert ctrl.cur_att_layer == 6 and len(ctrl.sums) == 6


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_frame_attention_on_foreign_tree(tokenizer, dtype):
    """attn1 of a foreign tree (class named ``FrameAttention``, the reference's attn1) runs on K1
    once registered: ``ops.frame_attention`` launches for every call, the controller's layer count
    stays 32 (attn1 is not hooked, ptp_utils.py:237), and the output -- to_q, K/V of frame 0,
    softmax, to_out (attention.py:282-329) -- matches the oracle within the north-star bars (fp32
    1e-4, bf16 2e-2 of max|ref|) at res-64-like (1040 tokens), res-16 and res-8 token counts."""
    import types
    import vp2p
    from vp2p import ops
    net = ForeignUNet().cuda().to(dtype)
    ctrl, _ = _controllers(tokenizer, False)
    vp2p.register_attention_control(types.SimpleNamespace(unet=net), ctrl)
    assert ctrl.num_att_layers == 32
    calls = []
    orig = ops.frame_attention

    def counting(*a, **k):
        calls.append(a[0].shape)
        return orig(*a, **k)

    ops.frame_attention = counting
    try:
        with torch.no_grad():
            for bi in (0, 4, 6):
                n = LEVELS[bi]
                x = _rng(55, bi).standard_normal((B * F_, n, C)).astype(np.float32)
                xt = torch.from_numpy(x).to(dtype)
                got = net.blocks[bi].attn1(xt.cuda(), video_length=F_).float().cpu().numpy()
                w = _weights(bi, 2, C)
                xr = xt.float().numpy()
                q = xr @ w["to_q"].T
                k = xr @ w["to_k"].T
                v = xr @ w["to_v"].T
                o = O.frame_attention(q.astype(np.float32), k.astype(np.float32), v.astype(np.float32),
                                      F_, HEADS)
                ref = o @ w["to_out_w"].T + w["to_out_b"]
                assert _rel(got, ref) < (1e-4 if dtype == torch.float32 else 2e-2), (bi, _rel(got, ref))
    finally:
        ops.frame_attention = orig
    assert len(calls) == 3
    assert ctrl.cur_att_layer == 0        # attn1 never reaches the controller
