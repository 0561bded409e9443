"""Frame-sharded execution.

CPU (gloo, world size 2): the exchange steps themselves -- frames<->tokens all-to-all, the cross-frame
GroupNorm statistics, frame-0 broadcast, slicing and gathering -- against single-process results.
GPU (two ranks on the one MI355X, gloo with host staging): a frame-sharded UNet3D forward with the P2P
controller equals the unsharded forward.
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _cpu_worker(rank, world, port, out_path):
    dist = _init(rank, world, port)
    from vp2p.frame_parallel import FrameShard
    torch.manual_seed(0)
    B, f, N, C = 3, 4, 8, 6
    full = torch.randn(B * f, N, C)                                  # '(b f) n c', identical on all ranks
    sh = FrameShard()
    loc = full.reshape(B, f, N, C)[:, rank * (f // world):(rank + 1) * (f // world)].reshape(-1, N, C)
    tok = sh.to_tokens(loc.contiguous(), B)
    want = full.reshape(B, f, N, C)[:, :, rank * (N // world):(rank + 1) * (N // world)].reshape(-1, N // world, C)
    ok = [torch.equal(tok, want), torch.equal(sh.to_frames(tok, B), loc)]
    # cross-frame GroupNorm statistics: sums over every rank's frames
    x = torch.randn(2, f * 5, 4, 3, dtype=torch.float64).float()   # (B, f*HW, G, Cg), same on all ranks
    xl = x.reshape(2, f, 5, 4, 3)[:, rank * (f // world):(rank + 1) * (f // world)].reshape(2, -1, 4, 3)
    mean, var = sh.group_norm_stats(xl, xl.shape[1] * 3)
    v_ref, m_ref = torch.var_mean(x, dim=(1, 3), unbiased=False)
    ok += [torch.allclose(mean, m_ref, atol=1e-6), torch.allclose(var, v_ref, atol=1e-5)]
    t = torch.full((4,), float(rank))
    sh.broadcast_(t)
    ok.append(bool((t == 0).all()))
    lat = torch.arange(2 * 3 * f * 2, dtype=torch.float32).reshape(2, 3, f, 2)
    ok.append(torch.equal(sh.gather(sh.local(lat, 2), 2), lat))
    flat = torch.arange(5, dtype=torch.float32) + 10 * rank
    ok.append(torch.equal(sh.all_gather_flat(flat), torch.cat([torch.arange(5.0) + 10 * r for r in range(world)])))
    torch.save(ok, out_path + f".{rank}")
    dist.destroy_process_group()


def test_exchanges_gloo_world2(tmp_path):
    port = _port()
    out = str(tmp_path / "res")
    mp.spawn(_cpu_worker, args=(2, port, out), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(out + f".{r}")
        assert all(res), res


# ------------------------------------------------------------------------------------------------
CFG = dict(block_out_channels=(256, 256, 512, 512), cross_attention_dim=64, attention_head_dim=8)


def _unet_case(frames):
    import numpy as np
    import spec
    import vp2p
    from vp2p.tokenizer import SyntheticCLIPTokenizer
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    prompts, swap, blend, eq, cross, self_ = spec.CONFIGS["rabbit"]
    tok = SyntheticCLIPTokenizer()
    unet = init_random_(UNet3DConditionModel(**CFG), seed=0, std=0.05).cuda().to(memory_format=torch.channels_last)
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, ((blend[0],), (blend[1],)), eq,
                                tokenizer=tok)
    vp2p.register_attention_control(type("M", (), {"unet": unet})(), ctrl)
    g = np.random.default_rng(7)
    x = torch.from_numpy(g.standard_normal((4, 4, frames, 64, 64)).astype(np.float32)).cuda()
    ctx = torch.from_numpy(g.standard_normal((4, 77, 64)).astype(np.float32)).cuda()
    ctx[:2] = ctx[0]
    return unet, ctrl, x, ctx


def _gpu_worker(rank, world, port, out_path, frames):
    dist = _init(rank, world, port)
    from vp2p.frame_parallel import FrameShard, frame_parallel
    unet, ctrl, x, ctx = _unet_case(frames)
    sh = FrameShard()
    with torch.no_grad(), frame_parallel(sh):
        y = unet(sh.local(x, 2), 481, ctx).sample
        y = sh.gather(y, 2)
        lb = sh.gather(ctrl.attention_store.lb_acc, 1)
    if rank == 0:
        torch.save({"y": y.cpu(), "lb": lb.cpu()}, out_path)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_frame_sharded_unet_matches_single(tmp_path):
    frames = 4
    out = str(tmp_path / "sharded.pt")
    mp.spawn(_gpu_worker, args=(2, _port(), out, frames), nprocs=2, join=True)
    got = torch.load(out)
    sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
    unet, ctrl, x, ctx = _unet_case(frames)
    with torch.no_grad():
        ref = unet(x, 481, ctx).sample.cpu()
    err = (got["y"] - ref).abs().max() / ref.abs().max()
    assert err < 1e-4, float(err)
    lb_ref = ctrl.attention_store.lb_acc.cpu()
    assert ((got["lb"] - lb_ref).abs().max() / lb_ref.abs().max()) < 1e-4


# ------------------------------------------------------------------------------------------------
def _edit_worker(rank, world, port, out_path, frames, steps):
    """A short fast-mode edit (LocalBlend on from the first step) under the bench's EditLayout:
    world 2 = CFG split, world 4 = CFG split x 2 frame shards."""
    dist = _init(rank, world, port)
    from vp2p.frame_parallel import EditLayout, frame_parallel
    from vp2p.pipeline import VideoP2PPipeline
    import spec
    unet, ctrl, x, ctx = _unet_case(frames)
    ctrl.local_blend.start_blend = 0
    lay = EditLayout()
    with torch.no_grad(), frame_parallel(lay):
        lat = VideoP2PPipeline(unet)(spec.CONFIGS["rabbit"][0], lay.frames_local(frames),
                                     latents=lay.local(x[:1], 2), controller=ctrl, fast=True,
                                     text_embeddings=ctx, num_inference_steps=steps)
        if lay.frames is not None:
            lat = lay.frames.gather(lat, 2)
    torch.save(lat.cpu(), out_path + f".{rank}")
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_cfg_split_edit_matches_single(tmp_path, world):
    """The bench's multi-GPU decomposition (frame_parallel.EditLayout: CFG halves on two rank groups,
    frames sharded inside each half; the per-step all-gather of the UNet outputs and the LocalBlend
    broadcast) reproduces the single-rank edit.  All ranks share the one GPU (gloo, host staging)."""
    frames, steps = 4, 3
    out = str(tmp_path / "edit")
    mp.spawn(_edit_worker, args=(world, _port(), out, frames, steps), nprocs=world, join=True)
    sys.path.insert(0, os.path.join(ROOT, "video-p2p_amd"))
    import spec
    from vp2p.pipeline import VideoP2PPipeline
    unet, ctrl, x, ctx = _unet_case(frames)
    ctrl.local_blend.start_blend = 0
    with torch.no_grad():
        ref = VideoP2PPipeline(unet)(spec.CONFIGS["rabbit"][0], frames, latents=x[:1], controller=ctrl, fast=True,
                                     text_embeddings=ctx, num_inference_steps=steps).cpu()
    for r in range(world):
        got = torch.load(out + f".{r}")
        err = (got - ref).abs().max() / ref.abs().max()
        assert err < 1e-4, (r, float(err))
