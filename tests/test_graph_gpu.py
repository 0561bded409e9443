"""HIP-graph replay of the edit loop (VideoP2PPipeline(..., graphs=True)) is bit-identical to the eager
loop: the captured per-step graphs bake the same kernels with the same arguments
(pipeline_tuneavideo.py:394-430 per step, run_videop2p.py:286-329 decisions per step)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _edit_setup(tokenizer, frames=2):
    import bench
    import vp2p
    from vp2p.pipeline import VideoP2PPipeline
    from vp2p.unet3d import UNet3DConditionModel, init_random_
    unet = init_random_(UNet3DConditionModel(), seed=0).to("cuda", torch.bfloat16)
    unet = unet.to(memory_format=torch.channels_last).eval()
    prompts, swap, blend, eq, cross, self_ = bench.RABBIT
    ctrl = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, blend, eq, tokenizer=tokenizer)
    vp2p.register_attention_control(type("M", (), {"unet": unet})(), ctrl)
    g = torch.Generator().manual_seed(1)
    unc = torch.randn(1, 77, 768, generator=g)
    emb = torch.cat([unc, unc, torch.randn(2, 77, 768, generator=g)]).cuda()
    return VideoP2PPipeline(unet), ctrl, prompts, emb


@pytest.mark.timeout(300)
def test_graphed_edit_bit_equal(tokenizer):
    pipe, ctrl, prompts, emb = _edit_setup(tokenizer)
    steps = 14          # crosses the cross-replace (10) and LocalBlend (counter > 10) edges
    outs = {}
    entries = None
    for seed in (2, 3):
        x_t = torch.randn(1, 4, 2, 64, 64, generator=torch.Generator().manual_seed(seed)).cuda()
        with torch.no_grad():
            ctrl.reset()
            eager = pipe(prompts, 2, latents=x_t, controller=ctrl, fast=True, text_embeddings=emb,
                         num_inference_steps=steps)
            seen = []
            ctrl.reset()
            graphed = pipe(prompts, 2, latents=x_t, controller=ctrl, fast=True, text_embeddings=emb,
                           num_inference_steps=steps, graphs=True,
                           callback=lambda i, t, lat: seen.append((i, t)))
        assert [i for i, _ in seen] == list(range(steps))
        assert torch.isfinite(eager).all()
        assert torch.equal(eager, graphed), float((eager - graphed).abs().max())
        outs[seed] = graphed
        entries = entries if seed == 3 else pipe._graph_cache[1]
    # the second seed replayed the graphs captured for the first (the same cache entry)
    assert pipe._graph_cache[1] is entries
    assert not torch.equal(outs[2], outs[3])


@pytest.mark.timeout(300)
def test_graphed_edits_new_controller_memory_bounded(tokenizer):
    """a session that builds a controller per edit keeps ONE captured edit: the previous
    edit's graphs, pool and controller are released, so device memory does not grow edit after edit."""
    import bench
    import vp2p
    pipe, ctrl, prompts, emb = _edit_setup(tokenizer)
    prompts, swap, blend, eq, cross, self_ = bench.RABBIT
    x_t = torch.randn(1, 4, 2, 64, 64, generator=torch.Generator().manual_seed(2)).cuda()
    used = []
    for k in range(3):
        c = vp2p.make_controller(prompts, swap, {"default_": cross}, self_, blend, eq, tokenizer=tokenizer)
        vp2p.register_attention_control(type("M", (), {"unet": pipe.unet})(), c)
        with torch.no_grad():
            pipe(prompts, 2, latents=x_t, controller=c, fast=True, text_embeddings=emb, num_inference_steps=4,
                 graphs=True)
        del c
        torch.cuda.synchronize()
        used.append(torch.cuda.memory_allocated())
    assert pipe._graph_cache[1].controller is not None
    assert used[2] <= used[0] + (64 << 20), used
