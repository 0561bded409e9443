"""CPU checks of the C-ABI boundary: the library loads, exports every symbol include/vp2p.h declares,
and the ctypes structs have the C layout (sizeof/offsetof compiled from the header with gcc)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vp2p.h")
LIB = os.path.join(ROOT, "video-p2p_amd", "lib", "libvp2p_hip.so")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t)\s+(vp2p_\w+)\s*\(", src, re.M)))


def test_header_declares_the_exports():
    from vp2p import _lib
    assert sorted(_lib.EXPORTS) == _declared()


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built (run __graft_entry__.build())")
def test_library_exports_every_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in _declared() if s not in syms]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_library_loads_and_reports_abi():
    from vp2p import _lib
    lib = _lib.load()
    assert lib.vp2p_abi_version() == _lib.ABI_VERSION
    assert 40 in _lib.supported_head_dims() and 160 in _lib.supported_head_dims()
    # host-side validation only (no kernel launch): bad arguments are rejected before any launch
    assert lib.vp2p_cross_kv_workspace_bytes(4, 77, 8, 40, 1) > 0
    assert lib.vp2p_cross_kv_workspace_bytes(4, 200, 8, 40, 1) == -4
    assert lib.vp2p_cross_kv_workspace_bytes(4, 77, 8, 41, 1) == -3
    assert lib.vp2p_frame_attn_fwd(None, None) == -1
    assert lib.vp2p_temporal_attn_p2p_fwd(None, None) == -1
    gn = _lib.GroupNormArgs(x=1, y=1, batch=4, frames=8, rows=4096, channels=320, groups=32, eps=1e-5, dtype=1)
    assert lib.vp2p_group_norm_parts(ctypes.byref(gn)) > 0
    gn.channels = 324
    assert lib.vp2p_group_norm_parts(ctypes.byref(gn)) == -4
    assert lib.vp2p_group_norm_stats(ctypes.byref(gn), None) == -4
    assert lib.vp2p_layer_norm_fwd(None, None) == -1
    assert lib.vp2p_geglu_fwd(None, None, 1, 8, 1, None) == -1


def test_struct_layout_matches_header(tmp_path):
    from vp2p import _lib
    structs = {"vp2p_frame_attn_args": _lib.FrameAttnArgs, "vp2p_cross_attn_args": _lib.CrossAttnArgs,
               "vp2p_temporal_attn_args": _lib.TemporalAttnArgs, "vp2p_step_args": _lib.StepArgs,
               "vp2p_group_norm_args": _lib.GroupNormArgs, "vp2p_layer_norm_args": _lib.LayerNormArgs,
               "vp2p_frame_attn_bwd_args": _lib.FrameAttnBwdArgs,
               "vp2p_temporal_attn_bwd_args": _lib.TemporalAttnBwdArgs,
               "vp2p_nulltext_loss_args": _lib.NullTextLossArgs, "vp2p_conv_args": _lib.ConvArgs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(c), "-o", str(exe)], check=True)
    got = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    for line in filter(None, got):
        cname, field, val = line.split()
        py = structs[cname]
        want = ctypes.sizeof(py) if field == "size" else getattr(py, field).offset
        assert int(val) == want, (cname, field, val, want)


def test_linear_alpha_rejects_residual_epilogue():
    """The output scale is defined only for the plain epilogue: with a residual the shape is unsupported."""
    import ctypes
    from vp2p import _lib
    lib = _lib.load()
    a = _lib.ConvArgs(None, None, None, None, None, 1, 4096, 1, 320, 320, 4096, 1, 1, 1, 0, _lib.BF16,
                      _lib.CONV_EPI_NONE)
    assert lib.vp2p_conv2d_supported(ctypes.byref(a)) == 1
    a.alpha = 0.5
    assert lib.vp2p_conv2d_supported(ctypes.byref(a)) == 1
    a.residual = 16
    assert lib.vp2p_conv2d_supported(ctypes.byref(a)) == 0
    a.residual = None
    a.alpha = float("nan")
    assert lib.vp2p_conv2d_supported(ctypes.byref(a)) == 0


def test_linear_rule_table():
    """The K10-vs-hipBLASLt projection choice is a fixed table of M ranges (no timing at run time)."""
    from vp2p import ops
    r = ops.LinearRule()
    assert r.use_k10(131072, 320, 320)            # the res-64 projections (measured K10 0.71x hipBLASLt)
    assert not r.use_k10(131072, 123, 456)        # pairs not in the table stay on the library
    for k, runs in r.rules.items():
        K, N = (int(t) for t in k.split("|"))
        assert K % 64 == 0 and N % 160 == 0
        for lo, hi in runs:
            assert (lo is None or lo > 0) and (hi is None or lo is None or hi >= lo)
    r.rules = {"640|640": [[None, 4096], [65536, 65536], [131072, None]]}
    assert r.use_k10(10, 640, 640) and r.use_k10(4096, 640, 640) and not r.use_k10(8192, 640, 640)
    assert r.use_k10(65536, 640, 640) and not r.use_k10(100000, 640, 640) and r.use_k10(10 ** 7, 640, 640)


def test_conv_gn_parts_host():
    """vp2p_conv2d_gn_parts (ABI 15): the tiles per GroupNorm sample the epilogue writes partials for --
    the one-pass tile's rows -- or 0 where the epilogue cannot produce them (host logic, no GPU)."""
    import ctypes
    from vp2p import _lib
    lib = _lib.load()

    def args(n, h, cin, cout, k=3):
        a = _lib.ConvArgs(None, None, None, None, None, n, h, h, cin, cout, h, h, k, 1, (k - 1) // 2, _lib.BF16,
                          _lib.CONV_EPI_NONE)
        return a
    a = args(32, 64, 320, 320)                    # the 8-frame edit's res-64 conv1: wide 256-row tile
    a.gn_groups, a.gn_rows = 32, 8 * 64 * 64
    assert lib.vp2p_conv2d_gn_parts(ctypes.byref(a)) == 8 * 64 * 64 // 256
    a.gn_rows = 64 * 64                           # per-frame statistics (Transformer3DModel.norm)
    assert lib.vp2p_conv2d_gn_parts(ctypes.byref(a)) == 16
    a.residual = 16                               # conv2 + shortcut: statistics of the stored sum
    assert lib.vp2p_conv2d_gn_parts(ctypes.byref(a)) == 16
    a.residual = None
    a.gn_groups = 7                               # groups must divide the channels
    assert lib.vp2p_conv2d_gn_parts(ctypes.byref(a)) == 0
    a.gn_groups, a.gn_rows = 32, 100              # rows per sample not a multiple of the tile
    assert lib.vp2p_conv2d_gn_parts(ctypes.byref(a)) == 0
    b = args(4, 8, 1280, 1280)                    # res-8, small M: split-K, no one-pass epilogue
    b.gn_groups, b.gn_rows = 32, 64
    assert lib.vp2p_conv2d_gn_parts(ctypes.byref(b)) == 0
    c = args(32, 64, 320, 320)
    c.img_add, c.residual = 16, 32                # a per-image add only without a residual
    assert lib.vp2p_conv2d_supported(ctypes.byref(c)) == 0


def test_conv_plan_host(monkeypatch):
    """vp2p_conv2d_plan (ABI 16): the K10 launch plan per shape -- the measured rules of DESIGN §4
    (profiles/r06_k10_plan_*.jsonl, r06_small_clip_*): 8-frame edit on the wide tile, the 3-frame clip's
    64x64 convs on 192 x 320, its 16x16 long-K convs on 4 slices of 192 x 320, the 1-frame clip's on
    the short tile (host logic, no GPU)."""
    import ctypes
    from vp2p import _lib
    lib = _lib.load()

    def plan(n, h, cin, cout, k=3, up=0, epi=_lib.CONV_EPI_NONE):
        a = _lib.ConvArgs(None, None, None, None, None, n, h, h, cin, cout, h, h, k, 1, (k - 1) // 2, _lib.BF16,
                          epi)
        a.upsample = up
        t, ks = ctypes.c_int32(-1), ctypes.c_int32(-1)
        assert lib.vp2p_conv2d_plan(ctypes.byref(a), ctypes.byref(t), ctypes.byref(ks)) == 0
        return t.value, ks.value

    monkeypatch.delenv("VP2P_K10_PLAN", raising=False)
    assert plan(32, 64, 320, 320) == (2, 1)           # 8 frames, 64x64: 512 wide tiles
    assert plan(32, 8, 1280, 1280) == (0, 4)          # 8 frames, 8x8: 128 tiles x 4 slices
    assert plan(12, 64, 320, 320) == (4, 1)           # 3 frames, 64x64: 256 tiles of 192 x 320
    assert plan(12, 64, 960, 320) == (4, 1)
    assert plan(12, 32, 640, 640) == (0, 1)           # 3 frames, 32x32: 384 tiles of 128 x 160
    assert plan(12, 16, 1280, 1280) == (4, 4)         # 3 frames, 16x16, 180 K-steps: 64 tiles x 4
    assert plan(12, 16, 2560, 1280) == (4, 4)
    assert plan(12, 16, 640, 1280) == (3, 1)          # 90 K-steps: one pass on the short tile
    assert plan(12, 16, 1280, 1280, up=1) == (4, 4)   # the Upsample3D conv there
    assert plan(4, 64, 320, 320) == (3, 1)            # 1 frame, 64x64: 512 short tiles
    assert plan(12, 64, 320, 320, k=1) == (5, 1)      # K = 320 projection: the K10s stream
    a = _lib.ConvArgs(None, None, None, None, None, 768, 1, 1, 1280, 1280, 1, 1, 1, 1, 0, _lib.BF16,
                      _lib.CONV_EPI_NONE)
    t, ks = ctypes.c_int32(-1), ctypes.c_int32(-1)
    assert lib.vp2p_conv2d_plan(ctypes.byref(a), ctypes.byref(t), ctypes.byref(ks)) == 0
    assert (t.value, ks.value) == (3, 1)               # short-K projection, 48 tiles: one pass, not split
    monkeypatch.setenv("VP2P_K10_PLAN", "0,1")         # the A/B override, where valid
    assert plan(12, 64, 320, 320) == (0, 1)
    monkeypatch.delenv("VP2P_K10_PLAN")
    geglu = plan(32, 16, 1280, 10240, k=1, epi=_lib.CONV_EPI_GEGLU)
    monkeypatch.setenv("VP2P_K10_PLAN", "4,2")         # invalid for the GEGLU epilogue: ignored
    assert plan(32, 16, 1280, 10240, k=1, epi=_lib.CONV_EPI_GEGLU) == geglu
    monkeypatch.delenv("VP2P_K10_PLAN")
    a.cin = 100                                        # unsupported shape
    assert lib.vp2p_conv2d_plan(ctypes.byref(a), ctypes.byref(t), ctypes.byref(ks)) == -4


def test_geglu_interleave_layout():
    """K10's GEGLU weight order: per 32 rows, 16 value rows then the matching 16 gate rows."""
    import torch
    from vp2p import ops
    inner, k = 160, 4
    w = torch.arange(2 * inner * k, dtype=torch.float32).reshape(2 * inner, k)
    b = torch.arange(2 * inner, dtype=torch.float32)
    wi, bi = ops.geglu_interleave(w, b)
    for blk in range(inner // 16):
        assert torch.equal(wi[32 * blk:32 * blk + 16], w[16 * blk:16 * blk + 16])
        assert torch.equal(wi[32 * blk + 16:32 * blk + 32], w[inner + 16 * blk:inner + 16 * blk + 16])
        assert torch.equal(bi[32 * blk + 16:32 * blk + 32], b[inner + 16 * blk:inner + 16 * blk + 16])
