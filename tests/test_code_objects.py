"""CPU checks of the built gfx950 code objects (no GPU needed): the kernels whose correctness rests on
hand-counted vector-memory waits or hand-placed instruction order use no scratch.  A spill would add
scratch loads / stores: unaccounted vector-memory operations under the K10s stream's counted `vmcnt`
(conv.hip, conv_kernel_k320) and the K1 pp kernel's pinned slots (frame_attn_pp.hip)."""
import os
import re
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("VP2P_LIB") or os.path.join(ROOT, "video-p2p_amd", "lib", "libvp2p_hip.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _gfx950_objects(path):
    """The gfx950 ELF code objects of every clang offload bundle in the library's fat binary."""
    data = open(path, "rb").read()
    i = data.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + len(MAGIC))[0]
        p = i + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode(errors="replace")
            p += tlen
            if "gfx950" in triple and size:
                yield data[i + off:i + off + size]
        i = data.find(MAGIC, i + 1)


def _kernel_meta(tmp_path):
    meta = {}
    for k, obj in enumerate(_gfx950_objects(LIB)):
        f = tmp_path / f"co{k}.elf"
        f.write_bytes(obj)
        out = subprocess.run([READELF, "--notes", str(f)], capture_output=True, text=True).stdout
        name = None
        for line in out.splitlines():
            m = re.match(r"\s*\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
                meta.setdefault(name, {})
                continue
            m = re.match(r"\s*\.(private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):\s+(\d+)", line)
            if m and name:
                meta[name][m.group(1)] = int(m.group(2))
    return meta


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(READELF)), reason="library or llvm-readelf missing")
def test_counted_wait_kernels_use_no_scratch(tmp_path):
    meta = _kernel_meta(tmp_path)
    picked = {n: m for n, m in meta.items() if "conv_kernel_k320" in n or "frame_attn_kernel_pp" in n}
    assert len([n for n in picked if "conv_kernel_k320" in n]) >= 3, sorted(meta)[:20]
    assert any("frame_attn_kernel_pp" in n for n in picked)
    for n, m in picked.items():
        assert m.get("private_segment_fixed_size", 0) == 0 and m.get("vgpr_spill_count", 0) == 0, (n, m)
