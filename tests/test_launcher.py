"""bench.py's multi-rank launcher and the EditLayout exchanges, rehearsed on the CPU with gloo.

``python bench.py --gpus N`` must start the N ranks itself (a torchrun CHILD process; the parent
never touches the GPU and never execs) -- the driver's SCALE run uses it, or an external torchrun.
``--mode selftest`` runs the layout's collectives (CFG all-gather, frame-0 broadcast, the attn_temp
all-to-all round trip) on CPU tensors and checks them against the single-rank answer."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n,layout", [(2, "cfg-split x2"), (4, "cfg-split x2 x frame-sharded x2"),
                                      (8, "cfg-split x2 x frame-sharded x4")])
def test_bench_launches_ranks(n, layout):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--mode", "selftest"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 prints exactly one line
    assert lines[0]["selftest"] == "ok" and lines[0]["world"] == n and lines[0]["layout"] == layout


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mode", "selftest"],
                         capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr
