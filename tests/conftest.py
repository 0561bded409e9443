import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "video-p2p_amd"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    from vp2p.tuning import use_tuned_libraries
    use_tuned_libraries()            # before the first convolution initialises MIOpen
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"))


def record(test: str, **metrics):
    """Append measured parity numbers to $VP2P_PARITY_REPORT (JSON lines) when it is set, so a GPU
    run leaves the actual errors / PSNRs behind (profiles/r02_parity_*.jsonl)."""
    path = os.environ.get("VP2P_PARITY_REPORT")
    if path:
        import json
        with open(path, "a") as fh:
            fh.write(json.dumps({"test": test, **metrics}) + "\n")


@pytest.fixture(scope="session")
def golden_models():
    """Reference outputs of tuneavideo's own model files (tests/golden/make_golden_models.py)."""
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "golden_models.npz"))


def model_state(module_factory, seed: int):
    """{name: fp32 CPU tensor} of ``module_factory()``'s state dict filled by model_spec.param_values
    (the weights make_golden_models.py gave the reference's module of the same keys)."""
    import torch
    import model_spec as MS
    keys = {k: tuple(v.shape) for k, v in module_factory().state_dict().items()}
    return {k: torch.from_numpy(MS.param_values(k, s, seed)) for k, s in keys.items()}


@pytest.fixture(scope="session")
def tokenizer():
    from vp2p.tokenizer import SyntheticCLIPTokenizer
    return SyntheticCLIPTokenizer()
