import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
SEP = "::"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")


def rel_err(a, b) -> float:
    """SURVEY section 4 tolerance norm: max|a-b| / max|b| per tensor."""
    import torch
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)


class Golden:
    """Grouped view over ``golden_modules.npz``: ``Golden(z, 'mhdiff0')``."""

    def __init__(self, z, case):
        self.z, self.case = z, case

    def __getitem__(self, k):
        return self.z[f"{self.case}/{k}"]

    def has(self, k):
        return f"{self.case}/{k}" in self.z.files

    def state_dict(self, dtype=None):
        import torch
        pre = f"{self.case}/sd{SEP}"
        out = {}
        for f in self.z.files:
            if f.startswith(pre):
                t = torch.from_numpy(self.z[f])
                if f.endswith("freqs_cis"):
                    t = torch.view_as_complex(t.float().contiguous())
                elif dtype is not None and t.is_floating_point():
                    t = t.to(dtype)
                out[f[len(pre):]] = t
        return out

    def grads(self):
        import torch
        pre = f"{self.case}/grad{SEP}"
        return {f[len(pre):]: torch.from_numpy(self.z[f]) for f in self.z.files if f.startswith(pre)}


@pytest.fixture(scope="session")
def golden():
    return np.load(os.path.join(GOLDEN, "golden_modules.npz"))


@pytest.fixture(scope="session")
def golden_curve():
    return np.load(os.path.join(GOLDEN, "golden_loss_curve.npz"))
