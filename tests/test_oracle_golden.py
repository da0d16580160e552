"""Pin the CPU oracle against vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only; runs here and on the GPU box."""
import math

import pytest
import torch

from conftest import Golden, rel_err
from oracle import diffattn_oracle as orc

TOL64 = 1e-6          # fixture values are stored fp32; fp64 recompute must agree to ~1e-7


def _run(fn, x, params):
    x = x.clone().requires_grad_(True)
    for p in params.values():
        if p.is_floating_point():
            p.requires_grad_(True)
    out = fn(x)
    return x, out


def _check_case(g: Golden, fn, grad_keys=True):
    sd = g.state_dict(torch.float64)
    leaf = {k: v for k, v in sd.items() if "lambda_init" not in k and not k.endswith("freqs_cis")}
    x = torch.from_numpy(g["in0"]).double().requires_grad_(True)
    for v in leaf.values():
        v.requires_grad_(True)
    out = fn(x, sd)
    assert rel_err(out, g["out"]) < TOL64
    gout = torch.from_numpy(g["gout"]).double()
    (out * gout).sum().backward()
    assert rel_err(x.grad, g["grad_in0"]) < TOL64
    if grad_keys:
        for name, ref in g.grads().items():
            got = leaf[name].grad
            assert got is not None, name
            assert rel_err(got, ref) < TOL64, name


def test_group_layer_norm(golden):
    g = Golden(golden, "gln")
    _check_case(g, lambda x, sd: orc.group_layer_norm(x, sd["weight"], sd["bias"]))


@pytest.mark.parametrize("ci", range(4))
def test_diff_head(golden, ci):
    g = Golden(golden, f"diffhead{ci}")
    hs, C, T, blk, layer = [int(v) for v in g["meta"]]
    _check_case(g, lambda x, sd: orc.diff_head(x, sd, layer, blk))
    # lambda_init side effect of get_lambda (diff_transformer.py:44)
    assert abs(float(g["sd::lambda_init"]) - float(orc.lambda_init_for_layer(layer))) < 1e-7


@pytest.mark.parametrize("ci", range(4))
def test_multihead_diff(golden, ci):
    g = Golden(golden, f"mhdiff{ci}")
    H, hs, C, T, blk, layer = [int(v) for v in g["meta"]]
    _check_case(g, lambda x, sd: orc.multihead_diff_attention(x, sd, H, layer, blk))
    # the MHA's own buffer stays 0.8 -> the output scale is the constant 0.2
    assert float(g["sd::lambda_init"]) == pytest.approx(0.8)


@pytest.mark.parametrize("ci", range(4))
def test_alternating_head(golden, ci):
    g = Golden(golden, f"althead{ci}")
    N, hs, C, T, blk, layer = [int(v) for v in g["meta"]]
    _check_case(g, lambda x, sd: orc.alternating_diff_head(x, sd, N, layer, blk))


@pytest.mark.parametrize("ci", range(3))
def test_multihead_alternating(golden, ci):
    g = Golden(golden, f"mhalt{ci}")
    N, H, hs, C, T, blk, layer = [int(v) for v in g["meta"]]
    _check_case(g, lambda x, sd: orc.multihead_alternating_diff_attention(x, sd, H, N, layer, blk))


def test_control_multihead(golden):
    g = Golden(golden, "ctrlmha")
    H, hs, C, T, blk = [int(v) for v in g["meta"]]
    _check_case(g, lambda x, sd: orc.control_multihead(x, sd, H, blk))


def test_rope(golden):
    fc = orc.precompute_freqs_cis(32, 40)
    ref = torch.view_as_complex(torch.from_numpy(golden["rope/freqs"]).contiguous())
    assert torch.equal(fc, ref)
    x = torch.from_numpy(golden["rope/x"])
    assert torch.equal(orc.apply_rotary_emb(x, fc), torch.from_numpy(golden["rope/out"]))


def test_dlambda_identity():
    torch.manual_seed(0)
    B, T, hs = 2, 9, 8
    q1, k1, q2, k2 = (torch.randn(B, T, hs, dtype=torch.float64) for _ in range(4))
    v = torch.randn(B, T, 2 * hs, dtype=torch.float64)
    lam = torch.tensor(0.37, dtype=torch.float64, requires_grad=True)
    out = orc.diff_core([q1, q2], [k1, k2], v, torch.stack([torch.ones((), dtype=torch.float64), -lam]))
    dO = torch.randn_like(out)
    (out * dO).sum().backward()
    a2 = orc.causal_softmax(q2, k2, 1 / math.sqrt(hs))
    assert lam.grad.item() == pytest.approx(orc.dlambda_identity(dO, a2, v).item(), rel=1e-10)


def test_errors():
    with pytest.raises(RuntimeError):
        orc.ndiff_lambdas([], [], 1)
    sd = {}
    with pytest.raises(RuntimeError):
        orc.diff_head(torch.zeros(1, 9, 4), sd, 1, 8)


def test_lr_pins(golden_curve):
    # SURVEY section 8c measured these from the reference scheduler (train.py:95-107)
    pins = golden_curve["curve/lr_pins"]
    want = [0.0, 3.2e-7, 3.1968e-4, 3.2e-4, 1.95235e-4, 6e-5]
    for a, b in zip(pins, want):
        assert a == pytest.approx(b, rel=1e-4, abs=1e-12)


def test_flops_contract():
    f, fb = orc.flops_attention(8, 16, 4096, 64, 128, 2)
    assert f == pytest.approx(549.76e9, rel=1e-4)
    assert fb == pytest.approx(1099.51e9, rel=1e-4)
