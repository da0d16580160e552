"""Attention-map dropout (nn.Dropout on every softmax map: diff_transformer.py:66-67,
Ndiff_transformer.py:114, control.py:59) in the fused kernels.

The kernels draw the mask from a counter-based hash of (seed, b, h, i, q, k)
(include/diffattn.h, csrc/attn_kernels.h fmix32/drop_key/drop_mul), so the test
restates that hash in numpy, builds the masks, and runs the reference algorithm
in fp64 with those masks applied -- ``A_i -> A_i * m_i / (1-p)`` before the
combination -- forward and backward.  The reference draws its masks from torch's
Philox stream, which no other implementation reproduces bit for bit; the
contract that carries over is the distribution (independent Bernoulli(1-p) keep
per map element, kept values scaled by 1/(1-p)), checked statistically below.
"""
import math

import numpy as np
import pytest
import torch

from conftest import rel_err
from test_gpu_parity import TOL, DEV, _ops, _rope64
from oracle import diffattn_oracle as orc

pytestmark = pytest.mark.gpu

_M32 = np.uint64(0xFFFFFFFF)


def _fmix32(x):
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & _M32
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & _M32
    x ^= x >> np.uint64(16)
    return x


def drop_masks(seed, p, B, H, N, T):
    """(B, H, N, T, T) float64 multipliers m/(1-p) of the kernels' dropout."""
    lo, hi = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    thr = max(1, min(int(p * 2 ** 32), 2 ** 32 - 1))
    idx = np.arange(B * H * N, dtype=np.uint64)
    keys = _fmix32(lo ^ _fmix32((idx + hi) & _M32))
    q = np.arange(T, dtype=np.uint64)[:, None]
    k = np.arange(T, dtype=np.uint64)[None, :]
    qa = (q * np.uint64(0x9E3779B1)) & _M32
    kb = (k * np.uint64(0x7FEB352D)) & _M32
    out = np.empty((B * H * N, T, T), dtype=np.float64)
    scale = float(np.float32(1.0 / (1.0 - p)))
    for j, key in enumerate(keys):
        x = _fmix32(((key + qa) & _M32) ^ kb)
        out[j] = np.where(x >= thr, scale, 0.0)
    return torch.from_numpy(out.reshape(B, H, N, T, T))


def _oracle_dropped(qkv64, coef64, H, N, hs, dv, masks, freqs_c=None):
    B, T, _ = qkv64.shape
    nq = H * N * hs
    q = qkv64[..., :nq].view(B, T, H, N, hs)
    k = qkv64[..., nq:2 * nq].view(B, T, H, N, hs)
    v = qkv64[..., 2 * nq:].view(B, T, H, dv)
    outs = []
    for h in range(H):
        diff = None
        for i in range(N):
            qi, ki = q[:, :, h, i], k[:, :, h, i]
            if freqs_c is not None:
                qi, ki = _rope64(qi, freqs_c), _rope64(ki, freqs_c)
            a = orc.causal_softmax(qi, ki, 1.0 / math.sqrt(hs)) * masks[:, h, i]
            diff = a * coef64[h, i] if diff is None else diff + coef64[h, i] * a
        outs.append(diff @ v[:, :, h])
    return torch.cat(outs, dim=-1)


DROP_CASES = [  # H, N, hs, T, dv, rope, p
    (2, 2, 64, 129, 128, False, 0.1), (1, 3, 32, 200, 64, True, 0.3), (2, 4, 32, 97, 64, True, 0.1),
    (2, 2, 128, 130, 256, False, 0.5), (2, 1, 64, 150, 64, True, 0.1),     # the control model's N=1, dv=hs
    (1, 2, 64, 700, 128, False, 0.2),
    # branch-split forward (one branch per workgroup + combine) with the mask: N = 3 / 4 at hs = 64
    (2, 3, 64, 150, 128, True, 0.2), (1, 4, 64, 100, 128, False, 0.1),
    # backward in branch groups of two (head size >= 96, N = 3 / 4)
    (1, 3, 96, 120, 192, True, 0.2), (1, 4, 128, 90, 256, False, 0.1),
    # branch counts without an N-branch plan (branch-split forward, grouped backward: the
    # mask keys keep the call's branch index and count), a zero-padded head size
    (1, 5, 64, 130, 128, True, 0.2), (1, 6, 32, 100, 64, False, 0.1), (1, 2, 48, 90, 96, False, 0.2),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H,N,hs,T,dv,rope,p", DROP_CASES)
def test_dropout_matches_restated_masks(dtype, H, N, hs, T, dv, rope, p):
    ops = _ops()
    from differential_transformer_replication_amd import _lib
    assert ops.attention_supported(dtype, hs, N, dv)
    g = torch.Generator().manual_seed(7 * T + N)
    B, seed = 2, 0x1234_5678_9ABC + T
    W = ops.packed_width(H, N, hs, dv)
    qkv = torch.randn(B, T, W, generator=g)
    coef = torch.randn(H, N, generator=g) * 0.5
    coef[:, 0] = 1.0
    do = torch.randn(B, T, H * dv, generator=g)
    freqs_c = orc.precompute_freqs_cis(hs, T) if rope else None
    masks = drop_masks(seed, p, B, H, N, T)
    x64 = qkv.to(dtype).double().requires_grad_(True)
    c64 = coef.double().requires_grad_(True)
    ref = _oracle_dropped(x64, c64, H, N, hs, dv, masks, freqs_c)
    ref.backward(do.to(dtype).double())

    xg = qkv.to(dtype).to(DEV).requires_grad_(True)
    cg = coef.to(DEV).requires_grad_(True)
    freqs = torch.view_as_real(freqs_c[:T]).contiguous().to(DEV) if rope else None
    out = ops.diff_attention(xg, cg, H, N, hs, freqs, dv=dv, dropout_p=p, seed=seed)
    out.backward(do.to(dtype).to(DEV))
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert rel_err(out.float().cpu(), ref) < tol
    nq = H * N * hs
    gx = xg.grad.float().cpu()
    assert rel_err(gx[..., :nq], x64.grad[..., :nq]) < tol, "dQ"
    assert rel_err(gx[..., nq:2 * nq], x64.grad[..., nq:2 * nq]) < tol, "dK"
    assert rel_err(gx[..., 2 * nq:], x64.grad[..., 2 * nq:]) < tol, "dV"
    assert rel_err(cg.grad.cpu(), c64.grad) < tol, "dcoef"


def test_dropout_mask_statistics():
    """Keep rate 1-p within 5 sigma over every causal element, independent of
    branch (two branches' masks agree only at the rate of independent draws)."""
    p, B, H, N, T = 0.3, 2, 3, 2, 256
    m = drop_masks(987654321, p, B, H, N, T) > 0
    causal = torch.tril(torch.ones(T, T, dtype=torch.bool))
    n = int(causal.sum()) * B * H * N
    kept = float(m[..., causal].sum())
    assert abs(kept / n - (1 - p)) < 5 * math.sqrt(p * (1 - p) / n)
    both = float((m[:, :, 0] & m[:, :, 1])[..., causal].sum()) / (n // N)
    assert abs(both - (1 - p) ** 2) < 5 * math.sqrt((1 - p) ** 2 * (1 - (1 - p) ** 2) / (n // N))


def test_dropout_expectation_and_seeding():
    """Over many seeds the dropped output averages to the undropped one (the
    1/(1-p) scaling); one seed is deterministic; p = 0 is the plain kernel."""
    ops = _ops()
    H, N, hs, T, B = 1, 2, 64, 96, 1
    g = torch.Generator().manual_seed(3)
    W = ops.packed_width(H, N, hs, 2 * hs)
    qkv = torch.randn(B, T, W, generator=g).to(DEV)
    coef = torch.tensor([[1.0, -0.4]], device=DEV)
    base = ops.diff_attention(qkv, coef, H, N, hs)
    assert torch.equal(ops.diff_attention(qkv, coef, H, N, hs, dropout_p=0.0, seed=5), base)
    a = ops.diff_attention(qkv, coef, H, N, hs, dropout_p=0.2, seed=11)
    assert torch.equal(a, ops.diff_attention(qkv, coef, H, N, hs, dropout_p=0.2, seed=11))
    assert not torch.equal(a, ops.diff_attention(qkv, coef, H, N, hs, dropout_p=0.2, seed=12))
    acc = torch.zeros_like(base)
    n = 400
    for s in range(n):
        acc += ops.diff_attention(qkv, coef, H, N, hs, dropout_p=0.2, seed=1000 + s)
    # the rows with many keys average tightly; judge the later half
    assert rel_err((acc / n)[:, T // 2:].cpu(), base[:, T // 2:].cpu()) < 0.05


def test_modules_train_with_dropout():
    """Training-mode modules with dropout > 0 run the fused kernels (no fallback)
    and follow torch.manual_seed like the reference's nn.Dropout."""
    from differential_transformer_replication_amd import diff_transformer as D, Ndiff_transformer as ND
    from differential_transformer_replication_amd import control as C
    torch.manual_seed(0)
    mods = [D.MultiHeadDiffAttention(4, 32, 128, 0.1, 64), ND.MultiHeadAlternatingDiffAttention(2, 32, 64, 0.1, 64, 3),
            C.MultiHeadAttention(2, 64, 128, 0.1, 64)]
    for m in mods:
        m = m.to(DEV).train()
        C_ = m.proj.out_features
        x = torch.randn(2, 50, C_, device=DEV, requires_grad=True)
        call = (lambda x: m(x, 1)) if not isinstance(m, C.MultiHeadAttention) else m
        torch.manual_seed(5)
        y1 = call(x)
        torch.manual_seed(5)
        y2 = call(x)
        y3 = call(x)
        assert torch.equal(y1, y2) and not torch.equal(y1, y3)
        y1.square().sum().backward()
        assert torch.isfinite(x.grad).all()
        m.eval()
        with torch.no_grad():
            assert torch.equal(call(x), call(x))
