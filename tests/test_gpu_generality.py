"""Shapes the reference accepts beyond the built N-branch kernel plans.

The reference takes any ``n_terms >= 1`` (Ndiff_transformer.py:40-126) and any head size
``n_embd // (2 n_head)`` (diff_transformer.py:111), in any dtype -- its ``estimate_loss``
runs fp32 with no autocast (train.py:124-138).  Here:

- a branch count without an N-branch plan (N >= 5; fp32 N = 3 / 4 at head sizes 96 / 128)
  runs as branch groups that have one (csrc/capi.hip): the forward as N single-branch
  workgroups plus a run-time-N combine, the backward group by group, dV summed over the
  groups, d(coef) reduced over all N;
- a head size without its own plan (up to 128; 129-256 in 16-bit on the head-size-256 plans)
  runs zero-padded in the next built one (ops.padded_head): zero Q_i / K_i columns leave every
  score unchanged, zero V columns add output columns that are dropped.

Checked against the fp64 oracle at the north star's tolerances (fp32 1e-4, bf16 2e-2).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err
from oracle import diffattn_oracle as orc
from test_gpu_parity import TOL, DEV, _ops, _oracle_core, _rope64

pytestmark = pytest.mark.gpu


def _core_case(dtype, H, N, hs, T, rope, dv=None, B=2, seed=0):
    ops = _ops()
    dv = 2 * hs if dv is None else dv
    g = torch.Generator().manual_seed(seed + 1000 * N + hs + T)
    W = ops.packed_width(H, N, hs, dv)
    qkv = torch.randn(B, T, W, generator=g)
    coef = torch.randn(H, N, generator=g) * 0.5
    coef[:, 0] = 1.0
    do = torch.randn(B, T, H * dv, generator=g)
    freqs_c = orc.precompute_freqs_cis(hs, max(T, 8)) if rope else None
    x64 = qkv.to(dtype).double().requires_grad_(True)
    c64 = coef.double().requires_grad_(True)
    if dv == 2 * hs:
        ref = _oracle_core(x64, c64, H, N, hs, freqs_c)
    else:                                       # standard attention (control.py:38-63): N = 1, dv = hs
        nq = H * hs
        q = x64[..., :nq].view(B, T, H, hs)
        k = x64[..., nq:2 * nq].view(B, T, H, hs)
        v = x64[..., 2 * nq:].view(B, T, H, dv)
        outs = []
        for h in range(H):
            qh, kh = q[:, :, h], k[:, :, h]
            if rope:
                qh, kh = _rope64(qh, freqs_c), _rope64(kh, freqs_c)
            outs.append(c64[h, 0] * (orc.causal_softmax(qh, kh, 1.0 / math.sqrt(hs)) @ v[:, :, h]))
        ref = torch.cat(outs, dim=-1)
    ref.backward(do.to(dtype).double())
    xg = qkv.to(dtype).to(DEV).requires_grad_(True)
    cg = coef.to(DEV).requires_grad_(True)
    freqs = torch.view_as_real(freqs_c[:T]).contiguous().to(DEV) if rope else None
    out = ops.diff_attention(xg, cg, H, N, hs, freqs, dv)
    out.backward(do.to(dtype).to(DEV))
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert out.shape == (B, T, H * dv)
    assert rel_err(out.float().cpu(), ref) < tol, "O"
    nq = H * N * hs
    gx = xg.grad.float().cpu()
    assert rel_err(gx[..., :nq], x64.grad[..., :nq]) < tol, "dQ"
    assert rel_err(gx[..., nq:2 * nq], x64.grad[..., nq:2 * nq]) < tol, "dK"
    assert rel_err(gx[..., 2 * nq:], x64.grad[..., 2 * nq:]) < tol, "dV"
    assert rel_err(cg.grad.cpu(), c64.grad) < tol, "dcoef"


GROUP_CASES = [  # H, N, hs, T, rope
    (2, 5, 64, 130, True), (1, 6, 32, 97, False), (1, 8, 16, 70, True), (2, 5, 128, 66, False),
    (1, 7, 96, 90, True), (1, 5, 64, 700, False),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,N,hs,T,rope", GROUP_CASES)
def test_any_branch_count(dtype, H, N, hs, T, rope):
    """N >= 5 (no N-branch plan): branch-split forward + grouped backward vs fp64."""
    from differential_transformer_replication_amd import _lib
    assert _lib.supported(dtype, hs, N, 2 * hs)
    _core_case(dtype, H, N, hs, T, rope)


@pytest.mark.parametrize("N,hs,rope", [(3, 96, True), (4, 96, False), (3, 128, True), (4, 128, False),
                                       (2, 128, True)])
def test_fp32_n_diff_plans(N, hs, rope):
    """fp32 at head sizes 96 / 128 with N = 2..4 (the reference's fp32 eval of the N-diff
    model, train.py:124-138): grouped where no fp32 N-branch plan is built."""
    from differential_transformer_replication_amd import _lib
    assert _lib.supported(torch.float32, hs, N, 2 * hs)
    _core_case(torch.float32, 1, N, hs, 150, rope)


PAD_CASES = [  # H, N, hs, T, rope, dv_is_hs
    (2, 2, 8, 65, False, False), (1, 2, 24, 100, True, False), (2, 2, 48, 129, False, False),
    (1, 3, 80, 70, True, False), (1, 2, 100, 90, False, False), (1, 5, 40, 80, True, False),
    (2, 1, 16, 77, True, True), (1, 1, 48, 100, True, True), (1, 1, 72, 64, False, True),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H,N,hs,T,rope,std", PAD_CASES)
def test_padded_head_sizes(dtype, H, N, hs, T, rope, std):
    """Head sizes without their own plan (8, 24, 40, 48, 72, 80, 100; the control model's
    dv = hs at 16 / 48 / 72) on the zero-padded plan of the next built head size."""
    ops = _ops()
    dv = hs if std else 2 * hs
    hp = ops.padded_head(dtype, hs, N, dv)
    assert hp is not None and hp > hs
    _core_case(dtype, H, N, hs, T, rope, dv=dv)


def test_head_size_limits_raise():
    """Head sizes 129-256 run in 16-bit on the head-size-256 plans (test_gpu_parity.py
    test_core_large_head_sizes); fp32 differential plans stop at 128 and nothing goes past 256."""
    ops = _ops()
    x = torch.zeros(1, 4, ops.packed_width(1, 2, 136, 272), device=DEV)
    with pytest.raises(RuntimeError, match="no gfx950 kernel"):
        ops.diff_attention(x, torch.ones(1, 2, device=DEV), 1, 2, 136)
    x = torch.zeros(1, 4, ops.packed_width(1, 2, 264, 528), device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="no gfx950 kernel"):
        ops.diff_attention(x, torch.ones(1, 2, device=DEV), 1, 2, 264)


def _oracle_alternating_transformer(sd, idx, tgt, n_head, n_layer, n_terms, block):
    """AlternatingDiffTransformer.forward (Ndiff_transformer.py:212-230) with Block.forward
    (:176-179) and SwiGLU (:148-158) on the oracle's attention restatement: token
    embeddings only (RoPE inside every head), 1-based layer index."""
    B, T = idx.shape
    C_ = sd["ln_f.weight"].shape[0]
    x = sd["token_embedding_table.weight"][idx]
    for i in range(n_layer):
        p = f"blocks.{i}."
        h = F.layer_norm(x, (C_,), sd[p + "ln1.weight"], sd[p + "ln1.bias"], 1e-5)
        x = x + orc.multihead_alternating_diff_attention(h, sd, n_head, n_terms, i + 1, block, prefix=p + "diff_attn.")
        h = F.layer_norm(x, (C_,), sd[p + "ln2.weight"], sd[p + "ln2.bias"], 1e-5)
        gate = F.silu(F.linear(h, sd[p + "ffwd.0.linear_gate.weight"], sd[p + "ffwd.0.linear_gate.bias"]))
        xf = F.linear(h, sd[p + "ffwd.0.linear_xform.weight"], sd[p + "ffwd.0.linear_xform.bias"])
        x = x + F.linear(gate * xf, sd[p + "ffwd.1.weight"], sd[p + "ffwd.1.bias"])
    x = F.layer_norm(x, (C_,), sd["ln_f.weight"], sd["ln_f.bias"], 1e-5)
    logits = F.linear(x, sd["lm_head.weight"], sd["lm_head.bias"])
    V = logits.shape[-1]
    return logits.view(B * T, V), F.cross_entropy(logits.view(B * T, V), tgt.view(B * T))


@pytest.mark.parametrize("n_terms", [3, 4, 5])
def test_alternating_transformer_fp32_eval(n_terms):
    """AlternatingDiffTransformer(12000, 768, 4, 2, 512, 0.0, n_terms) in fp32 eval mode
    under no_grad -- what the reference's estimate_loss runs (train.py:124-138) for the
    N-diff models of train.py:213-221 (head size 96) -- logits and loss vs the fp64 oracle."""
    from differential_transformer_replication_amd import Ndiff_transformer as ND
    torch.manual_seed(n_terms)
    m = ND.AlternatingDiffTransformer(12000, 768, 4, 2, 512, 0.0, n_terms=n_terms)
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "lambda_" in n:
                p.copy_(torch.randn(p.shape, generator=g) * 0.1)
    full = m.state_dict()
    sd = {k: (v.double() if v.is_floating_point() else v) for k, v in full.items()   # freqs_cis stays complex64
          if not k.endswith("tril") and not k.endswith("lambda_init")}
    idx = torch.randint(0, 12000, (2, 256), generator=g)
    tgt = torch.randint(0, 12000, (2, 256), generator=g)
    with torch.no_grad():
        ref_logits, ref_loss = _oracle_alternating_transformer(sd, idx, tgt, 4, 2, n_terms, 512)
    m = m.to(DEV).eval()
    with torch.no_grad():
        logits, loss = m(idx.to(DEV), tgt.to(DEV))
    torch.cuda.synchronize()
    assert logits.dtype == torch.float32
    assert rel_err(logits.cpu(), ref_logits) < 1e-4
    assert abs(float(loss) - float(ref_loss)) < 1e-4 * abs(float(ref_loss))
