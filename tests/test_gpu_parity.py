"""GPU parity: the HIP kernels (through the C ABI) against the CPU oracle.

Tolerance (SURVEY section 4 norm, max|a-b|/max|b| per tensor; BASELINE.json
north_star): fp32 <= 1e-4, bf16/fp16 <= 2e-2, on outputs and every gradient.
"""
import math

import numpy as np
import pytest
import torch

from conftest import Golden, rel_err
from oracle import diffattn_oracle as orc

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 1e-4, torch.bfloat16: 2e-2, torch.float16: 2e-2}
DEV = "cuda"


def _ops():
    from differential_transformer_replication_amd import ops
    return ops


def _oracle_core(qkv64, coef64, H, N, hs, freqs_c=None):
    """Per-head oracle on the packed layout (CPU fp64)."""
    B, T, W = qkv64.shape
    dv = 2 * hs
    nq = H * N * hs
    q = qkv64[..., :nq].view(B, T, H, N, hs)
    k = qkv64[..., nq:2 * nq].view(B, T, H, N, hs)
    v = qkv64[..., 2 * nq:].view(B, T, H, dv)
    outs = []
    for h in range(H):
        qs = [q[:, :, h, i] for i in range(N)]
        ks = [k[:, :, h, i] for i in range(N)]
        if freqs_c is not None:
            qs = [_rope64(t, freqs_c) for t in qs]
            ks = [_rope64(t, freqs_c) for t in ks]
        outs.append(orc.diff_core(qs, ks, v[:, :, h], coef64[h]))
    return torch.cat(outs, dim=-1)


def _rope64(x, freqs_c):
    # fp64 restatement of apply_rotary_emb (the oracle's own is fp32 by definition)
    T = x.shape[1]
    ang = torch.view_as_real(freqs_c[:T]).double()
    c, s = ang[..., 0], ang[..., 1]
    a, b = x[..., 0::2], x[..., 1::2]
    out = torch.stack([a * c - b * s, a * s + b * c], dim=-1)
    return out.flatten(-2)


CASES = [  # H, N, hs, T, rope
    (2, 2, 64, 129, False), (1, 2, 16, 7, False), (3, 2, 32, 200, False), (2, 3, 64, 65, True),
    (2, 4, 32, 97, True), (1, 1, 64, 64, True), (2, 2, 128, 130, False), (1, 4, 64, 70, False),
    (2, 2, 64, 1, False), (1, 2, 64, 256, True),
    # long enough for the K/V ring to wrap many times under the staggered schedule
    (1, 2, 64, 1100, False), (1, 1, 64, 777, False), (1, 3, 32, 1500, True),
    # head size 96 (the reference's default TrainingConfig: train.py:60-61, diff_transformer.py:111),
    # N = 4 at head sizes 96 / 128 (dQ 32-key tiles, dK/dV row vectors from global memory)
    (2, 2, 96, 129, False), (1, 1, 96, 200, False), (1, 3, 96, 70, True), (1, 4, 96, 100, True),
    (1, 4, 128, 97, False), (1, 2, 96, 700, True), (1, 3, 128, 130, False),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,N,hs,T,rope", CASES)
def test_core_fwd_bwd(dtype, H, N, hs, T, rope):
    _core_case(dtype, H, N, hs, T, rope)


# Every built native 3- / 4-branch backward plan, forced by ABI 7's per-stage group caps
# (dta_attn_bwd_args.group_max_dq / group_max_dkdv = 4).  The library's defaults run
# 16-bit head sizes >= 64 as branch groups of two, so without the caps these plans -- one
# wave per SIMD, the largest register and LDS footprints -- would go unexercised.
NATIVE_CASES = [  # H, N, hs, T, rope
    (1, 3, 128, 130, False), (1, 4, 128, 97, False), (1, 3, 96, 70, True), (1, 4, 96, 100, True),
    (2, 3, 64, 65, True), (1, 4, 64, 70, False), (2, 3, 32, 200, False), (1, 4, 32, 97, True),
    (1, 3, 128, 700, True),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,N,hs,T,rope", NATIVE_CASES)
def test_core_native_backward_plans(dtype, H, N, hs, T, rope):
    with _ops().bwd_group_caps(4, 4):
        _core_case(dtype, H, N, hs, T, rope)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_native_hs128_n3_sampled_rows(dtype):
    """The native 16-bit (hs 128, N 3) backward plans at B=8, H=8, T=4096 (groups forced
    off): O, dQ, dK, dV, d(coef) on sampled rows of spread (b, h) pairs against fp64."""
    with _ops().bwd_group_caps(4, 4):
        _long_case(B=8, H=8, N=3, hs=128, T=4096, pairs=[(0, 0), (7, 7), (3, 5), (5, 2)], n_rows=24,
                   dtype=dtype, seed=71)


# ABI 7 dv_f32 = NULL at the default caps: dK/dV runs in branch groups (16-bit, head size 64,
# N = 3 / 4: groups of 2) and each later group reads, adds and re-stores the 16-bit dV itself
# (the per-lane read-add-store epilogue) instead of summing in the fp32 workspace.
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,N,hs,T,rope", [(2, 3, 64, 129, False), (1, 4, 64, 200, True), (1, 3, 128, 97, False)])
def test_core_dv_groups_without_f32_workspace(dtype, H, N, hs, T, rope):
    ops = _ops()
    from differential_transformer_replication_amd import _lib
    assert _lib.load().dta_attn_bwd_dkdv_groups(_lib.dtype_code(dtype), hs, N, 2 * hs, 0) > 1
    ops._DV_F32_WORKSPACE[0] = False
    try:
        _core_case(dtype, H, N, hs, T, rope)
    finally:
        ops._DV_F32_WORKSPACE[0] = True


# Head sizes above 128 (the reference takes any n_embd // (2 n_head), diff_transformer.py:111): the
# 16-bit head-size-256 plans, directly and zero-padded (160), N = 1..3 (the backward as single-branch
# groups), RoPE on some.
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,N,hs,T,rope", [(1, 2, 256, 70, False), (2, 1, 256, 97, True), (1, 3, 256, 65, True),
                                           (2, 2, 160, 130, True), (1, 2, 200, 40, False)])
def test_core_large_head_sizes(dtype, H, N, hs, T, rope):
    assert _ops().padded_head(dtype, hs, N, 2 * hs) == 256
    _core_case_any(dtype, H, N, hs, T, rope)


def _core_case_any(dtype, H, N, hs, T, rope):
    """_core_case through ops.diff_attention's padding (head sizes without their own plan)."""
    ops = _ops()
    g = torch.Generator().manual_seed(1000 * H + 100 * N + hs + T)
    B = 2
    W = ops.packed_width(H, N, hs, 2 * hs)
    qkv = torch.randn(B, T, W, generator=g)
    coef = torch.randn(H, N, generator=g) * 0.5
    coef[:, 0] = 1.0
    do = torch.randn(B, T, H * 2 * hs, generator=g)
    freqs_c = orc.precompute_freqs_cis(hs, max(T, 8)) if rope else None
    x64 = qkv.to(dtype).double().requires_grad_(True)
    c64 = coef.double().clone().requires_grad_(True)
    ref = _oracle_core(x64, c64, H, N, hs, freqs_c)
    ref.backward(do.to(dtype).double())
    xg = qkv.to(dtype).to(DEV).requires_grad_(True)
    cg = coef.to(DEV).requires_grad_(True)
    freqs = torch.view_as_real(freqs_c[:T]).contiguous().to(DEV) if rope else None
    out = ops.diff_attention(xg, cg, H, N, hs, freqs)
    out.backward(do.to(dtype).to(DEV))
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert rel_err(out.float().cpu(), ref) < tol
    nq = H * N * hs
    gx = xg.grad.float().cpu()
    for name, sl in (("dQ", slice(0, nq)), ("dK", slice(nq, 2 * nq)), ("dV", slice(2 * nq, None))):
        assert rel_err(gx[..., sl], x64.grad[..., sl]) < tol, name
    assert rel_err(cg.grad.cpu(), c64.grad) < tol, "dcoef"


# ABI 8 lse_c = NULL: the 16-bit key-major kernel without the |c_i| fold (the C ABI's other path;
# ops always passes the workspace), including negative and zero first coefficients.
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,N,hs,T,rope", [(2, 2, 64, 129, False), (2, 3, 64, 65, True), (1, 2, 128, 130, False)])
def test_core_without_lse_c(dtype, H, N, hs, T, rope):
    ops = _ops()
    ops._LSE_C_WORKSPACE[0] = False
    try:
        _core_case(dtype, H, N, hs, T, rope)
    finally:
        ops._LSE_C_WORKSPACE[0] = True


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("c0", [-0.7, 0.0])
def test_core_fold_signs(dtype, c0):
    """The |c_i| fold (ABI 8 lse_c) with a negative or zero first coefficient and mixed signs:
    dV's operand is formed relative to branch 0's sign, dK_i takes sign(c_i), c_i = 0 gives P~ = 0."""
    ops = _ops()
    H, N, hs, T, B = 3, 3, 64, 150, 2
    g = torch.Generator().manual_seed(77)
    W = ops.packed_width(H, N, hs, 2 * hs)
    qkv = torch.randn(B, T, W, generator=g)
    coef = torch.tensor([[c0, -0.4, 0.3], [c0, 0.5, -0.2], [1.0, 0.0, -0.6]])
    do = torch.randn(B, T, H * 2 * hs, generator=g)
    x64 = qkv.to(dtype).double().requires_grad_(True)
    c64 = coef.double().clone().requires_grad_(True)
    ref = _oracle_core(x64, c64, H, N, hs)
    ref.backward(do.to(dtype).double())
    xg = qkv.to(dtype).to(DEV).requires_grad_(True)
    cg = coef.to(DEV).requires_grad_(True)
    out = ops.diff_attention(xg, cg, H, N, hs)
    out.backward(do.to(dtype).to(DEV))
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert rel_err(out.float().cpu(), ref) < tol
    nq = H * N * hs
    gx = xg.grad.float().cpu()
    for name, sl in (("dQ", slice(0, nq)), ("dK", slice(nq, 2 * nq)), ("dV", slice(2 * nq, None))):
        assert rel_err(gx[..., sl], x64.grad[..., sl]) < tol, name
    assert rel_err(cg.grad.cpu(), c64.grad) < tol, "dcoef"


# ABI 6 obr_dtype = fp16 (ops: DTA_OBR_F16=1, 16-bit activations): O_i stored as fp16 for the
# backward's delta_i.  The forward's epilogue then keeps its per-lane stores (the LDS bounce
# takes fp32 O_i only), so this also covers that path; parity against fp64 at the usual bar.
OBR16_CASES = [(2, 2, 64, 129, False), (2, 3, 64, 65, True), (1, 2, 128, 130, False), (1, 4, 32, 97, True)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,N,hs,T,rope", OBR16_CASES)
def test_core_fp16_branch_outputs(dtype, H, N, hs, T, rope, monkeypatch):
    monkeypatch.setenv("DTA_OBR_F16", "1")
    assert _ops()._obr_dtype(dtype) == torch.float16
    _core_case(dtype, H, N, hs, T, rope)


def _core_case(dtype, H, N, hs, T, rope):
    ops = _ops()
    from differential_transformer_replication_amd import _lib
    assert _lib.supported(dtype, hs, N, 2 * hs)      # every case runs (natively or in branch groups)
    g = torch.Generator().manual_seed(1000 * H + 100 * N + hs + T)
    B = 2
    W = ops.packed_width(H, N, hs, 2 * hs)
    qkv = torch.randn(B, T, W, generator=g)
    coef = torch.randn(H, N, generator=g) * 0.5
    coef[:, 0] = 1.0
    do = torch.randn(B, T, H * 2 * hs, generator=g)
    freqs_c = orc.precompute_freqs_cis(hs, max(T, 8)) if rope else None
    # quantise inputs to the kernel dtype so both sides see identical values
    qkv_q = qkv.to(dtype).double()
    do_q = do.to(dtype).double()
    x64 = qkv_q.clone().requires_grad_(True)
    c64 = coef.double().clone().requires_grad_(True)
    ref = _oracle_core(x64, c64, H, N, hs, freqs_c)
    ref.backward(do_q)

    xg = qkv.to(dtype).to(DEV).requires_grad_(True)
    cg = coef.to(DEV).requires_grad_(True)
    freqs = torch.view_as_real(freqs_c[:T]).contiguous().to(DEV) if rope else None
    out = ops.diff_attention(xg, cg, H, N, hs, freqs)
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


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_forced_rescale(dtype):
    """The deferred online-softmax rescale (taken only when a row's running max
    grows by more than 2^8 inside a block) is rare on random data, so force it
    (cdna_hip_programming.md 5.4 rule 26): one key of branch 0 aligned with every
    query makes that branch's max jump by ~10 (log2 units) at a late tile."""
    ops = _ops()
    H, N, hs, T, B = 2, 2, 64, 900, 1
    g = torch.Generator().manual_seed(7)
    W = ops.packed_width(H, N, hs, 2 * hs)
    nq = H * N * hs
    qkv = torch.randn(B, T, W, generator=g) * 0.3
    u = torch.ones(hs) / math.sqrt(hs)
    q = qkv[..., :nq].view(B, T, H, N, hs)
    k = qkv[..., nq:2 * nq].view(B, T, H, N, hs)
    q[:, :, :, 0] += 2.0 * u
    # branch-0 score of key 700 ~ 60/sqrt(hs) = 7.5 for every query: a jump of ~10 (log2 units)
    # over the running max, with P(key 700) ~ 0.7 -- not saturated, so dS = P(dP - delta) stays
    # well conditioned
    k[:, 700, :, 0] = 30.0 * u
    k[:, 333, 1, 1] = -40.0 * u           # a large negative outlier in the other branch
    coef = torch.tensor([[1.0, -0.4], [1.0, -0.6]])
    do = torch.randn(B, T, H * 2 * hs, generator=g)
    qkv_q = qkv.to(dtype).double()
    x64 = qkv_q.clone().requires_grad_(True)
    c64 = coef.double().clone().requires_grad_(True)
    ref = _oracle_core(x64, c64, H, N, hs)
    ref.backward(do.to(dtype).double())
    xg = qkv.to(dtype).to(DEV).requires_grad_(True)
    cg = coef.to(DEV).requires_grad_(True)
    out = ops.diff_attention(xg, cg, H, N, hs)
    out.backward(do.to(dtype).to(DEV))
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert rel_err(out.float().cpu(), ref) < tol
    gx = xg.grad.float().cpu()
    for name, sl in (("dQ", slice(0, nq)), ("dK", slice(nq, 2 * nq)), ("dV", slice(2 * nq, None))):
        assert rel_err(gx[..., sl], x64.grad[..., sl]) < tol, name
    assert rel_err(cg.grad.cpu(), c64.grad) < tol, "dcoef"


# growth of branch 0's row maximum past its first key tile ~ jump / 4 * log2(e) log2 units
GROWTH_JUMPS = [30.0, 55.0, 85.0, 125.0, 200.0, 4000.0]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("jump", GROWTH_JUMPS)
def test_forward_max_growth(dtype, jump):
    """The 16-bit forward keeps each row's reference maximum fixed after the first key
    tile (no per-tile maximum), so a P packed for the PV product may exceed 1 by as much
    as the row maximum grew; a workgroup whose P could leave the operand type's range
    re-runs on the per-tile-maximum path (fp16: a lane's tile sum above 2^15 < 65504;
    bf16: above 2^60).  Growth: jump 30 ~ +11 log2 units (fixed-reference path everywhere),
    55 / 85 / 125 ~ +20 / +31 / +45 (fp16 re-runs, bf16 stays: P up to 2^45 in bf16),
    200 ~ +72 (re-run), 4000 (exp2 overflows fp32: re-run).  The paired N = 2 plan (cfg2's);
    forward output against the fp64 oracle, every row finite."""
    ops = _ops()
    H, N, hs, T, B = 2, 2, 64, 900, 1
    g = torch.Generator().manual_seed(11)
    W = ops.packed_width(H, N, hs, 2 * hs)
    nq = H * N * hs
    qkv = torch.randn(B, T, W, generator=g) * 0.3
    u = torch.ones(hs) / math.sqrt(hs)
    q = qkv[..., :nq].view(B, T, H, N, hs)
    k = qkv[..., nq:2 * nq].view(B, T, H, N, hs)
    q[:, :, :, 0] += 2.0 * u
    k[:, 700, :, 0] = jump * u
    coef = torch.tensor([[1.0, -0.4], [1.0, -0.6]])
    x64 = qkv.to(dtype).double()
    ref = _oracle_core(x64, coef.double(), H, N, hs)
    out = ops.diff_attention(qkv.to(dtype).to(DEV), coef.to(DEV), H, N, hs).float().cpu()
    assert torch.isfinite(out).all()
    assert rel_err(out, ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [48, 384, 2048, 4104])
def test_group_ln_scale(dtype, C):
    ops = _ops()
    g = torch.Generator().manual_seed(C)
    x = torch.randn(3, 37, C, generator=g) * 3 + 1
    w = 1 + 0.1 * torch.randn(1, 1, C, generator=g)
    b = 0.1 * torch.randn(1, 1, C, generator=g)
    dy = torch.randn(3, 37, C, generator=g)
    xq = x.to(dtype).double().requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    b64 = b.double().requires_grad_(True)
    ref = orc.group_layer_norm(xq, w64, b64) * (1 - torch.tensor(0.8).double())
    ref.backward(dy.to(dtype).double())
    xg = x.to(dtype).to(DEV).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    bg = b.to(DEV).requires_grad_(True)
    out = ops.group_ln_scale(xg, wg, bg, 1e-5, float(1 - torch.tensor(0.8)))
    out.backward(dy.to(dtype).to(DEV))
    tol = TOL[dtype]
    assert rel_err(out.float().cpu(), ref) < tol
    assert rel_err(xg.grad.float().cpu(), xq.grad) < tol
    assert rel_err(wg.grad.cpu(), w64.grad) < tol
    assert rel_err(bg.grad.cpu(), b64.grad) < tol


def test_rope_kernel_matches_reference_fixture(golden):
    """dta_rope (fp32) bitwise-close to the reference apply_rotary_emb fixture."""
    from differential_transformer_replication_amd import _lib
    lib = _lib.load()
    fc = torch.view_as_complex(torch.from_numpy(golden["rope/freqs"]).contiguous())
    x = torch.from_numpy(golden["rope/x"])                      # (2, 17, 32)
    want = torch.from_numpy(golden["rope/out"])
    B, T, hs = x.shape
    src = x.view(B, T, 1, 1, hs).to(DEV)
    dst = torch.empty_like(src)
    freqs = torch.view_as_real(fc[:T]).contiguous().to(DEV)
    a = _lib.RopeArgs(_lib.DTA_F32, B, T, 1, 1, hs, 0, 0, _lib.tensor5(src), _lib.tensor5(dst), freqs.data_ptr())
    _lib.check(lib.dta_rope(a, _lib.stream_handle(src.device)))
    torch.cuda.synchronize()
    assert (dst.view(B, T, hs).cpu() - want).abs().max().item() < 1e-6


# ---- full-length shapes, checked on sampled query rows ----------------------------------
def _sample_rows(T, n, seed):
    fixed = [0, 1, 31, 32, 63, 64, 127, 128, 255, 256, 511, 512, T // 2 - 1, T // 2, T - 65, T - 64, T - 2, T - 1]
    g = torch.Generator().manual_seed(seed)
    rnd = torch.randint(0, T, (n,), generator=g).tolist()
    return sorted({r for r in fixed + rnd if 0 <= r < T})


def _rows_reference(q, k, v, coef, rows, do_rows, freqs_c=None):
    """fp64 restatement of diff_core (diff_transformer.py:57-72 / Ndiff_transformer.py:
    102-125) for the query rows ``rows`` of ONE (b, h) over the full key range.
    q, k: (T, N, hs); v: (T, dv); coef (N,); do_rows (R, dv).  Returns out_R and the
    gradients of sum(out_R * do_R) w.r.t. q (rows only), k, v and coef -- equal to the
    full problem's gradients when dO is zero on every other row.  With ``freqs_c`` every
    Q_i / K_i is rotated first (apply_rotary_emb, Ndiff_transformer.py:11-22, 104-109) and
    the gradients are w.r.t. the unrotated projections, as the kernels return them."""
    T, N, hs = k.shape
    q = q.double().requires_grad_(True)
    k = k.double().requires_grad_(True)
    v = v.double().requires_grad_(True)
    c = coef.double().requires_grad_(True)
    qr, kr = q, k
    if freqs_c is not None:
        qr = _rope64(q.transpose(0, 1), freqs_c).transpose(0, 1)      # (N, T, hs) rows -> (T, N, hs)
        kr = _rope64(k.transpose(0, 1), freqs_c).transpose(0, 1)
    r = torch.tensor(rows)
    keep = torch.arange(T)[None, :] <= r[:, None]                       # causal: key <= query
    out = 0
    for i in range(N):
        s = (qr[r, i] @ kr[:, i].t()) / math.sqrt(hs)
        a = torch.softmax(s.masked_fill(~keep, float("-inf")), dim=-1)
        out = out + c[i] * (a @ v)
    (out * do_rows.double()).sum().backward()
    return out.detach(), q.grad, k.grad, v.grad, c.grad


def _rows_reference_bf16(q, k, v, coef, rows, do_rows):
    """The reference algorithm itself under bf16 autocast (diff_transformer.py:57-72 with
    train.py's autocast, here bf16): scores from a bf16 matmul, scaled in bf16, softmax in
    fp32, the fp32 combination cast to bf16 for @V -- on the same rows as _rows_reference
    (no RoPE).  Returns (out_R, dQ_R, dK, dV, dcoef)."""
    T, N, hs = k.shape
    q = q.to(torch.bfloat16).requires_grad_(True)
    k = k.to(torch.bfloat16).requires_grad_(True)
    v = v.to(torch.bfloat16).requires_grad_(True)
    c = coef.float().requires_grad_(True)
    r = torch.tensor(rows)
    keep = torch.arange(T)[None, :] <= r[:, None]
    diff = 0
    for i in range(N):
        s = (q[r, i] @ k[:, i].t()) * hs ** -0.5
        a = torch.softmax(s.masked_fill(~keep, float("-inf")).float(), dim=-1)
        diff = diff + c[i] * a
    out = diff.to(torch.bfloat16) @ v
    (out.float() * do_rows.float()).sum().backward()
    return out.detach(), q.grad[r], k.grad, v.grad, c.grad


def _long_case(B, H, N, hs, T, pairs, n_rows, dtype=torch.bfloat16, seed=0, rope=False, dv=None, qk_scale=1.0,
               ref_bar=False):
    """Sampled-row parity of a full-length shape.  ``dv``: value width (2 hs; hs for the
    control model's N = 1 plans).  ``qk_scale`` multiplies Q and K (large logits).
    ``ref_bar``: each tensor's bar is max(tol, 2x the reference algorithm's own error under
    bf16 autocast on the same rows, _rows_reference_bf16) instead of tol."""
    ops = _ops()
    freqs_c = orc.precompute_freqs_cis(hs, T) if rope else None
    freqs = torch.view_as_real(freqs_c).contiguous().to(DEV) if rope else None
    dv = 2 * hs if dv is None else dv
    W = ops.packed_width(H, N, hs, dv)
    nq = H * N * hs
    g = torch.Generator(device=DEV).manual_seed(seed)
    qkv = torch.randn(B, T, W, device=DEV, generator=g)
    qkv[..., :2 * nq] *= qk_scale
    qkv = qkv.to(dtype)
    coef = torch.randn(H, N, device=DEV, generator=g) * 0.5
    if N > 1:
        coef[:, 0] = 1.0
    else:
        coef.fill_(1.0)
    do = torch.zeros(B, T, H, dv, device=DEV, dtype=dtype)
    rows = {}
    for j, (b, h) in enumerate(pairs):
        rows[(b, h)] = _sample_rows(T, n_rows, seed + j)
        r = torch.tensor(rows[(b, h)], device=DEV)
        do[b, r, h] = torch.randn(len(r), dv, device=DEV, generator=g).to(dtype)
    xg = qkv.clone().requires_grad_(True)
    cg = coef.clone().requires_grad_(True)
    out = ops.diff_attention(xg, cg, H, N, hs, freqs, dv)
    out.backward(do.view(B, T, H * dv))
    torch.cuda.synchronize()
    tol = TOL[dtype]
    out = out.view(B, T, H, dv)
    gx = xg.grad
    for (b, h), rr in rows.items():
        x = qkv[b].float().cpu()
        q = x[:, :nq].view(T, H, N, hs)[:, h]
        k = x[:, nq:2 * nq].view(T, H, N, hs)[:, h]
        v = x[:, 2 * nq:].view(T, H, dv)[:, h]
        d_r = do[b, rr, h].float().cpu()
        o_ref, dq_ref, dk_ref, dv_ref, dc_ref = _rows_reference(q, k, v, coef[h].cpu(), rr, d_r, freqs_c)
        bars = dict.fromkeys(("O", "dQ", "dK", "dV", "dcoef"), tol)
        if ref_bar:
            alg = _rows_reference_bf16(q, k, v, coef[h].cpu(), rr, d_r)
            for name, a_, r_ in zip(bars, alg, (o_ref, dq_ref[rr], dk_ref, dv_ref, dc_ref)):
                bars[name] = max(tol, 2.0 * rel_err(a_, r_))
        where = f"b={b} h={h}"
        assert rel_err(out[b, rr, h].float().cpu(), o_ref) < bars["O"], "O " + where
        gb = gx[b].float().cpu()
        dq = gb[:, :nq].view(T, H, N, hs)[:, h]
        assert rel_err(dq[rr], dq_ref[rr]) < bars["dQ"], "dQ " + where
        others = torch.ones(T, dtype=torch.bool)
        others[rr] = False
        assert dq[others].abs().max().item() == 0.0, "dQ nonzero on rows with dO = 0 " + where
        assert rel_err(gb[:, nq:2 * nq].view(T, H, N, hs)[:, h], dk_ref) < bars["dK"], "dK " + where
        assert rel_err(gb[:, 2 * nq:].view(T, H, dv)[:, h], dv_ref) < bars["dV"], "dV " + where
        assert rel_err(cg.grad[h].cpu(), dc_ref) < bars["dcoef"], "dcoef " + where


def test_cfg5_long_context_sampled_rows():
    """BASELINE configs[4]: causal T=32768, hs=128 (dv=256), N=2, bf16 -- the hs=128
    plan's long K/V ring and its LSE over 32k keys, against fp64 on 48+ rows per head."""
    _long_case(B=1, H=2, N=2, hs=128, T=32768, pairs=[(0, 0), (0, 1)], n_rows=48)


def test_cfg5_control_long_context_sampled_rows():
    """bench.py's cfg5 comparison leg, control.py's standard attention on the fused kernels
    (N = 1, hs = dv = 128, coefficient 1) at T = 32768, bf16: O, dQ, dK, dV on sampled rows
    of two heads against fp64 (control.py:38-63)."""
    _long_case(B=1, H=2, N=1, hs=128, T=32768, pairs=[(0, 0), (0, 1)], n_rows=48, seed=51, dv=128)


@pytest.mark.parametrize("N", [2, 3])
def test_large_logits_sampled_rows(N):
    """Scores with |S * scale * log2e| up to ~30 (Q and K x2.5; trained models reach such
    logits): the backward recomputes P from the forward's LSE through its own bf16
    operands (sl2-prescaled Q or K), so the bars are 2x the reference algorithm's own
    bf16-autocast error on the same rows (at least 2e-2).  cfg2's paired N = 2 plan and
    the N = 3 branch-split one."""
    _long_case(B=1, H=2, N=N, hs=64, T=4096, pairs=[(0, 0), (0, 1)], n_rows=40, seed=61 + N, qk_scale=2.5,
               ref_bar=True)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("jump", [55.0, 85.0, 125.0])
def test_forward_max_growth_branch_split(dtype, jump):
    """test_forward_max_growth on the branch-split N = 1 plan at cfg3's shape (B=2, H=6,
    hs=64, N=3, T=2048) with RoPE on: branch 0's key 700 lies along the two slowest RoPE
    pairs, so the spike survives the rotation for every later query (growth ~ +20 / +31 /
    +45 log2 units).  Forward rows (most past the spike) against fp64; all finite."""
    ops = _ops()
    B, H, N, hs, T = 2, 6, 3, 64, 2048
    g = torch.Generator().manual_seed(int(jump))
    W = ops.packed_width(H, N, hs, 2 * hs)
    nq = H * N * hs
    qkv = torch.randn(B, T, W, generator=g) * 0.3
    u = torch.zeros(hs)
    u[-4:] = 0.5                                # unit vector over the two slowest pairs
    q = qkv[..., :nq].view(B, T, H, N, hs)
    k = qkv[..., nq:2 * nq].view(B, T, H, N, hs)
    q[:, :, :, 0] += 2.0 * u
    k[:, 700, :, 0] = jump * u
    qkv = qkv.to(dtype)
    coef = torch.tensor([[1.0, -0.5, 0.3]]).repeat(H, 1) + 0.05 * torch.randn(H, N, generator=g)
    freqs_c = orc.precompute_freqs_cis(hs, T)
    freqs = torch.view_as_real(freqs_c).contiguous().to(DEV)
    out = ops.diff_attention(qkv.to(DEV), coef.to(DEV), H, N, hs, freqs).float().cpu().view(B, T, H, 2 * hs)
    assert torch.isfinite(out).all()
    rows = sorted(set(_sample_rows(T, 24, int(jump))) | {699, 700, 701, 1000, 2047})
    x = qkv.float()
    for b, h in [(0, 0), (1, 5), (0, 3)]:
        qb = x[b, :, :nq].view(T, H, N, hs)[:, h]
        kb = x[b, :, nq:2 * nq].view(T, H, N, hs)[:, h]
        vb = x[b, :, 2 * nq:].view(T, H, 2 * hs)[:, h]
        o_ref = _rows_reference(qb, kb, vb, coef[h], rows, torch.zeros(len(rows), 2 * hs), freqs_c)[0]
        assert rel_err(out[b, rows, h], o_ref) < TOL[dtype], (b, h)


def test_cfg2_full_shape_sampled_rows():
    """BASELINE configs[1] at its full shape (B=8, H=16, hs=64, T=4096, bf16), checked on
    sampled rows of (b, h) pairs spread over the grid (first, last, middle)."""
    pairs = [(0, 0), (7, 15), (3, 7), (5, 2), (1, 12), (6, 9)]
    _long_case(B=8, H=16, N=2, hs=64, T=4096, pairs=pairs, n_rows=40, seed=11)


def test_ndiff_long_sampled_rows():
    """N=4 at T=8192 (hs=64): the N-term plan over a long ring."""
    _long_case(B=1, H=2, N=4, hs=64, T=8192, pairs=[(0, 0), (0, 1)], n_rows=32, seed=5)


@pytest.mark.parametrize("N", [3, 4])
def test_cfg3_shape_rope_sampled_rows(N):
    """BASELINE configs[2]'s attention shape (hs=64, T=2048, H=6, bf16) with RoPE on, as
    the N-diff model always runs it: the forward rotation pass and the inverse rotation
    in the dQ / dK epilogues over a ring that wraps T/64 times; N=3 takes the full-dv
    forward plan, N=4 the dv-chunked one.  O, dQ, dK, dV and d(coef) on sampled rows of
    (b, h) pairs spread over B=2 x H=6 against fp64."""
    pairs = [(0, 0), (1, 5), (0, 3), (1, 2)]
    _long_case(B=2, H=6, N=N, hs=64, T=2048, pairs=pairs, n_rows=40, seed=30 + N, rope=True)


def test_cfg2_shape_rope_sampled_rows():
    """N=2 hs=64 at T=4096 with RoPE (the control-model / rotated path at the cfg2 shape)."""
    _long_case(B=1, H=4, N=2, hs=64, T=4096, pairs=[(0, 0), (0, 3)], n_rows=32, seed=41, rope=True)


def test_backward_reductions_are_reproducible():
    """d(coef) (hence the lambda grads) and GroupLayerNorm dw/db are summed from
    partials in a fixed order, not by float atomics: two backward passes over the
    same inputs agree bitwise."""
    ops = _ops()
    H, N, hs, T, B = 4, 2, 64, 777, 2
    g = torch.Generator().manual_seed(21)
    W = ops.packed_width(H, N, hs, 2 * hs)
    qkv = torch.randn(B, T, W, generator=g).to(torch.bfloat16).to(DEV)
    coef = (torch.randn(H, N, generator=g) * 0.5).to(DEV)
    do = torch.randn(B, T, H * 2 * hs, generator=g).to(torch.bfloat16).to(DEV)
    w = (1 + 0.1 * torch.randn(1, 1, H * 2 * hs, generator=g)).to(DEV)
    b = (0.1 * torch.randn(1, 1, H * 2 * hs, generator=g)).to(DEV)
    grads = []
    for _ in range(2):
        xg = qkv.clone().requires_grad_(True)
        cg = coef.clone().requires_grad_(True)
        wg, bg = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        out = ops.group_ln_scale(ops.diff_attention(xg, cg, H, N, hs), wg, bg, 1e-5, 0.2)
        out.backward(do)
        torch.cuda.synchronize()
        grads.append([t.grad.clone() for t in (xg, cg, wg, bg)])
    for a, b_ in zip(*grads):
        assert torch.equal(a, b_)


@pytest.mark.parametrize("rows", [1, 9, 513, 5003])
@pytest.mark.parametrize("dtype,C", [(torch.bfloat16, 2048), (torch.float32, 256), ("mixed", 1024)])
def test_ln_bwd_row_ring_ragged(rows, dtype, C):
    """The LayerNorm backward's register ring (three row groups in flight for rows up to 2048
    columns, round 6) and its one-launch ordered dw/db reduce at row counts that leave the
    ring part-filled: fewer rows than workgroups, 513 (the 512-workgroup cap plus one), and
    5003 (~9.8 rows per workgroup).  "mixed": fp32 x normalised into bf16 y, bf16 dy
    (dta_ln_args.io_dtype, the Blocks' LayerNorm under autocast).  Against fp64 torch
    (diff_transformer.py:15-20 restated), and dw / db bitwise reproducible run to run."""
    ops = _ops()
    g = torch.Generator().manual_seed(rows * 7 + C)
    x = torch.randn(rows, C, generator=g) * 2 + 0.5
    w = 1 + 0.1 * torch.randn(C, generator=g)
    b = 0.1 * torch.randn(C, generator=g)
    dy = torch.randn(rows, C, generator=g)
    xdt = torch.float32 if dtype == "mixed" else dtype
    ydt = torch.bfloat16 if dtype == "mixed" else dtype
    xq = x.to(xdt).double().requires_grad_(True)
    w64, b64 = w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = orc.group_layer_norm(xq, w64, b64) * 0.2
    ref.backward(dy.to(ydt).double())
    grads = []
    for _ in range(2):
        xg = x.to(xdt).to(DEV).requires_grad_(True)
        wg, bg = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
        out = ops._GroupLNScale.apply(xg, wg, bg, 1e-5, 0.2, None, ydt if dtype == "mixed" else None)
        assert out.dtype == ydt
        out.backward(dy.to(ydt).to(DEV))
        grads.append((wg.grad.clone(), bg.grad.clone()))
    tol = TOL[torch.bfloat16] if ydt == torch.bfloat16 else TOL[torch.float32]
    assert rel_err(out.float().cpu(), ref) < tol
    assert rel_err(xg.grad.float().cpu(), xq.grad) < tol
    assert rel_err(wg.grad.cpu(), w64.grad) < tol
    assert rel_err(bg.grad.cpu(), b64.grad) < tol
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])
