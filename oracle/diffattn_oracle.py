"""CPU restatement of the reference's differential-attention hot path.

TEST INFRASTRUCTURE ONLY.  This module is the parity checker: only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it.  The product path (``differential_transformer_replication_amd``)
never imports, calls or falls back to anything in here.

It restates, in eager PyTorch on the CPU, what the reference computes, one
reference op for one oracle op (per-head Python loop, materialised T x T maps,
``masked_fill(-inf)`` then ``softmax``), in whatever float dtype the caller
passes (fp64 for golden checks, fp32 for the timed CPU baseline).  Every
function cites the reference line range it follows
(``/root/reference/<file>:<lines>``).

Pinning: ``tests/test_oracle_golden.py`` checks every function here against
vectors produced by running the reference modules themselves
(``tests/golden/make_golden.py``); the oracle is therefore "pinned", not
"parity unpinned".

Everything is functional: weights arrive as a ``state_dict``-shaped mapping so
the same fixtures drive both the oracle and the product modules.
"""
from __future__ import annotations

import math
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

LN_EPS = 1e-5               # diff_transformer.py:9 / Ndiff_transformer.py:27
MHA_LAMBDA_INIT = 0.8       # diff_transformer.py:86 (never updated -> x0.2)


# ---------------------------------------------------------------- norms ---
def group_layer_norm(x: Tensor, weight: Tensor, bias: Tensor, eps: float = LN_EPS) -> Tensor:
    """LayerNorm over the whole concatenated width C' = H*2hs.

    Follows diff_transformer.py:15-20 (duplicated at Ndiff_transformer.py:33-38):
    mean, biased variance, ``(x-mean)/sqrt(var+eps)``, then ``*w + b``.
    Not per head and not RMS (SURVEY semantic 1).
    """
    mean = x.mean(dim=-1, keepdim=True)
    var = x.var(dim=-1, keepdim=True, unbiased=False)
    y = (x - mean) / (var + eps).sqrt()
    return y * weight + bias


# --------------------------------------------------------------- lambdas ---
def lambda_init_for_layer(layer_idx: int, dtype=torch.float32) -> Tensor:
    """``0.8 - 0.6*exp(-0.3*(l-1))`` computed in fp32 (diff_transformer.py:42-43)."""
    li = torch.tensor(layer_idx, dtype=torch.float32)
    return (0.8 - 0.6 * torch.exp(-0.3 * (li - 1.0))).to(dtype)


def diff_lambda(lq1: Tensor, lk1: Tensor, lq2: Tensor, lk2: Tensor, layer_idx: int) -> Tensor:
    """Scalar lambda of one DiffHead (diff_transformer.py:41-48).

    Elementwise products and a mean -- not a dot product (SURVEY semantic 3).
    """
    init = lambda_init_for_layer(layer_idx, lq1.dtype)
    lam = torch.exp(lq1 * lk1) - torch.exp(lq2 * lk2) + init
    return lam.mean()


def ndiff_lambdas(lqs: Sequence[Tensor], lks: Sequence[Tensor], layer_idx: int) -> Tensor:
    """(N,) lambdas of one AlternatingDiffHead (Ndiff_transformer.py:79-93)."""
    if len(lqs) == 0:
        # Ndiff_transformer.py:93 torch.stack([]) raises for n_terms=0
        raise RuntimeError("stack expects a non-empty TensorList")
    init = lambda_init_for_layer(layer_idx, lqs[0].dtype)
    out = []
    for i in range(len(lqs)):
        term = torch.exp(lqs[i] * lks[i])
        if i > 0:
            term = term - torch.exp(lqs[i - 1] * lks[i - 1])
        out.append((term + init).mean())
    return torch.stack(out)


def ndiff_coefficients(lams: Tensor) -> Tensor:
    """Signed map weights ``[+l0, -l1, +l2, -l3, ...]`` (Ndiff_transformer.py:118-123)."""
    signs = torch.tensor([1.0 if i % 2 == 0 else -1.0 for i in range(lams.shape[0])],
                         dtype=lams.dtype, device=lams.device)
    return lams * signs


# ------------------------------------------------------------------ RoPE ---
def precompute_freqs_cis(dim: int, end: int, theta: float = 10000.0) -> Tensor:
    """complex64 (end, dim/2) table (Ndiff_transformer.py:4-9, control.py:4-9)."""
    j = torch.arange(0, dim, 2)[: dim // 2].float()
    inv = 1.0 / (theta ** (j / dim))
    ang = torch.outer(torch.arange(end, device=inv.device).float(), inv)
    return torch.polar(torch.ones_like(ang), ang)


def apply_rotary_emb(x: Tensor, freqs_cis: Tensor) -> Tensor:
    """Rotate interleaved pairs (x[2j], x[2j+1]) in fp32, cast back
    (Ndiff_transformer.py:11-22)."""
    xc = torch.view_as_complex(x.float().reshape(*x.shape[:-1], -1, 2))
    rot = xc * freqs_cis[: x.shape[1], :].unsqueeze(0)
    return torch.view_as_real(rot).flatten(-2).type_as(x)


# ------------------------------------------------------------ attention ---
_TRIL: Dict[Tuple[int, str], Tensor] = {}


def _tril(T: int, device) -> Tensor:
    """The reference's persistent fp32 ``tril`` buffer (diff_transformer.py:31),
    built once per size (and device) like a registered buffer, not per call."""
    key = (T, str(device))
    t = _TRIL.get(key)
    if t is None:
        t = _TRIL[key] = torch.tril(torch.ones(T, T, dtype=torch.float32, device=device))
    return t


def causal_softmax(q: Tensor, k: Tensor, scale: float) -> Tensor:
    """``softmax(masked_fill(q k^T * scale, tril[:T,:T]==0, -inf))`` for (B,T,d)
    inputs (diff_transformer.py:57-65): the ``== 0`` compare runs every call, as in
    the reference; the buffer itself is persistent."""
    T = q.shape[1]
    att = (q @ k.transpose(-2, -1)) * scale
    att = att.masked_fill(_tril(T, att.device)[:T, :T] == 0, float("-inf"))
    return F.softmax(att, dim=-1)


def diff_core(qs: Sequence[Tensor], ks: Sequence[Tensor], v: Tensor, coeffs: Tensor,
              freqs_cis: Optional[Tensor] = None) -> Tensor:
    """Kernel-level contract: ``O = sum_i coeffs[i] * A_i @ V``.

    ``qs[i], ks[i]``: (B,T,hs); ``v``: (B,T,dv); ``coeffs``: (N,) already
    signed.  With ``freqs_cis`` the maps use RoPE'd Q/K (Ndiff_transformer.py:
    102-125); without, they are DiffHead's maps (diff_transformer.py:57-72, where
    coeffs = [1, -lambda]).  The combination order follows the reference:
    ``diff = c0*A0; diff = diff + c_i*A_i`` then ``diff @ v``.
    """
    hs = qs[0].shape[-1]
    scale = 1.0 / (hs ** 0.5)
    diff = None
    for i in range(len(qs)):
        q, k = qs[i], ks[i]
        if freqs_cis is not None:
            q = apply_rotary_emb(q, freqs_cis)
            k = apply_rotary_emb(k, freqs_cis)
        a = causal_softmax(q, k, scale)
        diff = a * coeffs[i] if diff is None else diff + coeffs[i] * a
    return diff @ v


def _check_len(T: int, block_size: int) -> None:
    # the reference fails with a broadcast RuntimeError when T > block_size
    # (tril[:T,:T] is smaller than the T x T map) -- SURVEY semantic 9
    if T > block_size:
        raise RuntimeError(f"sequence length {T} exceeds block_size {block_size}")


def diff_head(x: Tensor, sd: Mapping[str, Tensor], layer_idx: int, block_size: int,
              prefix: str = "") -> Tensor:
    """One DiffHead forward (diff_transformer.py:50-73)."""
    _check_len(x.shape[1], block_size)
    p = prefix
    k1 = x @ sd[p + "key1.weight"].t()
    q1 = x @ sd[p + "query1.weight"].t()
    k2 = x @ sd[p + "key2.weight"].t()
    q2 = x @ sd[p + "query2.weight"].t()
    v = x @ sd[p + "value.weight"].t()
    lam = diff_lambda(sd[p + "lambda_q1"], sd[p + "lambda_k1"],
                      sd[p + "lambda_q2"], sd[p + "lambda_k2"], layer_idx)
    scale = 1.0 / (k1.shape[-1] ** 0.5)
    a1 = causal_softmax(q1, k1, scale)
    a2 = causal_softmax(q2, k2, scale)
    return (a1 - lam * a2) @ v


def multihead_diff_attention(x: Tensor, sd: Mapping[str, Tensor], n_head: int,
                             layer_idx: int, block_size: int, prefix: str = "") -> Tensor:
    """MultiHeadDiffAttention forward (diff_transformer.py:88-93): per-head loop,
    cat, GroupLayerNorm, x(1-0.8), proj."""
    p = prefix
    outs = [diff_head(x, sd, layer_idx, block_size, f"{p}heads.{h}.") for h in range(n_head)]
    y = torch.cat(outs, dim=-1)
    y = group_layer_norm(y, sd[p + "group_norm.weight"], sd[p + "group_norm.bias"])
    # the MHA's own lambda_init buffer is 0.8 forever (SURVEY semantic 2), in the module dtype
    y = y * (1 - torch.tensor(MHA_LAMBDA_INIT).to(x.dtype))   # fp32 buffer cast to module dtype
    return y @ sd[p + "proj.weight"].t() + sd[p + "proj.bias"]


def alternating_diff_head(x: Tensor, sd: Mapping[str, Tensor], n_terms: int, layer_idx: int,
                          block_size: int, prefix: str = "") -> Tensor:
    """AlternatingDiffHead forward (Ndiff_transformer.py:95-126)."""
    _check_len(x.shape[1], block_size)
    p = prefix
    hs = sd[p + "value.weight"].shape[0] // 2
    v = x @ sd[p + "value.weight"].t()
    qs = [x @ sd[f"{p}queries.{i}.weight"].t() for i in range(n_terms)]
    ks = [x @ sd[f"{p}keys.{i}.weight"].t() for i in range(n_terms)]
    lams = ndiff_lambdas([sd[f"{p}lambda_qs.{i}"] for i in range(n_terms)],
                         [sd[f"{p}lambda_ks.{i}"] for i in range(n_terms)], layer_idx)
    freqs = sd.get(p + "freqs_cis")
    if freqs is None:
        freqs = precompute_freqs_cis(hs, block_size)
    return diff_core(qs, ks, v, ndiff_coefficients(lams), freqs_cis=freqs)


def multihead_alternating_diff_attention(x: Tensor, sd: Mapping[str, Tensor], n_head: int,
                                         n_terms: int, layer_idx: int, block_size: int,
                                         prefix: str = "") -> Tensor:
    """MultiHeadAlternatingDiffAttention forward (Ndiff_transformer.py:144-149)."""
    p = prefix
    outs = [alternating_diff_head(x, sd, n_terms, layer_idx, block_size, f"{p}heads.{h}.")
            for h in range(n_head)]
    y = torch.cat(outs, dim=-1)
    y = group_layer_norm(y, sd[p + "group_norm.weight"], sd[p + "group_norm.bias"])
    # the MHA's own lambda_init buffer is 0.8 forever (SURVEY semantic 2), in the module dtype
    y = y * (1 - torch.tensor(MHA_LAMBDA_INIT).to(x.dtype))   # fp32 buffer cast to module dtype
    return y @ sd[p + "proj.weight"].t() + sd[p + "proj.bias"]


def control_head(x: Tensor, sd: Mapping[str, Tensor], block_size: int, prefix: str = "") -> Tensor:
    """Standard causal head with RoPE (control.py:38-63)."""
    _check_len(x.shape[1], block_size)
    p = prefix
    k = x @ sd[p + "key.weight"].t()
    q = x @ sd[p + "query.weight"].t()
    v = x @ sd[p + "value.weight"].t()
    freqs = sd.get(p + "freqs_cis")
    if freqs is None:
        freqs = precompute_freqs_cis(k.shape[-1], block_size)
    k = apply_rotary_emb(k, freqs)
    q = apply_rotary_emb(q, freqs)
    a = causal_softmax(q, k, 1.0 / (k.shape[-1] ** 0.5))
    return a @ v


def control_multihead(x: Tensor, sd: Mapping[str, Tensor], n_head: int, block_size: int,
                      prefix: str = "") -> Tensor:
    """control.py:75-78."""
    p = prefix
    y = torch.cat([control_head(x, sd, block_size, f"{p}heads.{h}.") for h in range(n_head)], -1)
    return y @ sd[p + "proj.weight"].t() + sd[p + "proj.bias"]


# ------------------------------------------------- backward identities ---
def dlambda_identity(dO: Tensor, a2: Tensor, v: Tensor) -> Tensor:
    """SURVEY semantic 5: dL/dlambda = -<dO, A2 @ V> summed over (b,t,c)."""
    return -(dO * (a2 @ v)).sum()


def flops_attention(B: int, H: int, T: int, hs: int, dv: int, n_terms: int) -> Tuple[float, float]:
    """Algorithmic causal-halved matmul FLOPs:
    F_fwd = B*H*T^2*(N*hs + dv), F_bwd = 2*F_fwd."""
    f = float(B) * H * T * T * (n_terms * hs + dv)
    return f, 2.0 * f
