"""Incremental decoding for ``generate``.

The reference's ``generate`` (diff_transformer.py:177-185; the same loop in
Ndiff_transformer.py and control.py:163-171) runs a full forward over
``idx[:, -block_size:]`` for every new token and keeps only the last row of
logits.  Here the first call runs the
prompt once through the fused training kernels (prefill) and keeps every
layer's K_i / V rows in a KV cache; each further token costs one projection row
per layer and one ``dta_attn_decode`` launch (``ops.diff_attention_decode``)
instead of a T x T recompute.

Positions are absolute within the window (learned position table in
DiffTransformer, RoPE rows in AlternatingDiffTransformer and the control
StandardTransformer, which runs as N = 1 with dv = hs), so once the sequence
outgrows ``block_size`` the window slides, every cached row changes position,
and the step falls back to the reference's own full recompute of the cropped
window.  Sampling (softmax of the last logits, ``torch.multinomial``) is the
reference's, so with the same generator state the tokens match the
full-recompute path whenever the logits agree to sampling precision.
``DTA_KV_CACHE=0`` selects the full-recompute loop.  Decode steps replay one
captured HIP graph of the whole model step (the position lives on the device,
``dta_attn_decode`` reads its length there); ``DTA_DECODE_GRAPH=0`` launches
them eagerly instead.
"""
from __future__ import annotations

import os
from typing import Dict

import torch
from torch.nn import functional as F

from . import ops
from ._compat import mha_out_scale

__all__ = ["KVCache", "DecodeGraph", "DevicePosition", "cached_generate", "enabled"]


def enabled(idx: torch.Tensor, model=None) -> bool:
    if not idx.is_cuda or os.environ.get("DTA_KV_CACHE", "1") == "0":
        return False
    if model is not None:
        # the prefill runs on the fused kernels (ops.diff_attention: any built or padded head
        # size, any branch count); the decode kernel takes head sizes % 8 up to 128, N <= 4
        _, _, N, hs, dv, _ = _spec(model.blocks[0])
        return (ops.attention_supported(model.lm_head.weight.dtype, hs, N, dv) and N <= 4 and hs % 8 == 0
                and hs <= 128)
    return True


class KVCache:
    """Per-layer packed rows ``[K (H, N, hs) | V (H, dv)]`` of every cached position:
    (B, block_size, H*N*hs + H*dv) in the projection's dtype, allocated once."""

    def __init__(self):
        self.rows: Dict[int, torch.Tensor] = {}
        self.length = 0
        # parameters do not change inside generate(): the packed projection weight,
        # the branch coefficients and the RoPE table are built once per layer
        self.consts: Dict[int, tuple] = {}
        self.graph = None
        self.use_graph = os.environ.get("DTA_DECODE_GRAPH", "1") != "0"

    def layer(self, layer: int, B: int, cap: int, width: int, like: torch.Tensor) -> torch.Tensor:
        buf = self.rows.get(layer)
        if buf is None or buf.shape != (B, cap, width) or buf.dtype != like.dtype:
            buf = torch.empty(B, cap, width, device=like.device, dtype=like.dtype)
            self.rows[layer] = buf
        return buf


def _spec(block):
    """(attention module, H, N, hs, dv, block_size) of a Block: the differential
    MHAs (dv = 2hs), or control.py's standard MHA as N = 1, dv = hs."""
    if hasattr(block, "diff_attn"):
        a = block.diff_attn
        return a, a.num_heads, getattr(a, "n_terms", 2), a.head_size, 2 * a.head_size, a.block_size
    a = block.attn
    return a, a.num_heads, 1, a.head_size, a.head_size, a.heads[0].block_size


def _constants(attn, layer: int, H: int, hs: int, bs: int, device):
    freqs = None
    if hasattr(attn.heads[0], "freqs_cis"):
        from .Ndiff_transformer import rope_table
        freqs = rope_table(attn.heads[0].freqs_cis, bs, hs).to(device=device, dtype=torch.float32).contiguous()
    if hasattr(attn, "coefficients"):
        return attn.packed_weight(), attn.coefficients(layer), freqs
    # control.py MultiHeadAttention: packed [Q | K | V], one branch of weight 1
    return attn.packed_weight(), torch.ones(H, 1, device=device, dtype=torch.float32), freqs


def _attention_step(block, x: torch.Tensor, layer: int, cache: KVCache, pos: int) -> torch.Tensor:
    """The block's attention forward (MultiHead(Alternating)DiffAttention, or
    control.py's MultiHeadAttention) for the rows at positions pos .. pos+Tn-1,
    reading and extending the layer's cache."""
    attn, H, N, hs, dv, bs = _spec(block)
    consts = cache.consts.get(layer)
    if consts is None:
        consts = _constants(attn, layer, H, hs, bs, x.device)
        cache.consts[layer] = consts
    weight, coef, freqs = consts
    rope = freqs is not None
    qkv = F.linear(x, weight)
    B, Tn, W = qkv.shape
    nq = H * N * hs
    buf = cache.layer(layer, B, bs, W - nq, qkv)
    k_rows = buf[..., :nq].unflatten(-1, (H, N, hs))
    if pos == 0:
        # prefill: the prompt through the training kernels, then cache its K_i / V rows
        out = ops.diff_attention(qkv, coef, H, N, hs, None if freqs is None else freqs[:Tn], dv)
        src = qkv[..., nq:2 * nq].unflatten(-1, (H, N, hs))
        if rope:
            ops.rope_rows(src, k_rows[:, :Tn], freqs[:Tn])
        else:
            k_rows[:, :Tn].copy_(src)
        buf[:, :Tn, nq:].copy_(qkv[..., 2 * nq:])
    else:
        if Tn != 1:
            raise RuntimeError("decode steps take one new position at a time")
        dev = isinstance(pos, DevicePosition)
        q = qkv[:, :, :nq].unflatten(-1, (H, N, hs))               # (B, 1, H, N, hs)
        k_new = qkv[:, :, nq:2 * nq].unflatten(-1, (H, N, hs))
        v_new = qkv[:, :, 2 * nq:].unflatten(-1, (H, dv))
        v_rows = buf[..., nq:].unflatten(-1, (H, dv))
        if rope:
            tab = freqs.index_select(0, pos.idx) if dev else freqs[pos:pos + 1]
            q_rot, k_rot = torch.empty_like(q), torch.empty_like(k_new)
            ops.rope_rows(q, q_rot, tab)
            ops.rope_rows(k_new, k_rot, tab)
            q, k_new = q_rot, k_rot
        if dev:                                   # graph-replayable: position read on the device
            k_rows.index_copy_(1, pos.idx, k_new)
            v_rows.index_copy_(1, pos.idx, v_new)
            out = ops.diff_attention_decode(q[:, 0], k_rows, v_rows, coef, bs, pos.length)
        else:
            k_rows[:, pos:pos + 1].copy_(k_new)
            v_rows[:, pos:pos + 1].copy_(v_new)
            out = ops.diff_attention_decode(q[:, 0], k_rows, v_rows, coef, pos + 1)
        out = out.view(B, 1, H * dv)
    if hasattr(attn, "group_norm"):
        gn = attn.group_norm
        out = ops.group_ln_scale(out, gn.weight, gn.bias, gn.eps, mha_out_scale(attn.lambda_init))
    return attn.dropout(attn.proj(out))


class DevicePosition:
    """The decode position held on the device (index and index + 1), so one
    captured graph replays for every position."""

    def __init__(self, device):
        self.idx = torch.zeros(1, dtype=torch.long, device=device)
        self.length = torch.ones(1, dtype=torch.int32, device=device)

    def set(self, p: int) -> None:
        self.idx.fill_(p)
        self.length.fill_(p + 1)


class DecodeGraph:
    """One decode step (every layer, Tn = 1) captured as a HIP graph: per token the
    host issues two fills and one graph launch instead of ~15 launches per layer."""

    def __init__(self, model, cache: "KVCache", B: int, device):
        self.tok = torch.zeros(B, 1, dtype=torch.long, device=device)
        self.pos = DevicePosition(device)
        # warm-up (allocator, cached constants) writes cache row block_size-1 only,
        # which is rewritten before it is ever read
        self.pos.set(model.block_size - 1)
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            _model_step(model, self.tok, cache, self.pos)
        torch.cuda.current_stream(device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.logits = _model_step(model, self.tok, cache, self.pos)

    def step(self, tok: torch.Tensor, p: int) -> torch.Tensor:
        self.tok.copy_(tok)
        self.pos.set(p)
        self.graph.replay()
        return self.logits.clone()


def _model_step(model, idx: torch.Tensor, cache: KVCache, pos: int) -> torch.Tensor:
    """The model's forward (diff_transformer.py:154-175 / Ndiff_transformer.py) over
    positions pos .. pos+T-1 of the window; returns the last row of logits."""
    T = idx.shape[1]
    x = model.token_embedding_table(idx)
    if hasattr(model, "position_embedding_table"):
        rows = pos.idx if isinstance(pos, DevicePosition) else torch.arange(pos, pos + T, device=idx.device)
        x = x + model.position_embedding_table(rows)
    for layer, block in enumerate(model.blocks, 1):
        x = x + _attention_step(block, block.ln1(x), layer, cache, pos)
        x = x + block.ffwd(block.ln2(x))
    return model.lm_head(model.ln_f(x[:, -1:]))[:, -1]


def last_logits(model, idx: torch.Tensor, cache: KVCache) -> torch.Tensor:
    """Logits of the newest position of ``idx``, reusing ``cache`` when the window
    has not slid (exposed for the parity tests)."""
    bs = model.block_size
    if cache.length == 0 or idx.shape[1] > bs or idx.shape[1] != cache.length + 1:
        cond = idx[:, -bs:]
        cache.length = 0
        logits = _model_step(model, cond, cache, 0)
        cache.length = cond.shape[1] if idx.shape[1] < bs else 0    # a full window slides next step
        return logits
    if cache.use_graph:
        if cache.graph is None:
            cache.graph = DecodeGraph(model, cache, idx.shape[0], idx.device)
        logits = cache.graph.step(idx[:, -1:], cache.length)
    else:
        logits = _model_step(model, idx[:, -1:], cache, cache.length)
    cache.length += 1
    if cache.length >= bs:
        cache.length = 0
    return logits


@torch.no_grad()
def cached_generate(model, idx: torch.Tensor, max_new_tokens: int) -> torch.Tensor:
    cache = KVCache()
    for _ in range(max_new_tokens):
        probs = F.softmax(last_logits(model, idx, cache), dim=-1)
        idx = torch.cat((idx, torch.multinomial(probs, num_samples=1)), dim=1)
    return idx
