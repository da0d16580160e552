"""Control model surface (reference ``control.py``): standard causal softmax
attention with RoPE, the comparison baseline.

The per-head projections are packed into one GEMM.  On the GPU the causal
attention runs on the SAME fused gfx950 kernels as the differential models, as
their N=1 case (one branch, coefficient 1, value width dv = hs; SURVEY 8(f) item
2), so config 5 compares like with like -- attention-map dropout included (the
kernels' counter-based mask, include/diffattn.h).  Two cases keep PyTorch's
``scaled_dot_product_attention`` instead: CPU tensors (the control model is not
the hot path and stays runnable on the host) and head sizes without a dv = hs
plan (head sizes above 128).
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn import functional as F

from . import kv_cache, ops
from ._compat import emit_tril_hooks, check_seq_len, attn_dropout_p
from .packing import ensure_packed, packed_linear
from .Ndiff_transformer import precompute_freqs_cis, apply_rotary_emb, rope_table

__all__ = ["precompute_freqs_cis", "apply_rotary_emb", "Head", "MultiHeadAttention", "SwiGLU", "Block",
           "StandardTransformer"]


def _fused_ok(x: torch.Tensor, p: float, hs: int) -> bool:
    # the fused kernels' standard-attention plans (dv = hs: head sizes 32, 64, 96, 128, 256, and
    # every other head size up to 256 zero-padded to one of them, ops.padded_head);
    # x.dtype is the projection's dtype under autocast too
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    return x.is_cuda and 0.0 <= p < 1.0 and ops.attention_supported(dt, hs, 1, hs)


def _fused_attention(qkv: torch.Tensor, H: int, hs: int, freqs_cis: torch.Tensor, p: float = 0.0) -> torch.Tensor:
    """qkv (B, T, 3*H*hs) packed [Q | K | V] -> (B, T, H*hs): RoPE + causal softmax
    attention with map dropout p (control.py:38-63) as the fused kernel's N=1, coef 1,
    dv=hs case."""
    T = qkv.shape[1]
    coef = torch.ones(H, 1, device=qkv.device, dtype=torch.float32)
    return ops.diff_attention(qkv, coef, H, 1, hs, rope_table(freqs_cis, T, hs), dv=hs, dropout_p=p)


def _rope_fp32(x: torch.Tensor, freqs_cis: torch.Tensor) -> torch.Tensor:
    # x (B, H, T, hs); interleaved pairs rotated in fp32 then cast back (control.py:11-22)
    T = x.shape[2]
    xc = torch.view_as_complex(x.float().reshape(*x.shape[:-1], -1, 2))
    return torch.view_as_real(xc * freqs_cis[:T].to(x.device)).flatten(-2).type_as(x)


class Head(nn.Module):
    """One RoPE causal head (control.py:24-63)."""

    def __init__(self, head_size, n_embd, dropout, block_size):
        super().__init__()
        self.key = nn.Linear(n_embd, head_size, bias=False)
        self.query = nn.Linear(n_embd, head_size, bias=False)
        self.value = nn.Linear(n_embd, head_size, bias=False)
        self.block_size = block_size
        self.head_size = head_size
        emit_tril_hooks(self, block_size)
        self.dropout = nn.Dropout(dropout)
        self.register_buffer("freqs_cis", precompute_freqs_cis(head_size, block_size))

    def forward(self, x):
        check_seq_len(x.shape[1], self.block_size)
        p = self.dropout.p if self.training else 0.0
        if _fused_ok(x, p, self.head_size):
            w = torch.cat([self.query.weight, self.key.weight, self.value.weight], 0)
            return _fused_attention(F.linear(x, w), 1, self.head_size, self.freqs_cis, p)
        q = _rope_fp32(self.query(x)[:, None], self.freqs_cis)
        k = _rope_fp32(self.key(x)[:, None], self.freqs_cis)
        v = self.value(x)[:, None]
        out = F.scaled_dot_product_attention(q, k, v, is_causal=True, dropout_p=p,
                                             scale=1.0 / (self.head_size ** 0.5))
        return out[:, 0]


class MultiHeadAttention(nn.Module):
    """control.py:64-78 with the H per-head projections packed into one GEMM."""

    def __init__(self, num_heads, head_size, n_embd, dropout, block_size):
        super().__init__()
        self.heads = nn.ModuleList([Head(head_size, n_embd, dropout, block_size) for _ in range(num_heads)])
        self.proj = nn.Linear(head_size * num_heads, n_embd)
        self.dropout = nn.Dropout(dropout)
        self.num_heads = num_heads
        self.head_size = head_size
        self._pack = {}                            # the shared storage of the heads' projections

    def packed_params(self):
        return ([h.query.weight for h in self.heads] + [h.key.weight for h in self.heads]
                + [h.value.weight for h in self.heads])

    def packed_weight(self) -> torch.Tensor:
        return ensure_packed(self.packed_params(), self._pack)

    def forward(self, x):
        B, T, _ = x.shape
        check_seq_len(T, self.heads[0].block_size)
        H, hs = self.num_heads, self.head_size
        qkv = packed_linear(x, self.packed_params(), self._pack)
        fc = self.heads[0].freqs_cis
        p = attn_dropout_p([h.dropout for h in self.heads], self.training)
        if _fused_ok(x, p, hs):
            out = _fused_attention(qkv, H, hs, fc, p)
        else:
            q, k, v = qkv.view(B, T, 3, H, hs).permute(2, 0, 3, 1, 4)
            q, k = _rope_fp32(q, fc), _rope_fp32(k, fc)
            out = F.scaled_dot_product_attention(q, k, v, is_causal=True, dropout_p=p, scale=1.0 / (hs ** 0.5))
            out = out.transpose(1, 2).reshape(B, T, H * hs)
        return self.dropout(ops.linear(out, self.proj))


class SwiGLU(nn.Module):
    """silu(W_g x) * (W_x x)  (control.py SwiGLU).  On the GPU the two Linears run as one
    GEMM over shared weight / bias packs (ops.packed_swiglu)."""

    def __init__(self, size_in, size_out):
        super().__init__()
        self.linear_gate = nn.Linear(size_in, size_out)
        self.linear_xform = nn.Linear(size_in, size_out)
        self._wpack = {}                           # shared storage of [W_gate; W_xform]
        self._bpack = {}                           # ... and of [b_gate; b_xform]

    def param_packs(self):
        """(holder, params) of the shared-storage groups (dp.BucketedAllReduce)."""
        g, x = self.linear_gate, self.linear_xform
        return [(self._wpack, [g.weight, x.weight]), (self._bpack, [g.bias, x.bias])]

    def forward(self, x):
        return ops.packed_swiglu(x, self.linear_gate, self.linear_xform, self._wpack, self._bpack)


class Block(nn.Module):
    """control.py:92-111 (head_size = n_embd // n_head)."""

    def __init__(self, n_embd, n_head, block_size, dropout):
        super().__init__()
        self.attn = MultiHeadAttention(n_head, n_embd // n_head, n_embd, dropout, block_size)
        self.ffwd = nn.Sequential(SwiGLU(n_embd, 4 * n_embd), nn.Linear(4 * n_embd, n_embd), nn.Dropout(dropout))
        self.ln1 = ops.LayerNorm(n_embd, autocast_out=True)
        self.ln2 = ops.LayerNorm(n_embd, autocast_out=True)

    def forward(self, x):
        # the residual add and ln2 in one pass on the GPU (ops.add_layer_norm)
        x, h = ops.add_layer_norm(x, self.attn(self.ln1(x)), self.ln2)
        return x + ops.ffn(self.ffwd, h)

    def forward_chained(self, x, h, next_ln):
        """forward() given h = ln1(x), returning (x_out, next_ln(x_out)): both residual
        adds fused with the LayerNorm that follows them (the model's block loop)."""
        x, h = ops.add_layer_norm(x, self.attn(h), self.ln2)
        return ops.add_layer_norm(x, ops.ffn(self.ffwd, h), next_ln)


class StandardTransformer(nn.Module):
    """control.py:113-171."""

    def __init__(self, vocab_size, n_embd, n_head, n_layer, block_size, dropout):
        super().__init__()
        self.block_size = block_size
        self.token_embedding_table = nn.Embedding(vocab_size, n_embd)
        self.blocks = nn.ModuleList([Block(n_embd, n_head, block_size, dropout) for _ in range(n_layer)])
        self.ln_f = ops.LayerNorm(n_embd, autocast_out=True)
        self.lm_head = nn.Linear(n_embd, vocab_size)
        self.apply(self._init_weights)

    def _init_weights(self, module):
        if isinstance(module, (nn.Linear, nn.Embedding)):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
            if isinstance(module, nn.Linear) and module.bias is not None:
                nn.init.zeros_(module.bias)

    def forward(self, idx, targets=None):
        B, T = idx.shape
        x = self.token_embedding_table(idx)
        # the block loop with every residual add fused into the LayerNorm after it
        n = len(self.blocks)
        h = self.blocks[0].ln1(x) if n else self.ln_f(x)
        for i, block in enumerate(self.blocks):
            x, h = block.forward_chained(x, h, self.blocks[i + 1].ln1 if i + 1 < n else self.ln_f)
        logits = self.lm_head(h)
        loss = None
        if targets is not None:
            logits = logits.view(B * T, -1)             # reference returns (B*T, V) with targets
            loss = F.cross_entropy(logits, targets.view(B * T))
        return logits, loss

    @torch.no_grad()
    def generate(self, idx, max_new_tokens):
        if kv_cache.enabled(idx, self):                  # KV-cache decode
            return kv_cache.cached_generate(self, idx, max_new_tokens)
        for _ in range(max_new_tokens):
            logits, _ = self(idx[:, -self.block_size:])
            probs = F.softmax(logits[:, -1, :], dim=-1)
            idx = torch.cat((idx, torch.multinomial(probs, num_samples=1)), dim=1)
        return idx
