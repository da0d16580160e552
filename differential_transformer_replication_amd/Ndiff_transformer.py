"""Drop-in replacement of the reference ``Ndiff_transformer.py`` module surface
(N-term alternating-sign differential attention with RoPE).

Same class names, constructor arguments (including the disagreeing defaults:
head ``n_terms=2``, Block/model ``n_terms=4``), ``state_dict`` keys and
parameter-creation order as ``/root/reference/Ndiff_transformer.py``.  The
per-head, per-branch loop (Ndiff_transformer.py:102-125, 145) runs as one RoPE
launch, one fused N-branch attention launch and one GroupLayerNorm x0.2 launch.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn import functional as F

from . import kv_cache, ops
from .packing import ensure_packed, packed_linear, packed_tensor
from ._compat import (emit_tril_hooks, lambda_init_value, check_seq_len, attn_dropout_p, fill_if_changed,
                      mha_out_scale)
from .diff_transformer import GroupLayerNorm, SwiGLU

__all__ = ["precompute_freqs_cis", "apply_rotary_emb", "GroupLayerNorm", "AlternatingDiffHead",
           "MultiHeadAlternatingDiffAttention", "SwiGLU", "Block", "AlternatingDiffTransformer"]


def precompute_freqs_cis(dim: int, end: int, theta: float = 10000.0):
    """complex64 (end, dim/2) rotation table (Ndiff_transformer.py:4-9)."""
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2)[: (dim // 2)].float() / dim))
    ang = torch.outer(torch.arange(end, device=inv.device), inv)
    return torch.polar(torch.ones_like(ang), ang)


def apply_rotary_emb(x: torch.Tensor, freqs_cis: torch.Tensor) -> torch.Tensor:
    """Eager interleaved-pair rotation in fp32, cast back (Ndiff_transformer.py:11-22).
    Exported for API compatibility; the model path rotates inside ``ops``."""
    xc = torch.view_as_complex(x.float().reshape(*x.shape[:-1], -1, 2))
    fc = freqs_cis.to(x.device)[: x.shape[1], :]
    return torch.view_as_real(xc * fc.unsqueeze(0)).flatten(-2).type_as(x)


def rope_table(freqs_cis: torch.Tensor, T: int, head_size: int) -> torch.Tensor:
    """fp32 (T, hs/2, 2) [cos, sin] table for the kernels; recomputed if the complex
    buffer was cast away by Module.to(real dtype)."""
    if not freqs_cis.is_complex():
        freqs_cis = precompute_freqs_cis(head_size, T).to(freqs_cis.device)
    return torch.view_as_real(freqs_cis[:T])


def alternating_coefficients(lqs: torch.Tensor, lks: torch.Tensor, init: float) -> torch.Tensor:
    """(..., N) signed weights [+l0, -l1, +l2, ...] from stacked (..., N, hs) lambda
    vectors: l0 = mean(e0) + init, l_i = mean(e_i - e_{i-1}) + init, e_i = exp(lq_i*lk_i)
    (Ndiff_transformer.py:79-93, 118-123)."""
    e = torch.exp(lqs * lks)
    prev = torch.cat([torch.zeros_like(e[..., :1, :]), e[..., :-1, :]], dim=-2)
    lam = (e - prev + init).mean(dim=-1)
    n = lam.shape[-1]
    sign = torch.tensor([1.0 if i % 2 == 0 else -1.0 for i in range(n)], device=lam.device, dtype=lam.dtype)
    return lam * sign


class AlternatingDiffHead(nn.Module):
    """N-branch differential head with RoPE (Ndiff_transformer.py:40-126)."""

    def __init__(self, head_size, n_embd, dropout, block_size, n_terms=2):
        super().__init__()
        self.n_terms = n_terms
        self.head_size = head_size
        self.block_size = block_size
        self.queries = nn.ModuleList([nn.Linear(n_embd, head_size, bias=False) for _ in range(n_terms)])
        self.keys = nn.ModuleList([nn.Linear(n_embd, head_size, bias=False) for _ in range(n_terms)])
        self.value = nn.Linear(n_embd, head_size * 2, bias=False)
        emit_tril_hooks(self, block_size)
        self.dropout = nn.Dropout(dropout)
        self.lambda_qs = nn.ParameterList([nn.Parameter(torch.zeros(head_size)) for _ in range(n_terms)])
        self.lambda_ks = nn.ParameterList([nn.Parameter(torch.zeros(head_size)) for _ in range(n_terms)])
        self.register_buffer("freqs_cis", precompute_freqs_cis(head_size, block_size))
        self.register_buffer("lambda_init", torch.tensor(0.8))

    def _check_terms(self):
        if self.n_terms < 1:
            # torch.stack([]) in get_lambda raises for n_terms=0 (Ndiff_transformer.py:93)
            raise RuntimeError("stack expects a non-empty TensorList")

    def get_lambda(self, layer_idx):
        """(N,) lambdas (Ndiff_transformer.py:79-93) with the buffer side effect."""
        self._check_terms()
        init = lambda_init_value(layer_idx, self.lambda_init)
        fill_if_changed(self.lambda_init, init)
        c = alternating_coefficients(torch.stack(list(self.lambda_qs)), torch.stack(list(self.lambda_ks)), init)
        sign = torch.tensor([1.0 if i % 2 == 0 else -1.0 for i in range(self.n_terms)], device=c.device)
        return c * sign

    def packed_weight(self) -> torch.Tensor:
        return torch.cat([q.weight for q in self.queries] + [k.weight for k in self.keys] + [self.value.weight], 0)

    def forward(self, x, layer_idx):
        self._check_terms()
        T = x.shape[1]
        check_seq_len(T, self.block_size)
        init = lambda_init_value(layer_idx, self.lambda_init)
        fill_if_changed(self.lambda_init, init)
        coef = alternating_coefficients(torch.stack(list(self.lambda_qs)).float()[None],
                                        torch.stack(list(self.lambda_ks)).float()[None], init)
        qkv = F.linear(x, self.packed_weight())
        return ops.diff_attention(qkv, coef, 1, self.n_terms, self.head_size,
                                  rope_table(self.freqs_cis, T, self.head_size),
                                  dropout_p=attn_dropout_p([self.dropout], self.training))


class MultiHeadAlternatingDiffAttention(nn.Module):
    """All heads and branches in one fused launch (Ndiff_transformer.py:128-146)."""

    def __init__(self, num_heads, head_size, n_embd, dropout, block_size, n_terms=2):
        super().__init__()
        self.heads = nn.ModuleList([AlternatingDiffHead(head_size, n_embd, dropout, block_size, n_terms)
                                    for _ in range(num_heads)])
        self.group_norm = GroupLayerNorm(num_heads, head_size)
        self.proj = nn.Linear(head_size * 2 * num_heads, n_embd)
        self.dropout = nn.Dropout(dropout)
        self.register_buffer("lambda_init", torch.tensor(0.8))
        self.num_heads = num_heads
        self.head_size = head_size
        self.n_terms = n_terms
        self.block_size = block_size
        self._pack = {}                            # the shared storage of the heads' projections
        self._lam_pack = {}                        # ... and of their lambda vectors

    def packed_params(self):
        """Every head's projection weights in the kernel's packed row order."""
        q = [m.weight for h in self.heads for m in h.queries]
        k = [m.weight for h in self.heads for m in h.keys]
        v = [h.value.weight for h in self.heads]
        return q + k + v

    def packed_weight(self) -> torch.Tensor:
        """The pack the per-head weights are views of (no copy)."""
        return ensure_packed(self.packed_params(), self._pack)

    def coefficients(self, layer_idx) -> torch.Tensor:
        init = lambda_init_value(layer_idx, self.heads[0].lambda_init)
        for h in self.heads:
            fill_if_changed(h.lambda_init, init)
        # the 2NH lambda vectors are row views of one pack: one copy forward, one add backward
        lam = packed_tensor(self.lambda_params(), self._lam_pack).view(
            2, self.num_heads, self.n_terms, self.head_size).float()
        return alternating_coefficients(*lam.unbind(0), init)

    def lambda_params(self):
        return [p for h in self.heads for p in h.lambda_qs] + [p for h in self.heads for p in h.lambda_ks]

    def param_packs(self):
        """(holder, params) of every shared-storage parameter group (dp.BucketedAllReduce)."""
        return [(self._pack, self.packed_params()), (self._lam_pack, self.lambda_params())]

    def forward(self, x, layer_idx):
        self.heads[0]._check_terms()
        T = x.shape[1]
        check_seq_len(T, self.block_size)
        coef = self.coefficients(layer_idx)
        qkv = packed_linear(x, self.packed_params(), self._pack)
        freqs = rope_table(self.heads[0].freqs_cis, T, self.head_size)
        out = ops.diff_attention(qkv, coef, self.num_heads, self.n_terms, self.head_size, freqs,
                                 dropout_p=attn_dropout_p([h.dropout for h in self.heads], self.training))
        gn = self.group_norm
        out = ops.group_ln_scale(out, gn.weight, gn.bias, gn.eps, mha_out_scale(self.lambda_init), gn._gpack)
        return self.dropout(ops.linear(out, self.proj))


class Block(nn.Module):
    """Ndiff_transformer.py:160-177 (n_terms default 4)."""

    def __init__(self, n_embd, n_head, block_size, dropout, n_terms=4):
        super().__init__()
        head_size = n_embd // (n_head * 2)
        self.diff_attn = MultiHeadAlternatingDiffAttention(n_head, head_size, n_embd, dropout, block_size, n_terms)
        self.ffwd = nn.Sequential(SwiGLU(n_embd, 4 * n_embd), nn.Linear(4 * n_embd, n_embd), nn.Dropout(dropout))
        self.ln1 = ops.LayerNorm(n_embd, autocast_out=True)
        self.ln2 = ops.LayerNorm(n_embd, autocast_out=True)

    def forward(self, x, layer_idx):
        # the residual add and ln2 in one pass on the GPU (ops.add_layer_norm)
        x, h = ops.add_layer_norm(x, self.diff_attn(self.ln1(x), layer_idx), self.ln2)
        return x + ops.ffn(self.ffwd, h)

    def forward_chained(self, x, h, layer_idx, next_ln):
        """forward() given h = ln1(x), returning (x_out, next_ln(x_out)): both residual
        adds fused with the LayerNorm that follows them (the model's block loop)."""
        x, h = ops.add_layer_norm(x, self.diff_attn(h, layer_idx), self.ln2)
        return ops.add_layer_norm(x, ops.ffn(self.ffwd, h), next_ln)


class AlternatingDiffTransformer(nn.Module):
    """Token embeddings only (no position table), RoPE inside attention
    (Ndiff_transformer.py:181-265)."""

    def __init__(self, vocab_size, n_embd, n_head, n_layer, block_size, dropout, n_terms=4):
        super().__init__()
        self.block_size = block_size
        self.token_embedding_table = nn.Embedding(vocab_size, n_embd)
        self.blocks = nn.ModuleList([Block(n_embd, n_head, block_size, dropout, n_terms) for _ in range(n_layer)])
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
        # (ln1 of the next block, ln_f after the last); 1-based layer index (:161)
        n = len(self.blocks)
        h = self.blocks[0].ln1(x) if n else self.ln_f(x)
        for layer, block in enumerate(self.blocks, 1):
            x, h = block.forward_chained(x, h, layer, self.blocks[layer].ln1 if layer < n else self.ln_f)
        logits = self.lm_head(h)
        loss = None
        if targets is not None:
            logits = logits.view(B * T, -1)             # reference returns (B*T, V) with targets
            loss = F.cross_entropy(logits, targets.view(B * T))
        return logits, loss

    @torch.no_grad()
    def generate(self, idx, max_new_tokens):
        if kv_cache.enabled(idx):                        # KV-cache decode
            return kv_cache.cached_generate(self, idx, max_new_tokens)
        for _ in range(max_new_tokens):
            logits, _ = self(idx[:, -self.block_size:])
            probs = F.softmax(logits[:, -1, :], dim=-1)
            idx = torch.cat((idx, torch.multinomial(probs, num_samples=1)), dim=1)
        return idx

    @staticmethod
    def from_pretrained(path):
        """Load a ``save_pretrained`` file (Ndiff_transformer.py:243-249); tensors and
        plain numbers only, so the safe loader is used."""
        ckpt = torch.load(path, weights_only=True, map_location="cpu")
        model = AlternatingDiffTransformer(**ckpt["model_args"])
        model.load_state_dict(ckpt["model_state"])
        return model

    def save_pretrained(self, path):
        """{model_args, model_state} (Ndiff_transformer.py:251-265)."""
        attn = self.blocks[0].diff_attn
        torch.save({
            "model_args": {
                "vocab_size": self.token_embedding_table.num_embeddings,
                "n_embd": self.token_embedding_table.embedding_dim,
                "n_head": len(attn.heads),
                "n_layer": len(self.blocks),
                "block_size": self.block_size,
                "dropout": attn.dropout.p,
                "n_terms": attn.heads[0].n_terms,
            },
            "model_state": self.state_dict(),
        }, path)
