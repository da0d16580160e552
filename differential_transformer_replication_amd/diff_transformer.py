"""Drop-in replacement of the reference ``diff_transformer.py`` module surface.

Class names, constructor arguments, forward signatures, parameter/buffer names
(hence ``state_dict`` keys) and parameter-creation order (hence seeded
initialisation) follow the reference (``/root/reference/diff_transformer.py``).
What changes is the execution: the per-head Python loop of eager ATen ops
(diff_transformer.py:89, 50-73) becomes one packed projection GEMM, one fused
HIP attention launch for all heads (``ops.diff_attention``) and one fused
GroupLayerNorm x0.2 launch (``ops.group_ln_scale``).  SwiGLU, Block and the
model shell are carried as plain PyTorch.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn import functional as F

from . import kv_cache, ops
from .packing import ensure_packed, packed_linear, packed_tensor
from ._compat import (emit_tril_hooks, lambda_init_value, check_seq_len, attn_dropout_p, fill_if_changed,
                      mha_out_scale)

__all__ = ["GroupLayerNorm", "DiffHead", "MultiHeadDiffAttention", "SwiGLU", "Block", "DiffTransformer"]


class GroupLayerNorm(nn.Module):
    """LayerNorm over the concatenated width num_heads*2*head_dim -- not per head,
    not RMS (diff_transformer.py:5-20, SURVEY semantic 1)."""

    def __init__(self, num_heads, head_dim):
        super().__init__()
        self.eps = 1e-5
        self.num_heads = num_heads
        self.head_dim = head_dim * 2
        width = num_heads * self.head_dim
        self.weight = nn.Parameter(torch.ones(1, 1, width))
        self.bias = nn.Parameter(torch.zeros(1, 1, width))
        self._gpack = {}                           # grad binding of (weight, bias), dp.BucketedAllReduce

    def param_packs(self):
        return [(self._gpack, [self.weight, self.bias])]

    def forward(self, x):
        return ops.group_ln_scale(x, self.weight, self.bias, self.eps, 1.0, self._gpack)


def _layer_lambda_coef(lq1, lk1, lq2, lk2, init: torch.Tensor) -> torch.Tensor:
    """(H, 2) signed branch weights [1, -lambda_h] with
    lambda = mean(exp(lq1*lk1) - exp(lq2*lk2) + init)  (diff_transformer.py:41-48, 70)."""
    lam = (torch.exp(lq1 * lk1) - torch.exp(lq2 * lk2) + init).mean(dim=-1)
    return torch.stack([torch.ones_like(lam), -lam], dim=-1)


class DiffHead(nn.Module):
    """One differential-attention head (diff_transformer.py:22-73)."""

    def __init__(self, head_size, n_embd, dropout, block_size):
        super().__init__()
        # creation order = reference order (seeded init parity)
        self.key1 = nn.Linear(n_embd, head_size, bias=False)
        self.query1 = nn.Linear(n_embd, head_size, bias=False)
        self.key2 = nn.Linear(n_embd, head_size, bias=False)
        self.query2 = nn.Linear(n_embd, head_size, bias=False)
        self.value = nn.Linear(n_embd, head_size * 2, bias=False)
        self.block_size = block_size
        self.head_size = head_size
        emit_tril_hooks(self, block_size)          # virtual `tril` buffer (SURVEY semantic 8)
        self.dropout = nn.Dropout(dropout)
        self.lambda_q1 = nn.Parameter(torch.zeros(head_size))
        self.lambda_k1 = nn.Parameter(torch.zeros(head_size))
        self.lambda_q2 = nn.Parameter(torch.zeros(head_size))
        self.lambda_k2 = nn.Parameter(torch.zeros(head_size))
        self.register_buffer("lambda_init", torch.tensor(0.8))

    def get_lambda(self, layer_idx):
        """diff_transformer.py:41-48, including the buffer side effect (:44)."""
        init = lambda_init_value(layer_idx, self.lambda_init)
        fill_if_changed(self.lambda_init, init)
        lam = torch.exp(self.lambda_q1 * self.lambda_k1) - torch.exp(self.lambda_q2 * self.lambda_k2) \
            + self.lambda_init
        return lam.mean()

    def packed_weight(self) -> torch.Tensor:
        """Rows in the kernel's packed order [Q (N=2, hs) | K (2, hs) | V (2hs)] for H=1."""
        return torch.cat([self.query1.weight, self.query2.weight, self.key1.weight, self.key2.weight,
                          self.value.weight], dim=0)

    def forward(self, x, layer_idx):
        check_seq_len(x.shape[1], self.block_size)
        init = lambda_init_value(layer_idx, self.lambda_init)
        fill_if_changed(self.lambda_init, init)
        coef = _layer_lambda_coef(self.lambda_q1[None].float(), self.lambda_k1[None].float(),
                                  self.lambda_q2[None].float(), self.lambda_k2[None].float(), init)
        qkv = F.linear(x, self.packed_weight())
        return ops.diff_attention(qkv, coef, 1, 2, self.head_size,
                                  dropout_p=attn_dropout_p([self.dropout], self.training))


class MultiHeadDiffAttention(nn.Module):
    """All heads in one fused launch (diff_transformer.py:75-93)."""

    def __init__(self, num_heads, head_size, n_embd, dropout, block_size):
        super().__init__()
        self.heads = nn.ModuleList([DiffHead(head_size, n_embd, dropout, block_size) for _ in range(num_heads)])
        self.group_norm = GroupLayerNorm(num_heads, head_size)
        self.proj = nn.Linear(head_size * 2 * num_heads, n_embd)
        self.dropout = nn.Dropout(dropout)
        self.register_buffer("lambda_init", torch.tensor(0.8))
        self.num_heads = num_heads
        self.head_size = head_size
        self.block_size = block_size
        self._pack = {}                            # the shared storage of the heads' projections
        self._lam_pack = {}                        # ... and of their lambda vectors

    def packed_params(self):
        """Every head's projection weights in the kernel's packed row order."""
        hs = self.heads
        q = [w for h in hs for w in (h.query1.weight, h.query2.weight)]
        k = [w for h in hs for w in (h.key1.weight, h.key2.weight)]
        v = [h.value.weight for h in hs]
        return q + k + v

    def packed_weight(self) -> torch.Tensor:
        """(2*H*2*hs + H*2hs, C): the pack the per-head weights are views of (no copy)."""
        return ensure_packed(self.packed_params(), self._pack)

    def coefficients(self, layer_idx) -> torch.Tensor:
        init = lambda_init_value(layer_idx, self.heads[0].lambda_init)
        for h in self.heads:                       # get_lambda's buffer side effect, every head
            fill_if_changed(h.lambda_init, init)
        # the 4H lambda vectors are row views of one pack: one copy forward, one add backward
        lam = packed_tensor(self.lambda_params(), self._lam_pack).view(4, self.num_heads, self.head_size).float()
        return _layer_lambda_coef(*lam.unbind(0), init)

    def lambda_params(self):
        return ([h.lambda_q1 for h in self.heads] + [h.lambda_k1 for h in self.heads]
                + [h.lambda_q2 for h in self.heads] + [h.lambda_k2 for h in self.heads])

    def param_packs(self):
        """(holder, params) of every shared-storage parameter group (dp.BucketedAllReduce)."""
        return [(self._pack, self.packed_params()), (self._lam_pack, self.lambda_params())]

    def forward(self, x, layer_idx):
        check_seq_len(x.shape[1], self.block_size)
        coef = self.coefficients(layer_idx)
        qkv = packed_linear(x, self.packed_params(), self._pack)
        out = ops.diff_attention(qkv, coef, self.num_heads, 2, self.head_size,
                                 dropout_p=attn_dropout_p([h.dropout for h in self.heads], self.training))
        # GroupLayerNorm then x(1 - lambda_init) with the MHA's own, never-updated 0.8 buffer
        gn = self.group_norm
        out = ops.group_ln_scale(out, gn.weight, gn.bias, gn.eps, mha_out_scale(self.lambda_init), gn._gpack)
        return self.dropout(ops.linear(out, self.proj))


class SwiGLU(nn.Module):
    """silu(W_g x) * (W_x x)  (diff_transformer.py:95-105).  On the GPU the two Linears run
    as one GEMM over shared weight / bias packs (ops.packed_swiglu)."""

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
    """Pre-LN residual block (diff_transformer.py:107-126)."""

    def __init__(self, n_embd, n_head, block_size, dropout):
        super().__init__()
        head_size = n_embd // (n_head * 2)
        self.diff_attn = MultiHeadDiffAttention(n_head, head_size, n_embd, dropout, block_size)
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


class DiffTransformer(nn.Module):
    """Token + position embeddings, Block x n_layer, ln_f, lm_head, CE loss
    (diff_transformer.py:128-185)."""

    def __init__(self, vocab_size, n_embd, n_head, n_layer, block_size, dropout):
        super().__init__()
        self.block_size = block_size
        self.token_embedding_table = nn.Embedding(vocab_size, n_embd)
        self.position_embedding_table = nn.Embedding(block_size, n_embd)
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
        pos = torch.arange(T, device=idx.device)
        x = self.token_embedding_table(idx) + self.position_embedding_table(pos)
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
        """Naive sampling: full forward per token, cropped to block_size (:177-185)."""
        if kv_cache.enabled(idx):                        # KV-cache decode
            return kv_cache.cached_generate(self, idx, max_new_tokens)
        for _ in range(max_new_tokens):
            logits, _ = self(idx[:, -self.block_size:])
            probs = F.softmax(logits[:, -1, :], dim=-1)
            idx = torch.cat((idx, torch.multinomial(probs, num_samples=1)), dim=1)
        return idx
