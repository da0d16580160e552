"""Reference-compatibility helpers shared by the module mirrors.

* The reference registers a persistent fp32 ``tril`` (block_size x block_size)
  buffer in every head (diff_transformer.py:31, Ndiff_transformer.py:59,
  control.py:31): 4 GiB per head at block 32768 and broadcast by DDP.  The
  fused kernels mask causally without it, so it is never allocated.  For
  ``state_dict`` key compatibility it is emitted on save (one shared CPU tensor
  per block_size, so ``torch.save`` stores it once) and dropped on load.
  ``DTA_EMIT_TRIL=0`` turns the emission off.
* ``lambda_init`` per layer is computed exactly like the reference (fp32 torch
  arithmetic, diff_transformer.py:42-43) and cached per layer index.
* Host-synchronising reads of module buffers are cached against the tensor's
  identity and version counter so a training step issues no ``.item()``.
"""
from __future__ import annotations

import functools
import os
from typing import Dict, Tuple

import torch

_TRIL_CACHE: Dict[int, torch.Tensor] = {}


def _tril(block_size: int) -> torch.Tensor:
    t = _TRIL_CACHE.get(block_size)
    if t is None:
        t = torch.tril(torch.ones(block_size, block_size))
        _TRIL_CACHE[block_size] = t
    return t


def emit_tril_hooks(module: torch.nn.Module, block_size: int) -> None:
    def save_hook(mod, state_dict, prefix, local_metadata):
        if os.environ.get("DTA_EMIT_TRIL", "1") != "0":
            state_dict[prefix + "tril"] = _tril(block_size)
        return state_dict

    def load_hook(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs):
        t = state_dict.pop(prefix + "tril", None)
        if t is not None and tuple(t.shape) != (block_size, block_size):
            error_msgs.append(f"{prefix}tril: shape {tuple(t.shape)} != ({block_size}, {block_size})")

    module._register_state_dict_hook(save_hook)
    module._register_load_state_dict_pre_hook(load_hook)


@functools.lru_cache(maxsize=None)
def _lambda_init_f32(layer_idx: int) -> float:
    li = torch.tensor(layer_idx, dtype=torch.float)
    return float(0.8 - 0.6 * torch.exp(-0.3 * (li - 1.0)))


def lambda_init_value(layer_idx: int, buf: torch.Tensor) -> float:
    """Value get_lambda copies into the head buffer (diff_transformer.py:42-44)."""
    return _lambda_init_f32(int(layer_idx))


_SCALAR_CACHE: Dict[int, Tuple[int, int, float]] = {}


def cached_scalar(t: torch.Tensor) -> float:
    """float(t) for a 0-d buffer, synchronising only when the tensor changed."""
    key = id(t)
    hit = _SCALAR_CACHE.get(key)
    if hit is not None and hit[0] == t._version and hit[1] == t.data_ptr():
        return hit[2]
    v = float(t.detach().float().cpu())
    _SCALAR_CACHE[key] = (t._version, t.data_ptr(), v)
    return v


def fill_if_changed(buf: torch.Tensor, value: float) -> None:
    """In-place fill of a 0-d buffer, skipped when it already holds ``value``."""
    key = id(buf)
    hit = _SCALAR_CACHE.get(key)
    if hit is not None and hit[0] == buf._version and hit[1] == buf.data_ptr() and hit[2] == value:
        return
    with torch.no_grad():
        buf.fill_(value)
    _SCALAR_CACHE[key] = (buf._version, buf.data_ptr(), value)


def mha_out_scale(lambda_init: torch.Tensor) -> float:
    """``1 - self.lambda_init`` of the MHA (0.8 forever -> 0.2, SURVEY semantic 2),
    computed in the buffer's dtype like diff_transformer.py:91."""
    v = cached_scalar(lambda_init)
    return float(1 - torch.tensor(v, dtype=lambda_init.dtype))


def check_seq_len(T: int, block_size: int) -> None:
    # the reference raises a broadcast RuntimeError when T > block_size (semantic 9)
    if T > block_size:
        raise RuntimeError(f"sequence length {T} exceeds block_size {block_size}")


def attn_dropout_p(drops, training: bool) -> float:
    """The attention-map dropout probability the fused kernels apply: the heads'
    nn.Dropout p in training (diff_transformer.py:66-67, Ndiff_transformer.py:114),
    0 in eval.  All heads of one module share it (the reference builds them with the
    same ``dropout``); differing per-head values are refused rather than ignored."""
    if not training:
        return 0.0
    ps = {float(d.p) for d in drops}
    if len(ps) != 1:
        raise NotImplementedError("the fused kernels apply one attention-dropout p to every head of a module")
    return ps.pop()
