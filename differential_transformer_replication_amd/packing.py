"""Packed per-head projection weights.

The reference creates five (N-diff: 2N+1) ``nn.Linear`` per head and projects
head by head (diff_transformer.py:53-55, Ndiff_transformer.py:97,104-109).  Here
every head's weights are row views of ONE contiguous tensor laid out in the
kernel's packed order ``[Q (H, N, hs) | K (H, N, hs) | V (H, dv)]``, so one GEMM
projects all heads with no per-step ``torch.cat`` of the weights.

The parameters themselves stay the reference's: one ``nn.Parameter`` per Linear,
same names, same ``state_dict`` keys, same seeded initial values (they are packed
by copy after initialisation).  Only their storage is shared:

* ``ensure_packed`` checks that the parameters are still consecutive rows of the
  pack (``Module.to``/``.cuda()``/``.half()`` give every parameter new storage)
  and re-packs them by one copy when they are not;
* ``packed_linear`` is an autograd Function over the pack whose backward
  returns each parameter's gradient as a row slice of one dW -- the same bf16
  GEMMs and casts autocast applies to an ``nn.Linear``.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch
from torch.nn import functional as F


def _intact(base: torch.Tensor, params: Sequence[torch.nn.Parameter]) -> bool:
    p0 = params[0]
    if base.device != p0.device or base.dtype != p0.dtype:
        return False
    ptr, es, off = base.data_ptr(), base.element_size(), 0
    for p in params:
        if p.data_ptr() != ptr + off * es or not p.is_contiguous():
            return False
        off += p.numel()
    return off == base.numel()


def ensure_packed(params: Sequence[torch.nn.Parameter], holder: Dict[str, torch.Tensor]) -> torch.Tensor:
    """The pack whose consecutive row blocks ARE ``params`` (re-packed by one copy
    whenever that no longer holds)."""
    base = holder.get("base")
    if base is not None and _intact(base, params):
        return base
    with torch.no_grad():
        base = torch.cat([p.detach().reshape(p.shape[0], -1) for p in params], 0).contiguous()
        off = 0
        for p in params:
            n = p.shape[0]
            p.data = base[off:off + n].view_as(p)
            off += n
    holder["base"] = base
    return base


class _PackedLinear(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, base, *params):
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        xc = x.to(dt)
        wc = base.to(dt)
        with torch.autocast("cuda", enabled=False):
            y = F.linear(xc, wc)
        ctx.save_for_backward(xc, wc)
        ctx.x_dtype = x.dtype
        ctx.rows = [p.shape[0] for p in params]
        ctx.w_dtype = base.dtype
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        dy = dy.to(wc.dtype)
        with torch.autocast("cuda", enabled=False):
            dx = (dy @ wc).to(ctx.x_dtype) if ctx.needs_input_grad[0] else None
            dw = dy.reshape(-1, dy.shape[-1]).t() @ xc.reshape(-1, xc.shape[-1])
        dw = dw.to(ctx.w_dtype)
        grads: List[torch.Tensor] = list(torch.split(dw, ctx.rows, 0))
        return (dx, None, *grads)


def packed_linear(x: torch.Tensor, params: Sequence[torch.nn.Parameter], holder: Dict[str, torch.Tensor]):
    """``x @ cat(params).T`` without the cat: one GEMM over the shared pack."""
    base = ensure_packed(params, holder)
    return _PackedLinear.apply(x, base, *params)
