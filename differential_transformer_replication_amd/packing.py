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

Packed gradient accumulation: when the parameters' ``.grad`` tensors are
themselves consecutive rows of one buffer in pack order (``dp.BucketedAllReduce``
lays its buckets out that way, see ``bind_grad``), the backward adds the whole dW
into that buffer in ONE kernel (casting bf16 -> fp32 on the fly) and reports each
parameter to the bucket's ready hook itself, instead of autograd running one
``AccumulateGrad`` add per parameter (2H..(2N+1)H small launches per module).
"""
from __future__ import annotations

import os
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


def bind_grad(holder: Dict, params: Sequence[torch.nn.Parameter], gflat: torch.Tensor, on_ready) -> None:
    """Declare ``gflat`` (1-D fp32, the params' numels in pack order) as the buffer
    the params' ``.grad`` views live in, and ``on_ready(p)`` as the hook to call once
    a parameter's gradient has been accumulated."""
    holder["grad"] = gflat
    holder["on_ready"] = on_ready


_ACC_KERNEL = os.environ.get("DTA_ACC_KERNEL", "1") != "0"      # A/B switch: 0 = torch's add_
_SPLITK = os.environ.get("DTA_SPLITK", "1") != "0"              # A/B switch: 0 = one bf16-output GEMM


def weight_grad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW = dy^T x for token-major (K, O) / (K, I) operands, the weight gradient of a
    Linear over K tokens.  bf16 on the GPU: fp32 output (no bf16 rounding of dW) and,
    when the (O, I) output has few 256x256 tiles for 256 CUs, split over K into S
    batched GEMMs of K/S tokens whose fp32 partials are summed (measured at the cfg4
    shapes, tools/gemm_splitk_probe.py: 1024x1024 199 -> 82 us, 3072x1024 304 -> 207,
    8192x1024 648 -> 590).  Otherwise the plain GEMM in the operands' dtype."""
    K, O = dy.shape
    I = x.shape[1]
    if not (_SPLITK and dy.is_cuda and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16):
        return dy.t() @ x
    tiles = -(-O // 256) * -(-I // 256)
    S = 8 if tiles <= 16 else (4 if tiles <= 128 else 1)
    while S > 1 and (K % S or (K // S) % 256):
        S //= 2
    if S == 1:
        return torch.mm(dy.t(), x, out_dtype=torch.float32)
    Kc = K // S
    part = torch.bmm(dy.view(S, Kc, O).transpose(1, 2), x.view(S, Kc, I), out_dtype=torch.float32)
    return part.sum(0)


def accumulate(g: torch.Tensor, d: torch.Tensor) -> None:
    """g += d for an fp32 gradient buffer and a bf16/fp16/fp32 gradient of the same
    numel: one HBM-bound HIP launch (dta_accumulate_f32) on the GPU, where torch's
    mixed-dtype add runs at a fraction of the HBM rate."""
    from . import _lib
    if (_ACC_KERNEL and g.is_cuda and d.is_cuda and g.dtype == torch.float32 and d.dtype in _lib._DTYPES and g.is_contiguous()
            and d.is_contiguous() and g.numel() == d.numel() and g.data_ptr() % 16 == 0 and d.data_ptr() % 16 == 0):
        lib = _lib.load()
        _lib.check(lib.dta_accumulate_f32(_lib.dtype_code(d.dtype), g.numel(), d.data_ptr(), g.data_ptr(),
                                          _lib.stream_handle(g.device)))
    else:
        g.view_as(d).add_(d)


def _grad_target(holder: Dict, params: Sequence[torch.nn.Parameter]):
    g = holder.get("grad")
    if g is None:
        return None
    ptr, off = g.data_ptr(), 0
    for p in params:                      # still the bound views (not set_to_none / replaced)?
        pg = p.grad
        if pg is None or pg.data_ptr() != ptr + off * 4 or pg.dtype != torch.float32:
            return None
        off += p.numel()
    return g if off == g.numel() else None


class _PackedLinear(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, base, holder, *params):
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        xc = x.to(dt)
        wc = base.to(dt)
        with torch.autocast("cuda", enabled=False):
            y = F.linear(xc, wc)
        ctx.save_for_backward(xc, wc)
        ctx.x_dtype = x.dtype
        ctx.rows = [p.shape[0] for p in params]
        ctx.w_dtype = base.dtype
        bound = holder is not None and "grad" in holder
        ctx.holder = holder if bound else None
        ctx.params = params if bound else None
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        dy = dy.to(wc.dtype)
        with torch.autocast("cuda", enabled=False):
            dx = (dy @ wc).to(ctx.x_dtype) if ctx.needs_input_grad[0] else None
            dw = weight_grad(dy.reshape(-1, dy.shape[-1]), xc.reshape(-1, xc.shape[-1]))
        if ctx.holder is not None and all(ctx.needs_input_grad[3:]):
            g = _grad_target(ctx.holder, ctx.params)
            if g is not None:
                accumulate(g, dw)                 # one launch, bf16 -> fp32 in the add
                hook = ctx.holder["on_ready"]
                for p in ctx.params:
                    hook(p)
                return (dx, None, None) + (None,) * len(ctx.rows)
        dw = dw.to(ctx.w_dtype)
        grads: List[torch.Tensor] = list(torch.split(dw, ctx.rows, 0))
        return (dx, None, None, *grads)


class _PackedParams(torch.autograd.Function):
    """The pack itself as a differentiable tensor of its parameters (used for the
    per-head lambda vectors): forward copies the small pack once (one launch instead
    of a ``torch.stack`` per vector kind); backward splits -- or, when bound, adds the
    whole gradient into the bound buffer in one launch."""

    @staticmethod
    def forward(ctx, base, holder, *params):
        bound = holder is not None and "grad" in holder
        ctx.holder = holder if bound else None
        ctx.params = params if bound else None
        ctx.shapes = [p.shape for p in params]
        return base.clone()

    @staticmethod
    def backward(ctx, d):
        if ctx.holder is not None and all(ctx.needs_input_grad[2:]):
            g = _grad_target(ctx.holder, ctx.params)
            if g is not None:
                accumulate(g, d)
                hook = ctx.holder["on_ready"]
                for p in ctx.params:
                    hook(p)
                return (None, None) + (None,) * len(ctx.shapes)
        rows = [sh[0] for sh in ctx.shapes]
        return (None, None) + tuple(t.reshape(sh) for t, sh in zip(torch.split(d, rows, 0), ctx.shapes))


def packed_tensor(params: Sequence[torch.nn.Parameter], holder: Dict[str, torch.Tensor]) -> torch.Tensor:
    """The (sum of rows, ...) pack of ``params`` as one autograd-tracked tensor."""
    base = ensure_packed(params, holder)
    return _PackedParams.apply(base, holder, *params)


def packed_linear(x: torch.Tensor, params: Sequence[torch.nn.Parameter], holder: Dict[str, torch.Tensor]):
    """``x @ cat(params).T`` without the cat: one GEMM over the shared pack."""
    base = ensure_packed(params, holder)
    return _PackedLinear.apply(x, base, holder, *params)
