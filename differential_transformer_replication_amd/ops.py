"""torch.autograd.Function wrappers over the C ABI (the only compute path).

``diff_attention(qkv, coef, ...)``
    Fused N-branch causal differential attention over a packed projection
    output ``qkv`` of shape (B, T, W), W = 2*H*N*hs + H*dv, laid out
    ``[Q (H, N, hs) | K (H, N, hs) | V (H, dv)]``.  Returns O of shape
    (B, T, H*dv) = concatenated per-head outputs (diff_transformer.py:89, before
    the GroupLayerNorm).  Backward writes dQ/dK/dV into one (B, T, W) buffer, so
    the projection GEMM's backward sees a single gradient tensor.
``group_ln_scale(x, w, b, eps, out_scale)``
    GroupLayerNorm over the last dim fused with the constant output scale
    (diff_transformer.py:15-20, 90-91).

There is no CPU or eager fallback: non-CUDA tensors raise.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Dict, List, Optional, Tuple

import torch
from torch.nn import functional as F

from . import _lib, packing

Tensor = torch.Tensor


def _require_gpu(*ts: Tensor) -> None:
    for t in ts:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError("differential_transformer_replication_amd ops run only on the MI355X "
                               "HIP path (libdiffattn.so); got a tensor on " + str(t.device))


class KernelTimer:
    """Optional HIP-event brackets around the two dominant launches (the fused
    forward kernel and the fused backward kernel).  Events are recorded on the
    stream the kernels are launched on (torch's current stream), so each pair
    brackets exactly one kernel.  Off by default (no events, no overhead)."""

    def __init__(self):
        self.active = False
        self._pairs: Dict[str, List[Tuple[torch.cuda.Event, torch.cuda.Event]]] = {}

    def start(self):
        self._pairs = {}
        self.active = True

    def stop(self):
        self.active = False

    @contextlib.contextmanager
    def region(self, name: str):
        if not self.active:
            yield
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        yield
        e1.record()
        self._pairs.setdefault(name, []).append((e0, e1))

    def mean_ms(self) -> Dict[str, Tuple[float, int]]:
        torch.cuda.synchronize()
        return {k: (sum(a.elapsed_time(b) for a, b in v) / len(v), len(v)) for k, v in self._pairs.items()}


TIMER = KernelTimer()


def supported(dtype: torch.dtype, hs: int, N: int, dv: int) -> bool:
    """Whether libdiffattn.so runs this shape as it is (dta_supported): an N-branch
    kernel plan, or branch groups over such plans for branch counts without one."""
    return bool(_lib.load().dta_supported(_lib.dtype_code(dtype), hs, N, dv))


def padded_head(dtype: torch.dtype, hs: int, N: int, dv: int) -> Optional[int]:
    """The head size the kernels run a head of size ``hs`` at: ``hs`` itself when it is
    built, else the smallest built head size above it (Q_i / K_i and V zero-padded, see
    ``diff_attention``), else None.  The reference accepts any head size
    (head_size = n_embd // (2 n_head), diff_transformer.py:111); the plans are built for
    16, 32, 64, 96, 128 and 256 (256: 16-bit diff plans, and the control's dv = hs in every
    dtype)."""
    if N < 1 or hs < 1 or dv not in (hs, 2 * hs) or (dv == hs and N != 1):
        return None
    for hp in (hs,) + tuple(h for h in (16, 32, 64, 96, 128, 256) if h > hs):
        if supported(dtype, hp, N, hp if dv == hs else 2 * hp):
            return hp
    return None


def attention_supported(dtype: torch.dtype, hs: int, N: int, dv: int) -> bool:
    """Whether ``diff_attention`` runs this shape on the HIP kernels (directly or padded)."""
    return padded_head(dtype, hs, N, dv) is not None


def packed_width(H: int, N: int, hs: int, dv: int) -> int:
    return 2 * H * N * hs + H * dv


def split_packed(qkv: Tensor, H: int, N: int, hs: int, dv: int):
    """Strided (B,T,H,N,hs)/(B,T,H,dv) views of the packed projection output."""
    B, T, W = qkv.shape
    nq = H * N * hs
    q = qkv[..., :nq].unflatten(-1, (H, N, hs))
    k = qkv[..., nq:2 * nq].unflatten(-1, (H, N, hs))
    v = qkv[..., 2 * nq:].unflatten(-1, (H, dv))
    return q, k, v


def _obr_dtype(dtype: torch.dtype) -> torch.dtype:
    """Storage type of the saved per-branch outputs O_i (ABI 6 obr_dtype): fp32.  fp16 O_i
    (DTA_OBR_F16=1, 16-bit activations) measured 0.7% off the cfg2 step but left one head's
    d(lambda) at 1.22 relative error in the default-config bf16 model, against a bar of 0.56
    (2x the reference algorithm's own bf16 error; fp32 O_i passes): the cancellation in
    sum_rows delta_i needs O_i unrounded."""
    if dtype != torch.float32 and os.environ.get("DTA_OBR_F16", "0") == "1":
        return torch.float16
    return torch.float32


# Whether the backward hands dta_attn_bwd the fp32 dV workspace (ABI 7 dv_f32) when dK/dV runs
# in more than one branch group.  Always on in the product; the C ABI's other path (dv_f32 NULL:
# each later group adds into the 16-bit dV) is exercised by the GPU tests with it off.
_DV_F32_WORKSPACE = [True]
# Whether the backward hands dta_attn_bwd the ABI 8 lse_c workspace (16-bit, no dropout: the key-major
# kernel folds |c_i| into its probabilities).  Always on in the product; the GPU tests turn it off to
# run the C ABI's unfolded 16-bit path.
_LSE_C_WORKSPACE = [True]

# Backward branch-group caps handed to dta_attn_bwd (ABI 7 group_max_dq / group_max_dkdv);
# (0, 0) = the library's per-stage defaults.  Tests set them with ``bwd_group_caps`` to run
# every built native N-branch backward plan.
_BWD_GROUP_MAX = [0, 0]


@contextlib.contextmanager
def bwd_group_caps(dq: int, dkdv: int):
    """Forward passes run within the block have their backward run dQ in branch groups of
    at most ``dq`` and dK/dV in groups of at most ``dkdv`` (0 = the library default for that
    stage).  The caps are taken at the forward and kept on the autograd context, so the
    backward may run after the block exits."""
    old = list(_BWD_GROUP_MAX)
    _BWD_GROUP_MAX[:] = [int(dq), int(dkdv)]
    try:
        yield
    finally:
        _BWD_GROUP_MAX[:] = old


class _DiffAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv: Tensor, coef: Tensor, H: int, N: int, hs: int, freqs: Optional[Tensor], dv: int,
                dropout_p: float, seed: int, scale: float):
        lib = _lib.load()
        _require_gpu(qkv, coef)
        if qkv.dim() != 3:
            raise RuntimeError("qkv must be (B, T, W)")
        qkv = qkv.contiguous()
        B, T, W = qkv.shape
        if W != packed_width(H, N, hs, dv):
            raise RuntimeError(f"packed width {W} != 2*H*N*hs + H*dv = {packed_width(H, N, hs, dv)}")
        dt = _lib.dtype_code(qkv.dtype)
        if not lib.dta_supported(dt, hs, N, dv):
            raise RuntimeError(f"no gfx950 kernel for head_size={hs}, n_terms={N}, dv={dv}, dtype={qkv.dtype}")
        coef = coef.detach().to(torch.float32).contiguous()
        dev = qkv.device
        stream = _lib.stream_handle(dev)
        q, k, v = split_packed(qkv, H, N, hs, dv)
        qk_rot = None
        rope_args = (None, _lib.DtaTensor())
        if freqs is not None:
            # RoPE of every Q_i/K_i (Ndiff_transformer.py:104-109): the K_i by one rotation pass,
            # the Q_i inside the forward kernel as it loads them (it also stores the rotated
            # rows into qk_rot for the backward)
            qk_rot = torch.empty(B, T, 2 * H, N, hs, device=dev, dtype=qkv.dtype)
            src = k
            ra = _lib.RopeArgs(dt, B, T, H, N, hs, 0, 0, _lib.tensor5(src), _lib.tensor5(qk_rot[:, :, H:]),
                               freqs.data_ptr())
            _lib.check(lib.dta_rope(ra, stream))
            k = qk_rot[:, :, H:]
            rope_args = (freqs.data_ptr(), _lib.tensor5(qk_rot[:, :, :H]))
        o = torch.empty(B, T, H, dv, device=dev, dtype=qkv.dtype)
        # the per-branch O_i for delta_i = <dO, O_i> (hence d(coef), d(lambda)), fp32
        obr = torch.empty(N, B, T, H, dv, device=dev, dtype=_obr_dtype(qkv.dtype))
        lse = torch.empty(N, B, H, T, device=dev, dtype=torch.float32)
        obr_t = _lib.DtaTensor(obr.data_ptr(), *obr.stride()[1:4], obr.stride(0))
        a = _lib.AttnFwdArgs(dt, B, T, H, N, hs, dv, scale, dropout_p,
                             _lib.tensor5(q), _lib.tensor5(k), _lib.tensor5(v), _lib.tensor5(o), obr_t,
                             lse.data_ptr(), coef.data_ptr(), seed, *rope_args, _lib.dtype_code(obr.dtype))
        with TIMER.region("attn_fwd"):
            _lib.check(lib.dta_attn_fwd(a, stream))
        ctx.save_for_backward(qkv, qk_rot, obr, lse, coef, freqs)
        ctx.dims = (H, N, hs, dv, scale)
        ctx.drop = (dropout_p, seed)
        # the backward branch-group caps in force at the forward (bwd_group_caps): saved here, so
        # a backward run after the block exits (or on another thread) uses the same caps
        ctx.caps = tuple(_BWD_GROUP_MAX)
        return o.view(B, T, H * dv)

    @staticmethod
    def backward(ctx, do: Tensor):
        lib = _lib.load()
        qkv, qk_rot, obr, lse, coef, freqs = ctx.saved_tensors
        H, N, hs, dv, scale = ctx.dims
        B, T, W = qkv.shape
        dev = qkv.device
        stream = _lib.stream_handle(dev)
        dt = _lib.dtype_code(qkv.dtype)
        do = do.to(qkv.dtype).contiguous().view(B, T, H, dv)
        q, k, v = split_packed(qkv, H, N, hs, dv)
        if qk_rot is not None:
            q, k = qk_rot[:, :, :H], qk_rot[:, :, H:]
        dqkv = torch.empty_like(qkv)
        dq, dk, dvv = split_packed(dqkv, H, N, hs, dv)
        dcoef = torch.empty(H, N, device=dev, dtype=torch.float32)
        delta = torch.empty(N, B, H, T, device=dev, dtype=torch.float32)
        # d(coef) from per-wave partials summed in a fixed order: reproducible lambda grads
        dcp = torch.empty(lib.dta_attn_bwd_dcoef_partial_bytes(B, T, H, N) // 4, device=dev, dtype=torch.float32)
        # dK/dV in more than one branch group: dV summed in fp32 across the groups (one rounding)
        dv32 = None
        caps = ctx.caps
        if dt != _lib.DTA_F32 and _DV_F32_WORKSPACE[0] and lib.dta_attn_bwd_dkdv_groups(dt, hs, N, dv, caps[1]) > 1:
            dv32 = torch.empty(B, T, H, dv, device=dev, dtype=torch.float32)
        # ABI 8: the |c_i|-folded key-major kernel's score seeds (16-bit, no dropout; private workspace)
        lsec = (torch.empty(N, B, H, T, device=dev, dtype=torch.float32)
                if dt != _lib.DTA_F32 and ctx.drop[0] == 0.0 and _LSE_C_WORKSPACE[0] else None)
        # with RoPE the kernels differentiate w.r.t. the rotated Q/K (qk_rot) and their
        # dQ / dK epilogues apply the inverse rotation, writing straight into dqkv
        obr_t = _lib.DtaTensor(obr.data_ptr(), *obr.stride()[1:4], obr.stride(0))
        a = _lib.AttnBwdArgs(dt, B, T, H, N, hs, dv, scale, ctx.drop[0],
                             _lib.tensor5(q), _lib.tensor5(k), _lib.tensor5(v), obr_t,
                             lse.data_ptr(), coef.data_ptr(), _lib.tensor5(do),
                             _lib.tensor5(dq), _lib.tensor5(dk), _lib.tensor5(dvv),
                             dcoef.data_ptr(), delta.data_ptr(), None, _lib.BWD_PRE,
                             freqs.data_ptr() if freqs is not None else None, dcp.data_ptr(), ctx.drop[1],
                             _lib.dtype_code(obr.dtype), *caps,
                             dv32.data_ptr() if dv32 is not None else None,
                             lsec.data_ptr() if lsec is not None else None)
        # (no PRE stage: with the d(coef) partials the DQ stage's ordered reduce writes dcoef whole)
        a.stages = _lib.BWD_DQ
        with TIMER.region("attn_bwd_dq"):
            _lib.check(lib.dta_attn_bwd(a, stream))
        a.stages = _lib.BWD_DKDV
        with TIMER.region("attn_bwd_dkdv"):
            _lib.check(lib.dta_attn_bwd(a, stream))
        return dqkv, dcoef, None, None, None, None, None, None, None, None


def diff_attention(qkv: Tensor, coef: Tensor, H: int, N: int, hs: int,
                   freqs: Optional[Tensor] = None, dv: Optional[int] = None, dropout_p: float = 0.0,
                   seed: Optional[int] = None) -> Tensor:
    """O = sum_i coef[h,i] dropout(softmax_causal(Q_i K_i^T/sqrt(hs))) V for every head.

    ``freqs``: fp32 (T, hs/2, 2) rotary table (view_as_real of freqs_cis[:T]) or None.
    ``dv``: value width per head; 2*hs for the differential models (default), hs for
    standard attention (N=1, coef 1: control.py:38-63).
    ``dropout_p``: nn.Dropout on every attention map (diff_transformer.py:66-67): each
    map element kept with probability 1-p and scaled by 1/(1-p), independently per map,
    from a counter-based hash of ``seed`` (include/diffattn.h); by default the seed is
    drawn from torch's generator, so ``torch.manual_seed`` makes runs repeatable.
    """
    if freqs is not None:
        freqs = freqs.to(device=qkv.device, dtype=torch.float32).contiguous()
    dropout_p = float(dropout_p)
    if not 0.0 <= dropout_p < 1.0:
        raise ValueError(f"dropout probability has to be in [0, 1), got {dropout_p}")
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if dropout_p > 0 else 0
    dv = 2 * hs if dv is None else dv
    scale = 1.0 / math.sqrt(hs)                 # diff_transformer.py:57, of the true head size
    hp = padded_head(qkv.dtype, hs, N, dv) if qkv.is_cuda else hs
    if hp is None:
        raise RuntimeError(f"no gfx950 kernel for head_size={hs}, n_terms={N}, dv={dv}, dtype={qkv.dtype} "
                           "(head sizes up to 256 are served; 129-256 in 16-bit for the differential models)")
    if hp == hs:
        return _DiffAttention.apply(qkv, coef, H, N, hs, freqs, dv, dropout_p, int(seed), scale)
    # a head size without its own plan runs in the next built one: Q_i / K_i zero-padded
    # to hp columns leave every score Q_i K_i^T unchanged (the softmax scale stays
    # 1/sqrt(hs)), V padded to dvp columns adds zero output columns, which are dropped;
    # the pad columns' gradients are discarded by the slices' backward
    dvp = hp if dv == hs else 2 * hp
    B, T, _ = qkv.shape
    q, k, v = split_packed(qkv, H, N, hs, dv)
    qkv_p = torch.cat([F.pad(q, (0, hp - hs)).flatten(2), F.pad(k, (0, hp - hs)).flatten(2),
                       F.pad(v, (0, dvp - dv)).flatten(2)], dim=-1)
    if freqs is not None:
        # identity rotation (cos 1, sin 0) on the pad pairs: they stay zero
        pad = torch.zeros(freqs.shape[0], (hp - hs) // 2, 2, device=freqs.device, dtype=freqs.dtype)
        pad[..., 0] = 1.0
        freqs = torch.cat([freqs, pad], dim=1).contiguous()
    out = _DiffAttention.apply(qkv_p, coef, H, N, hp, freqs, dvp, dropout_p, int(seed), scale)
    return out.view(B, T, H, dvp)[..., :dv].reshape(B, T, H * dv)


class _GroupLNScale(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, w: Tensor, b: Tensor, eps: float, out_scale: float, holder=None,
                y_dtype: Optional[torch.dtype] = None):
        lib = _lib.load()
        _require_gpu(x, w, b)
        # bound (dp.BucketedAllReduce, packing.bind_grad): dw/db accumulate straight into
        # the parameters' bucket-view gradients -- no zeros, no AccumulateGrad adds
        ctx.bound = (holder, (w, b)) if holder is not None and "grad" in holder else None
        C = x.shape[-1]
        x2 = x.contiguous().view(-1, C)
        rows = x2.shape[0]
        w32 = w.detach().to(torch.float32).contiguous().view(-1)
        b32 = b.detach().to(torch.float32).contiguous().view(-1)
        if w32.numel() != C or b32.numel() != C:
            raise RuntimeError("GroupLayerNorm weight/bias size must equal the normalised width")
        # io: an fp32 input normalised straight into a 16-bit output (and its backward
        # from that dtype's gradient), dta_ln_args.io_dtype
        io = 0
        if y_dtype is not None and y_dtype != x.dtype:
            if x.dtype != torch.float32 or y_dtype not in (torch.bfloat16, torch.float16):
                raise RuntimeError("LayerNorm output dtype may differ only for fp32 input and 16-bit output")
            io = 1 + _lib.dtype_code(y_dtype)
        y = torch.empty(x2.shape, device=x.device, dtype=y_dtype if io else x.dtype)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        a = _lib.LnArgs(_lib.dtype_code(x.dtype), rows, C, eps, out_scale, x2.data_ptr(), C, y.data_ptr(), C,
                        w32.data_ptr(), b32.data_ptr(), mean.data_ptr(), rstd.data_ptr(), None, 0, None, 0,
                        None, None, None, io)
        ctx.io = (io, y.dtype)
        _lib.check(lib.dta_ln_fwd(a, _lib.stream_handle(x.device)))
        ctx.save_for_backward(x2, w32, mean, rstd)
        ctx.meta = (eps, out_scale, x.shape, w.dtype, w.shape, b.dtype, b.shape)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy: Tensor):
        lib = _lib.load()
        x2, w32, mean, rstd = ctx.saved_tensors
        eps, out_scale, xshape, wdt, wshape, bdt, bshape = ctx.meta
        C = x2.shape[1]
        io, ydt = ctx.io
        dy2 = dy.to(ydt).contiguous().view(-1, C)
        dx = torch.empty_like(x2)
        g = None
        if ctx.bound is not None and ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
            holder, params = ctx.bound
            g = packing._grad_target(holder, params)
            if g is not None and g.numel() != 2 * C:
                g = None
        if g is not None:
            dw, db = g[:C], g[C:]
        else:
            dw = torch.zeros(C, device=x2.device, dtype=torch.float32)
            db = torch.zeros(C, device=x2.device, dtype=torch.float32)
        # per-block column partials summed in order: reproducible dw / db (no atomics)
        part = torch.empty(lib.dta_ln_bwd_workspace_bytes(x2.shape[0], C) // 4, device=x2.device, dtype=torch.float32)
        a = _lib.LnArgs(_lib.dtype_code(x2.dtype), x2.shape[0], C, eps, out_scale, x2.data_ptr(), C, None, 0,
                        w32.data_ptr(), None, mean.data_ptr(), rstd.data_ptr(), dy2.data_ptr(), C,
                        dx.data_ptr(), C, dw.data_ptr(), db.data_ptr(), part.data_ptr(), io)
        _lib.check(lib.dta_ln_bwd(a, _lib.stream_handle(x2.device)))
        if g is not None:
            hook = ctx.bound[0]["on_ready"]
            for p in ctx.bound[1]:
                hook(p)
            return dx.view(xshape), None, None, None, None, None, None
        return dx.view(xshape), dw.to(wdt).view(wshape), db.to(bdt).view(bshape), None, None, None, None


class _AddLN(torch.autograd.Function):
    """(x + a, LayerNorm(x + a)) in one pass: a Block's residual add feeding its next
    pre-LN (diff_transformer.py:121-125), fp32 residual stream x, 16-bit branch output a
    and LN output.  Backward: the residual gradient d(x + a) plus the LN backward, in one
    pass that also writes the branch's 16-bit gradient."""

    @staticmethod
    def forward(ctx, x: Tensor, a: Tensor, w: Tensor, b: Tensor, eps: float, holder, ydt: torch.dtype):
        lib = _lib.load()
        _require_gpu(x, a, w, b)
        C = x.shape[-1]
        x2 = x.contiguous().view(-1, C)
        a2 = a.to(ydt).contiguous().view(-1, C)
        rows = x2.shape[0]
        w32 = w.detach().to(torch.float32).contiguous().view(-1)
        b32 = b.detach().to(torch.float32).contiguous().view(-1)
        xo = torch.empty_like(x2)
        y = torch.empty(x2.shape, device=x.device, dtype=ydt)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        io = 1 + _lib.dtype_code(ydt)
        args = _lib.LnArgs(_lib.DTA_F32, rows, C, eps, 1.0, x2.data_ptr(), C, y.data_ptr(), C,
                           w32.data_ptr(), b32.data_ptr(), mean.data_ptr(), rstd.data_ptr(), None, 0, None, 0,
                           None, None, None, io, a2.data_ptr(), C, xo.data_ptr(), C)
        _lib.check(lib.dta_ln_fwd(args, _lib.stream_handle(x.device)))
        ctx.bound = (holder, (w, b)) if holder is not None and "grad" in holder else None
        ctx.save_for_backward(xo, w32, mean, rstd)
        ctx.meta = (eps, x.shape, a.dtype, ydt, w.dtype, w.shape, b.dtype, b.shape, io)
        return xo.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, dxo: Optional[Tensor], dy: Optional[Tensor]):
        lib = _lib.load()
        xo, w32, mean, rstd = ctx.saved_tensors
        eps, xshape, adt, ydt, wdt, wshape, bdt, bshape, io = ctx.meta
        C = xo.shape[1]
        dy2 = (dy.to(ydt).contiguous().view(-1, C) if dy is not None
               else torch.zeros(xo.shape, device=xo.device, dtype=ydt))
        dres = dxo.to(torch.float32).contiguous().view(-1, C) if dxo is not None else None
        dx = torch.empty_like(xo)
        da = torch.empty(xo.shape, device=xo.device, dtype=ydt)
        g = None
        if ctx.bound is not None and ctx.needs_input_grad[2] and ctx.needs_input_grad[3]:
            holder, params = ctx.bound
            g = packing._grad_target(holder, params)
            if g is not None and g.numel() != 2 * C:
                g = None
        if g is not None:
            dw, db = g[:C], g[C:]
        else:
            dw = torch.zeros(C, device=xo.device, dtype=torch.float32)
            db = torch.zeros(C, device=xo.device, dtype=torch.float32)
        part = torch.empty(lib.dta_ln_bwd_workspace_bytes(xo.shape[0], C) // 4, device=xo.device, dtype=torch.float32)
        args = _lib.LnArgs(_lib.DTA_F32, xo.shape[0], C, eps, 1.0, xo.data_ptr(), C, None, 0, w32.data_ptr(), None,
                           mean.data_ptr(), rstd.data_ptr(), dy2.data_ptr(), C, dx.data_ptr(), C, dw.data_ptr(),
                           db.data_ptr(), part.data_ptr(), io, None, 0, None, 0,
                           dres.data_ptr() if dres is not None else None, C, da.data_ptr(), C)
        _lib.check(lib.dta_ln_bwd(args, _lib.stream_handle(xo.device)))
        da_out = da.view(xshape).to(adt)
        if g is not None:
            hook = ctx.bound[0]["on_ready"]
            for p in ctx.bound[1]:
                hook(p)
            return dx.view(xshape), da_out, None, None, None, None, None
        return dx.view(xshape), da_out, dw.to(wdt).view(wshape), db.to(bdt).view(bshape), None, None, None


def add_layer_norm(x: Tensor, a: Tensor, ln: "LayerNorm"):
    """(x + a, ln(x + a)) -- a Block's residual add and the following pre-LN
    (diff_transformer.py:121-125).  One fused pass when x is the fp32 residual stream
    under autocast and ln emits the autocast dtype; otherwise the two ops."""
    C = x.shape[-1]
    if (_RES_FUSE and x.is_cuda and x.dtype == torch.float32 and isinstance(ln, LayerNorm) and ln.autocast_out
            and torch.is_autocast_enabled("cuda") and ln.weight is not None and ln.bias is not None
            and len(ln.normalized_shape) == 1 and C % 8 == 0 and C <= 8192 and a.shape == x.shape
            and a.dtype in (torch.bfloat16, torch.float16)):
        ydt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return _AddLN.apply(x, a, ln.weight, ln.bias, ln.eps, ln._gpack, ydt)
    xo = x + a
    return xo, ln(xo)


_RES_FUSE = os.environ.get("DTA_RES_FUSE", "1") != "0"        # A/B switch: 0 = add, then LayerNorm
_SWIGLU_BIAS = os.environ.get("DTA_SWIGLU_BIAS", "1") != "0"   # A/B switch: 0 = bias gradient by torch's sum


def group_ln_scale(x: Tensor, w: Tensor, b: Tensor, eps: float = 1e-5, out_scale: float = 1.0,
                   holder: Optional[Dict] = None) -> Tensor:
    """``holder``: the module's grad-binding dict (``param_packs``), or None."""
    return _GroupLNScale.apply(x, w, b, eps, out_scale, holder, None)


class LayerNorm(torch.nn.LayerNorm):
    """``nn.LayerNorm`` of the Blocks (``ln1``/``ln2``/``ln_f``: diff_transformer.py:111-126,
    Ndiff_transformer.py:164-179, control.py:92-111) on the HIP LN kernels for GPU
    tensors: same parameters, ``state_dict`` keys and fp32 statistics; under autocast
    it normalises in fp32 like ``F.layer_norm``'s autocast rule.  Host tensors (the
    control model on the CPU) and shapes the kernels do not take keep PyTorch's."""

    def __init__(self, *args, autocast_out: bool = False, **kwargs):
        super().__init__(*args, **kwargs)
        self._gpack = {}                      # grad binding of (weight, bias), dp.BucketedAllReduce
        # autocast_out: under autocast, write the output in the autocast dtype -- exact
        # when every consumer is an autocast GEMM (which would cast it anyway: the
        # Blocks' ln1/ln2/ln_f), and it saves the separate cast there and back
        self.autocast_out = autocast_out

    def param_packs(self):
        return [(self._gpack, [self.weight, self.bias])] if self.weight is not None and self.bias is not None else []

    def forward(self, x: Tensor) -> Tensor:
        C = x.shape[-1]
        if (not x.is_cuda or len(self.normalized_shape) != 1 or self.weight is None or self.bias is None
                or C % 8 or C > 8192):
            return super().forward(x)
        ydt = None
        if torch.is_autocast_enabled("cuda"):
            if x.dtype != torch.float32:
                x = x.float()
            if self.autocast_out:
                ydt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return _GroupLNScale.apply(x, self.weight, self.bias, self.eps, 1.0, self._gpack, ydt)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a: Tensor, b: Tensor):
        lib = _lib.load()
        _require_gpu(a, b)
        if a.shape != b.shape:
            raise RuntimeError("SwiGLU branches must have one shape")
        dt = torch.promote_types(a.dtype, b.dtype)
        a2 = a.to(dt).contiguous().view(-1, a.shape[-1])
        b2 = b.to(dt).contiguous().view(-1, a.shape[-1])
        out = torch.empty_like(a2)
        n = a2.shape[1]
        sa = _lib.SwigluArgs(_lib.dtype_code(dt), a2.shape[0], n, a2.data_ptr(), n, b2.data_ptr(), n,
                             out.data_ptr(), n, None, 0, None, 0, None, 0)
        _lib.check(lib.dta_swiglu_fwd(sa, _lib.stream_handle(a.device)))
        ctx.save_for_backward(a2, b2)
        ctx.meta = (a.shape, a.dtype, b.dtype)
        return out.view(a.shape)

    @staticmethod
    def backward(ctx, dout: Tensor):
        lib = _lib.load()
        a2, b2 = ctx.saved_tensors
        shape, adt, bdt = ctx.meta
        n = a2.shape[1]
        d2 = dout.to(a2.dtype).contiguous().view(-1, n)
        da, db = torch.empty_like(a2), torch.empty_like(b2)
        sa = _lib.SwigluArgs(_lib.dtype_code(a2.dtype), a2.shape[0], n, a2.data_ptr(), n, b2.data_ptr(), n,
                             None, 0, d2.data_ptr(), n, da.data_ptr(), n, db.data_ptr(), n)
        _lib.check(lib.dta_swiglu_bwd(sa, _lib.stream_handle(a2.device)))
        return da.view(shape).to(adt), db.view(shape).to(bdt)


def swiglu(a: Tensor, b: Tensor) -> Tensor:
    """``F.silu(a) * b`` in one pass forward and one backward (SwiGLU.forward of the
    reference models); GPU tensors whose last dim is a multiple of 8."""
    if not a.is_cuda or a.shape[-1] % 8 or a.shape != b.shape:
        return F.silu(a) * b
    return _SwiGLU.apply(a, b)


def _swiglu_launch(y2: Tensor, n: int, out: Optional[Tensor], dout: Optional[Tensor], dy: Optional[Tensor],
                   dbias: Optional[Tensor] = None):
    """dta_swiglu over the column halves of a packed (rows, 2n) projection: a = y2[:, :n],
    b = y2[:, n:]; forward writes ``out`` (rows, n), backward writes da | db into the halves
    of ``dy`` (rows, 2n)."""
    lib = _lib.load()
    es, rows, w = y2.element_size(), y2.shape[0], 2 * n
    a, b = y2.data_ptr(), y2.data_ptr() + n * es
    if dy is None:
        sa = _lib.SwigluArgs(_lib.dtype_code(y2.dtype), rows, n, a, w, b, w, out.data_ptr(), n,
                             None, 0, None, 0, None, 0)
        _lib.check(lib.dta_swiglu_fwd(sa, _lib.stream_handle(y2.device)))
    else:
        work = None
        if dbias is not None:
            work = torch.empty(lib.dta_swiglu_bwd_workspace_bytes(rows, n) // 4 + 4, device=y2.device,
                               dtype=torch.float32)
        sa = _lib.SwigluArgs(_lib.dtype_code(y2.dtype), rows, n, a, w, b, w, None, 0, dout.data_ptr(), n,
                             dy.data_ptr(), w, dy.data_ptr() + n * es, w,
                             dbias.data_ptr() if dbias is not None else None,
                             work.data_ptr() if work is not None else None)
        _lib.check(lib.dta_swiglu_bwd(sa, _lib.stream_handle(y2.device)))


class _PackedSwiGLU(torch.autograd.Function):
    """SwiGLU with its gate and xform Linears as ONE GEMM over a shared weight pack
    ``[W_gate; W_xform]`` (and bias pack): one (rows, 2n) projection whose halves feed
    the fused SwiGLU kernel; backward writes dA | dB into one (rows, 2n) gradient, so
    dX is one GEMM (K = 2n) instead of two plus an add, dW one GEMM and the bias
    gradient one column sum.  Casts as autocast applies them to the two nn.Linear."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, wbase, bbase, wholder, bholder, *params):
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        xc = x.to(dt)
        wc, bc = wbase.to(dt), bbase.view(-1).to(dt)
        with torch.autocast("cuda", enabled=False):
            y = F.linear(xc, wc, bc)
        n = wc.shape[0] // 2
        y2 = y.view(-1, 2 * n)
        out = torch.empty(y2.shape[0], n, device=y.device, dtype=y.dtype)
        _swiglu_launch(y2, n, out, None, None)
        ctx.save_for_backward(xc, wc, y2)
        ctx.x_dtype, ctx.w_dtype, ctx.n = x.dtype, wbase.dtype, n
        ctx.wrows = [params[0].shape[0], params[1].shape[0]]
        bound = (wholder is not None and "grad" in wholder and bholder is not None and "grad" in bholder)
        ctx.holders = (wholder, bholder) if bound else None
        ctx.params = params if bound else None
        return out.view(*x.shape[:-1], n)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dout):
        xc, wc, y2 = ctx.saved_tensors
        n = ctx.n
        d2 = dout.to(y2.dtype).contiguous().view(-1, n)
        dy = torch.empty_like(y2)
        # the bias gradient (column sums of dA | dB as stored) comes out of the same pass
        db = torch.empty(2 * n, device=y2.device, dtype=torch.float32) if _SWIGLU_BIAS else None
        _swiglu_launch(y2, n, None, d2, dy, db)
        with torch.autocast("cuda", enabled=False):
            dx = (dy @ wc).view(*xc.shape[:-1], xc.shape[-1]).to(ctx.x_dtype) if ctx.needs_input_grad[0] else None
            dw = packing.weight_grad(dy, xc.reshape(-1, xc.shape[-1]))
            if db is None:
                db = dy.sum(0)
        if ctx.holders is not None and all(ctx.needs_input_grad[5:]):
            wh, bh = ctx.holders
            gw = packing._grad_target(wh, ctx.params[:2])
            gb = packing._grad_target(bh, ctx.params[2:])
            if gw is not None and gb is not None:
                packing.accumulate(gw, dw)          # one launch each, bf16 -> fp32 in the add
                packing.accumulate(gb, db)
                for h, ps in ((wh, ctx.params[:2]), (bh, ctx.params[2:])):
                    for p in ps:
                        h["on_ready"](p)
                return (dx, None, None, None, None) + (None,) * 4
        dw = dw.to(ctx.w_dtype)
        db = db.to(ctx.w_dtype)
        gwg, gwx = torch.split(dw, ctx.wrows, 0)
        gbg, gbx = torch.split(db, ctx.wrows, 0)
        return (dx, None, None, None, None, gwg, gwx, gbg, gbx)


class _Linear(torch.autograd.Function):
    """``nn.Linear`` under the same autocast casts, with its weight gradient through
    ``packing.weight_grad`` (fp32 output, split over tokens when the output is small)."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, w, b):
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        xc, wc = x.to(dt), w.to(dt)
        bc = b.to(dt) if b is not None else None
        with torch.autocast("cuda", enabled=False):
            y = F.linear(xc, wc, bc)
        ctx.save_for_backward(xc, wc)
        ctx.dtypes = (x.dtype, w.dtype, b.dtype if b is not None else None)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        xdt, wdt, bdt = ctx.dtypes
        dy2 = dy.to(wc.dtype).reshape(-1, wc.shape[0])
        with torch.autocast("cuda", enabled=False):
            dx = (dy2 @ wc).view(*xc.shape[:-1], wc.shape[1]).to(xdt) if ctx.needs_input_grad[0] else None
            dw = packing.weight_grad(dy2, xc.reshape(-1, xc.shape[-1])).to(wdt) if ctx.needs_input_grad[1] else None
            db = dy2.sum(0).to(bdt) if bdt is not None and ctx.needs_input_grad[2] else None
        return dx, dw, db


def linear(x: Tensor, mod: torch.nn.Linear) -> Tensor:
    """``mod(x)`` for the reference's nn.Linear layers on the hot path's callers (the MHA
    output projection, the FFN output); GPU: ``_Linear``, else the module itself."""
    if not x.is_cuda or not x.is_floating_point():
        return mod(x)
    return _Linear.apply(x, mod.weight, mod.bias)


def ffn(seq: torch.nn.Sequential, x: Tensor) -> Tensor:
    """The Block's ``ffwd = Sequential(SwiGLU, Linear(4C, C), Dropout)`` (diff_transformer.py:114-119)
    with its Linear through ``linear``."""
    return seq[2](linear(seq[0](x), seq[1]))


def packed_swiglu(x: Tensor, gate: torch.nn.Linear, xform: torch.nn.Linear, wholder: Dict, bholder: Dict) -> Tensor:
    """SwiGLU.forward of the reference models (silu(W_g x + b_g) * (W_x x + b_x)) with
    both Linears' parameters as row views of shared packs (packing.ensure_packed)."""
    wparams, bparams = [gate.weight, xform.weight], [gate.bias, xform.bias]
    n = gate.weight.shape[0]
    if (not x.is_cuda or n % 8 or xform.weight.shape != gate.weight.shape or gate.bias is None
            or xform.bias is None or gate.weight.dtype != xform.weight.dtype):
        return swiglu(gate(x), xform(x))
    wbase = packing.ensure_packed(wparams, wholder)
    bbase = packing.ensure_packed(bparams, bholder)
    return _PackedSwiGLU.apply(x, wbase, bbase, wholder, bholder, *wparams, *bparams)


# ------------------------------------------------------------------ decode ---
def rope_rows(src: Tensor, dst: Tensor, table: Tensor) -> None:
    """dst = RoPE(src) for (B, T, H, N, hs) views whose rows are the positions of
    ``table`` (fp32 (T, hs/2, 2), already sliced to those positions).  No autograd:
    the KV-cache path of generate() only (Ndiff_transformer.py:11-22, 104-109)."""
    lib = _lib.load()
    _require_gpu(src, dst, table)
    B, T, H, N, hs = src.shape
    table = table.to(device=src.device, dtype=torch.float32).contiguous()
    ra = _lib.RopeArgs(_lib.dtype_code(dst.dtype), B, T, H, N, hs, 0, 0, _lib.tensor5(src), _lib.tensor5(dst),
                       table.data_ptr())
    _lib.check(lib.dta_rope(ra, _lib.stream_handle(src.device)))


def diff_attention_decode(q: Tensor, k_cache: Tensor, v_cache: Tensor, coef: Tensor, length: int,
                          length_dev: Optional[Tensor] = None) -> Tensor:
    """One new query row per (b, h) against the first ``length`` cached keys:
    o = sum_i coef[h,i] softmax(q_i K_i[:length]^T / sqrt(hs)) V[:length].

    q: (B, H, N, hs); k_cache: (B, T_cap, H, N, hs); v_cache: (B, T_cap, H, dv)
    (strided views, innermost dim contiguous).  Returns (B, H*dv).  Equals the last
    row of ``diff_attention`` over the same ``length`` positions (the causal mask
    keeps every key up to the query's own position).

    ``length_dev``: optional device int32 scalar holding the length, read by the
    kernels, so one captured HIP graph serves every position; ``length`` is then
    its upper bound (the cache capacity)."""
    lib = _lib.load()
    _require_gpu(q, k_cache, v_cache, coef)
    B, H, N, hs = q.shape
    T_cap, dv = k_cache.shape[1], v_cache.shape[-1]
    if tuple(k_cache.shape) != (B, T_cap, H, N, hs) or tuple(v_cache.shape) != (B, T_cap, H, dv):
        raise RuntimeError("k_cache/v_cache shapes do not match q")
    if not 1 <= length <= T_cap:
        raise RuntimeError(f"decode length {length} outside [1, {T_cap}]")
    if q.dtype != k_cache.dtype or q.dtype != v_cache.dtype:
        raise RuntimeError("q, k_cache and v_cache must share a dtype")
    if length_dev is not None:
        _require_gpu(length_dev)
        if length_dev.dtype != torch.int32 or length_dev.numel() != 1:
            raise RuntimeError("length_dev must be one device int32")
    coef = coef.detach().to(torch.float32).contiguous()
    o = torch.empty(B, 1, H, dv, device=q.device, dtype=q.dtype)
    nbytes = lib.dta_attn_decode_workspace_bytes(B, H, N, hs, dv, T_cap)
    ws = torch.empty(nbytes // 4, device=q.device, dtype=torch.float32)
    a = _lib.DecodeArgs(_lib.dtype_code(q.dtype), B, H, N, hs, dv, length, T_cap, 1.0 / math.sqrt(hs),
                        _lib.tensor5(q.unsqueeze(1)), _lib.tensor5(k_cache), _lib.tensor5(v_cache),
                        _lib.tensor5(o), coef.data_ptr(), ws.data_ptr(),
                        None if length_dev is None else length_dev.data_ptr())
    _lib.check(lib.dta_attn_decode(a, _lib.stream_handle(q.device)))
    return o.view(B, H * dv)
