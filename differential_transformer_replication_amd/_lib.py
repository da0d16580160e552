"""ctypes binding of ``libdiffattn.so`` (C ABI declared in ``include/diffattn.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C
differential_transformer_replication_amd/csrc``) for gfx950 only.  There is no
fallback: if the library is missing or cannot load, every op raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DTA_LIB", os.path.join(_HERE, "lib", "libdiffattn.so"))

DTA_BF16, DTA_F16, DTA_F32 = 0, 1, 2
_DTYPES = {torch.bfloat16: DTA_BF16, torch.float16: DTA_F16, torch.float32: DTA_F32}

ABI_VERSION = 8

# every symbol include/diffattn.h declares
EXPORTS = ("dta_attn_fwd", "dta_attn_bwd", "dta_attn_bwd_workspace_bytes", "dta_attn_bwd_dcoef_partial_bytes",
           "dta_ln_fwd", "dta_ln_bwd", "dta_ln_bwd_workspace_bytes",
           "dta_rope", "dta_cast_f32", "dta_error_string", "dta_abi_version", "dta_supported",
           "dta_attn_decode", "dta_attn_decode_workspace_bytes", "dta_swiglu_fwd", "dta_swiglu_bwd",
           "dta_accumulate_f32", "dta_swiglu_bwd_workspace_bytes", "dta_attn_bwd_dkdv_groups")


class DtaTensor(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("sb", ctypes.c_int64), ("st", ctypes.c_int64),
                ("sh", ctypes.c_int64), ("si", ctypes.c_int64)]


class SwigluArgs(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("rows", ctypes.c_int64), ("n", ctypes.c_int64),
                ("a", ctypes.c_void_p), ("a_stride", ctypes.c_int64),
                ("b", ctypes.c_void_p), ("b_stride", ctypes.c_int64),
                ("out", ctypes.c_void_p), ("out_stride", ctypes.c_int64),
                ("dout", ctypes.c_void_p), ("dout_stride", ctypes.c_int64),
                ("da", ctypes.c_void_p), ("da_stride", ctypes.c_int64),
                ("db", ctypes.c_void_p), ("db_stride", ctypes.c_int64),
                ("dbias", ctypes.c_void_p), ("dbias_work", ctypes.c_void_p)]


class AttnFwdArgs(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("B", ctypes.c_int32), ("T", ctypes.c_int32),
                ("H", ctypes.c_int32), ("n_terms", ctypes.c_int32), ("head_size", ctypes.c_int32),
                ("dv", ctypes.c_int32), ("scale", ctypes.c_float), ("dropout_p", ctypes.c_float),
                ("q", DtaTensor), ("k", DtaTensor), ("v", DtaTensor), ("o", DtaTensor),
                ("obr", DtaTensor), ("lse", ctypes.c_void_p), ("coef", ctypes.c_void_p),
                ("dropout_seed", ctypes.c_uint64), ("rope_freqs", ctypes.c_void_p), ("q_rot", DtaTensor),
                ("obr_dtype", ctypes.c_int32)]


class AttnBwdArgs(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("B", ctypes.c_int32), ("T", ctypes.c_int32),
                ("H", ctypes.c_int32), ("n_terms", ctypes.c_int32), ("head_size", ctypes.c_int32),
                ("dv", ctypes.c_int32), ("scale", ctypes.c_float), ("dropout_p", ctypes.c_float),
                ("q", DtaTensor), ("k", DtaTensor), ("v", DtaTensor), ("obr", DtaTensor),
                ("lse", ctypes.c_void_p), ("coef", ctypes.c_void_p), ("dout", DtaTensor),
                ("dq", DtaTensor), ("dk", DtaTensor), ("dv_out", DtaTensor),
                ("dcoef", ctypes.c_void_p), ("delta", ctypes.c_void_p), ("dq_f32", ctypes.c_void_p),
                ("stages", ctypes.c_int32), ("rope_freqs", ctypes.c_void_p), ("dcoef_partial", ctypes.c_void_p),
                ("dropout_seed", ctypes.c_uint64), ("obr_dtype", ctypes.c_int32),
                ("group_max_dq", ctypes.c_int32), ("group_max_dkdv", ctypes.c_int32),
                ("dv_f32", ctypes.c_void_p), ("lse_c", ctypes.c_void_p)]


BWD_PRE, BWD_DQ, BWD_DKDV = 1, 2, 4


class LnArgs(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("rows", ctypes.c_int64), ("C", ctypes.c_int64),
                ("eps", ctypes.c_float), ("out_scale", ctypes.c_float),
                ("x", ctypes.c_void_p), ("x_stride", ctypes.c_int64),
                ("y", ctypes.c_void_p), ("y_stride", ctypes.c_int64),
                ("w", ctypes.c_void_p), ("b", ctypes.c_void_p),
                ("mean", ctypes.c_void_p), ("rstd", ctypes.c_void_p),
                ("dy", ctypes.c_void_p), ("dy_stride", ctypes.c_int64),
                ("dx", ctypes.c_void_p), ("dx_stride", ctypes.c_int64),
                ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p), ("partial", ctypes.c_void_p), ("io_dtype", ctypes.c_int32),
                ("res", ctypes.c_void_p), ("res_stride", ctypes.c_int64), ("xo", ctypes.c_void_p),
                ("xo_stride", ctypes.c_int64), ("dres", ctypes.c_void_p), ("dres_stride", ctypes.c_int64),
                ("dx16", ctypes.c_void_p), ("dx16_stride", ctypes.c_int64)]


class RopeArgs(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("B", ctypes.c_int32), ("T", ctypes.c_int32),
                ("H", ctypes.c_int32), ("n_terms", ctypes.c_int32), ("head_size", ctypes.c_int32),
                ("inverse", ctypes.c_int32), ("src_f32", ctypes.c_int32),
                ("src", DtaTensor), ("dst", DtaTensor), ("freqs", ctypes.c_void_p)]


class DecodeArgs(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("B", ctypes.c_int32), ("H", ctypes.c_int32),
                ("n_terms", ctypes.c_int32), ("head_size", ctypes.c_int32), ("dv", ctypes.c_int32),
                ("length", ctypes.c_int32), ("t_cap", ctypes.c_int32), ("scale", ctypes.c_float),
                ("q", DtaTensor), ("k_cache", DtaTensor), ("v_cache", DtaTensor), ("o", DtaTensor),
                ("coef", ctypes.c_void_p), ("workspace", ctypes.c_void_p), ("length_dev", ctypes.c_void_p)]


_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and type the library.  Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(f"libdiffattn.so not found at {path}: run __graft_entry__.build() "
                               "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        lib = ctypes.CDLL(path)
        P = ctypes.POINTER
        lib.dta_attn_fwd.argtypes = [P(AttnFwdArgs), ctypes.c_void_p]
        lib.dta_attn_bwd.argtypes = [P(AttnBwdArgs), ctypes.c_void_p]
        lib.dta_ln_fwd.argtypes = [P(LnArgs), ctypes.c_void_p]
        lib.dta_ln_bwd.argtypes = [P(LnArgs), ctypes.c_void_p]
        lib.dta_rope.argtypes = [P(RopeArgs), ctypes.c_void_p]
        lib.dta_swiglu_fwd.argtypes = [P(SwigluArgs), ctypes.c_void_p]
        lib.dta_swiglu_bwd.argtypes = [P(SwigluArgs), ctypes.c_void_p]
        lib.dta_cast_f32.argtypes = [ctypes.c_int32] * 6 + [ctypes.c_void_p, DtaTensor, ctypes.c_void_p]
        lib.dta_swiglu_bwd_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64]
        lib.dta_swiglu_bwd_workspace_bytes.restype = ctypes.c_size_t
        lib.dta_accumulate_f32.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]
        lib.dta_attn_decode.argtypes = [P(DecodeArgs), ctypes.c_void_p]
        lib.dta_attn_decode_workspace_bytes.argtypes = [ctypes.c_int32] * 6
        lib.dta_attn_decode_workspace_bytes.restype = ctypes.c_size_t
        lib.dta_attn_bwd_workspace_bytes.argtypes = [ctypes.c_int32] * 5
        lib.dta_attn_bwd_workspace_bytes.restype = ctypes.c_size_t
        lib.dta_attn_bwd_dcoef_partial_bytes.argtypes = [ctypes.c_int32] * 4
        lib.dta_attn_bwd_dcoef_partial_bytes.restype = ctypes.c_size_t
        lib.dta_ln_bwd_workspace_bytes.argtypes = [ctypes.c_int64] * 2
        lib.dta_ln_bwd_workspace_bytes.restype = ctypes.c_size_t
        lib.dta_error_string.argtypes = [ctypes.c_int]
        lib.dta_error_string.restype = ctypes.c_char_p
        lib.dta_supported.argtypes = [ctypes.c_int32] * 4
        lib.dta_attn_bwd_dkdv_groups.argtypes = [ctypes.c_int32] * 5
        for fn in ("dta_attn_fwd", "dta_attn_bwd", "dta_attn_decode", "dta_ln_fwd", "dta_ln_bwd", "dta_rope", "dta_cast_f32",
                   "dta_abi_version", "dta_supported", "dta_swiglu_fwd", "dta_swiglu_bwd", "dta_accumulate_f32",
                   "dta_attn_bwd_dkdv_groups"):
            getattr(lib, fn).restype = ctypes.c_int
        if lib.dta_abi_version() != ABI_VERSION:
            raise RuntimeError(f"libdiffattn ABI {lib.dta_abi_version()} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().dta_error_string(rc).decode()
        raise RuntimeError(f"libdiffattn: {msg} (code {rc})")


def dtype_code(t: torch.dtype) -> int:
    try:
        return _DTYPES[t]
    except KeyError:
        raise RuntimeError(f"libdiffattn supports bf16, fp16 and fp32 activations, got {t}") from None


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def tensor5(t: torch.Tensor) -> DtaTensor:
    """[b][t][h][i][d] (5-d) or [b][t][h][e] (4-d) view -> strides struct."""
    if t.dim() == 5:
        sb, st, sh, si, sd = t.stride()
    elif t.dim() == 4:
        sb, st, sh, sd = t.stride()
        si = 0
    else:
        raise ValueError("expected a 4-d or 5-d view")
    if sd != 1:
        raise RuntimeError("innermost dimension must be contiguous")
    return DtaTensor(t.data_ptr(), sb, st, sh, si)


def supported(dtype: torch.dtype, head_size: int, n_terms: int, dv: int) -> bool:
    return bool(load().dta_supported(dtype_code(dtype), head_size, n_terms, dv))
