// capi.hip -- the extern "C" boundary of libdiffattn.so (include/diffattn.h).
// Validates every argument, then enqueues kernels on the caller's stream.
// Nothing here allocates, synchronises or keeps state.
#include "../../include/diffattn.h"
#include "dta_internal.h"

namespace dta {
int launch_attn_fwd_bf16(const FwdParams&, hipStream_t);
int launch_attn_fwd_f16(const FwdParams&, hipStream_t);
int launch_attn_fwd_f32(const FwdParams&, hipStream_t);
int launch_attn_dq_bf16(const BwdParams&, hipStream_t);
int launch_attn_dq_f16(const BwdParams&, hipStream_t);
int launch_attn_dq_f32(const BwdParams&, hipStream_t);
int launch_attn_dkdv_bf16(const BwdParams&, hipStream_t);
int launch_attn_dkdv_f16(const BwdParams&, hipStream_t);
int launch_attn_dkdv_f32(const BwdParams&, hipStream_t);
int launch_attn_fwd_bf16_drop(const FwdParams&, hipStream_t);
int launch_attn_fwd_f16_drop(const FwdParams&, hipStream_t);
int launch_attn_fwd_f32_drop(const FwdParams&, hipStream_t);
int launch_attn_dq_bf16_drop(const BwdParams&, hipStream_t);
int launch_attn_dq_f16_drop(const BwdParams&, hipStream_t);
int launch_attn_dq_f32_drop(const BwdParams&, hipStream_t);
int launch_attn_dkdv_bf16_drop(const BwdParams&, hipStream_t);
int launch_attn_dkdv_f16_drop(const BwdParams&, hipStream_t);
int launch_attn_dkdv_f32_drop(const BwdParams&, hipStream_t);
bool attn_native_bf16(int, int, int);
bool attn_native_f16(int, int, int);
bool attn_native_f32(int, int, int);

int launch_attn_fwd(int dtype, const FwdParams& p, hipStream_t st) {
  if (p.drop_thr) switch (dtype) {
    case DTA_BF16: return launch_attn_fwd_bf16_drop(p, st);
    case DTA_F16: return launch_attn_fwd_f16_drop(p, st);
    case DTA_F32: return launch_attn_fwd_f32_drop(p, st);
  }
  switch (dtype) {
    case DTA_BF16: return launch_attn_fwd_bf16(p, st);
    case DTA_F16: return launch_attn_fwd_f16(p, st);
    case DTA_F32: return launch_attn_fwd_f32(p, st);
  }
  return -2;
}
int launch_attn_dq(int dtype, const BwdParams& p, hipStream_t st) {
  if (p.drop_thr) switch (dtype) {
    case DTA_BF16: return launch_attn_dq_bf16_drop(p, st);
    case DTA_F16: return launch_attn_dq_f16_drop(p, st);
    case DTA_F32: return launch_attn_dq_f32_drop(p, st);
  }
  switch (dtype) {
    case DTA_BF16: return launch_attn_dq_bf16(p, st);
    case DTA_F16: return launch_attn_dq_f16(p, st);
    case DTA_F32: return launch_attn_dq_f32(p, st);
  }
  return -2;
}
int launch_attn_dkdv(int dtype, const BwdParams& p, hipStream_t st) {
  if (p.drop_thr) switch (dtype) {
    case DTA_BF16: return launch_attn_dkdv_bf16_drop(p, st);
    case DTA_F16: return launch_attn_dkdv_f16_drop(p, st);
    case DTA_F32: return launch_attn_dkdv_f32_drop(p, st);
  }
  switch (dtype) {
    case DTA_BF16: return launch_attn_dkdv_bf16(p, st);
    case DTA_F16: return launch_attn_dkdv_f16(p, st);
    case DTA_F32: return launch_attn_dkdv_f32(p, st);
  }
  return -2;
}
bool attn_native(int dtype, int hs, int n, int dv) {
  // dv = 2 hs (differential models) or, for standard attention (N = 1), dv = hs
  if (dv != 2 * hs && !(n == 1 && dv == hs)) return false;
  switch (dtype) {
    case DTA_BF16: return attn_native_bf16(hs, n, dv);
    case DTA_F16: return attn_native_f16(hs, n, dv);
    case DTA_F32: return attn_native_f32(hs, n, dv);
  }
  return false;
}
// Every branch count runs: natively, or -- where no N-branch plan is built (N >= 5, fp32
// N = 3 / 4 at head sizes 96 / 128) -- as branch groups that each have one, on top of the
// single-branch plan (the forward then runs branch-split, the backward group by group).
bool attn_supported(int dtype, int hs, int n, int dv) {
  if (n < 1) return false;
  return attn_native(dtype, hs, n, dv) || (n >= 2 && dv == 2 * hs && attn_native(dtype, hs, 1, dv));
}
// size of the next branch group of the backward: the largest native branch count <= cap
int branch_group(int dtype, int hs, int left, int dv, int cap) {
  for (int g = left < cap ? left : cap; g > 1; --g)
    if (attn_native(dtype, hs, g, dv)) return g;
  return 1;
}
// largest backward branch group per stage (16-bit; fp32 keeps 4).  The 3- / 4-branch
// backward plans at head size >= 64 have no room for the paired two-waves-per-SIMD layout
// (Q rows, K/V tiles and accumulators of 3-4 branches overflow 80 KB of LDS and 256 VGPRs)
// and run one wave per SIMD with spills; groups of <= 2 branches recompute dP = dO V^T once
// per group but run the paired plans.  Measured per kernel (profiles/r04_bwd_groups.json,
// bf16, native -> groups of two): dK/dV hs 64 N = 3 0.464 -> 0.44 ms, hs 96 N = 4 11.6 ->
// 3.4 ms, hs 128 N = 4 8.4 -> 2.9 ms; dQ hs 128 N = 4 4.0 -> 2.0 ms, but dQ at hs 64 / 96
// N = 3 0.40 -> 0.45 / 1.69 -> 1.84 ms and hs 96 N = 4 2.27 -> 2.35 ms, so dQ groups at
// head size 128, and at 64 for N >= 4 (0.487 either way: no re-base needed).  Head size 32
// keeps the native plans for both.  Where the two groupings differ, the delta rows take the
// dK/dV grouping's encoding: written so by attn_dq when one dQ launch holds every branch
// (round 6, BwdParams::kstarts, profiles/r06t_ab_dq_kstarts.json), else re-based after the
// dQ launches (delta_rebase_kernel, ~3-7 us, profiles/r04_bwd_rebase.json).
// DTA_BWD_GROUP_MAX (A/B builds) overrides both caps.
int bwd_group_cap(int dtype, int hs, int n, bool dkdv) {
#ifdef DTA_BWD_GROUP_MAX
  return DTA_BWD_GROUP_MAX;
#else
  if (dtype == DTA_F32) return 4;
  if (hs >= 192) return 1;            // head size 256: the single-branch plans (the N = 2 ones spill)
  if (dkdv) return hs >= 64 ? 2 : 4;
  return (hs >= 128 || (hs >= 64 && hs < 96 && n >= 4)) ? 2 : 4;
#endif
}
// group starts of the backward of an N-branch problem as a bit mask (bit i: a group
// starts at branch i)
uint64_t group_starts(int dtype, int hs, int n, int dv, int cap) {
  uint64_t m = 0;
  for (int g0 = 0, ng; g0 < n; g0 += ng) {
    ng = branch_group(dtype, hs, n - g0, dv, cap);
    m |= 1ull << g0;
  }
  return m;
}
}  // namespace dta

using namespace dta;

namespace {

constexpr float kLog2e = 1.4426950408889634f;

int esize(int dtype) { return dtype == DTA_F32 ? 4 : 2; }

// attention dropout probability -> (keep threshold on a 32-bit hash, 1/(1-p)); p in [0, 1)
bool drop_params(float p, uint64_t seed, uint32_t& thr, float& scale, uint32_t& lo, uint32_t& hi) {
  if (!(p >= 0.f && p < 1.f)) return false;
  const double t = (double)p * 4294967296.0;
  thr = p > 0.f ? (uint32_t)(t < 1.0 ? 1.0 : (t > 4294967295.0 ? 4294967295.0 : t)) : 0u;
  scale = p > 0.f ? (float)(1.0 / (1.0 - (double)p)) : 1.f;
  lo = (uint32_t)seed;
  hi = (uint32_t)(seed >> 32);
  return true;
}

// element alignment every pointer/stride must have: one 16-byte vector
int vec_elems(int dtype) { return 16 / esize(dtype); }

bool aligned_ptr(const void* p) { return p && (reinterpret_cast<uintptr_t>(p) % 16) == 0; }

bool ok_tensor(const dta_tensor& t, int dtype, bool with_i) {
  const int64_t v = vec_elems(dtype);
  if (!aligned_ptr(t.ptr)) return false;
  if (t.sb % v || t.st % v || t.sh % v) return false;
  if (with_i && t.si % v) return false;
  return t.sb >= 0 && t.st >= 0 && t.sh >= 0 && t.si >= 0;
}

T5 t5(const dta_tensor& t) { return T5{t.ptr, t.sb, t.st, t.sh, t.si}; }

// obr (the per-branch O_i): fp32 (obr_dtype 0 or DTA_F32), or fp16 with 16-bit activations
bool ok_obr(const dta_tensor& t, int obr_dtype, int dtype) {
  if (obr_dtype == DTA_F16) return dtype != DTA_F32 && ok_tensor(t, DTA_F16, true);
  return (obr_dtype == 0 || obr_dtype == DTA_F32) && ok_tensor(t, DTA_F32, true);
}

int status(int e) {
  if (e == 0) return DTA_OK;
  if (e == -2) return DTA_ERR_UNSUPPORTED;
  return DTA_ERR_LAUNCH;
}

bool ok_dims(int dtype, int B, int T, int H, int N, int hs, int dv) {
  if (dtype < DTA_BF16 || dtype > DTA_F32) return false;
  return B >= 0 && T >= 0 && H > 0 && N > 0 && hs > 0 && dv > 0;
}

}  // namespace

#ifndef DTA_STAMPS
#define DTA_STAMPS 0
#endif
#if DTA_STAMPS
// diagnostic builds only: one device buffer for the kernels' per-wave stamp sums
static unsigned long long* stamp_buf() {
  static unsigned long long* b = [] {
    void* p = nullptr;
    if (hipMalloc(&p, 64 << 20) || hipMemset(p, 0, 64 << 20)) p = nullptr;
    return (unsigned long long*)p;
  }();
  return b;
}
#else
static unsigned long long* stamp_buf() { return nullptr; }
#endif

extern "C" {

#if DTA_STAMPS
// copy the stamp buffer to the host (diagnostic builds only; not in include/diffattn.h)
int dta_debug_stamps(void* dst, size_t bytes) {
  if (!stamp_buf() || bytes > (64u << 20)) return DTA_ERR_INVALID;
  return hipMemcpy(dst, stamp_buf(), bytes, hipMemcpyDeviceToHost) ? DTA_ERR_LAUNCH : DTA_OK;
}
#endif

int dta_abi_version(void) { return DTA_ABI_VERSION; }

const char* dta_error_string(int code) {
  switch (code) {
    case DTA_OK: return "ok";
    case DTA_ERR_INVALID: return "invalid argument (shape, null/misaligned pointer or stride)";
    case DTA_ERR_UNSUPPORTED: return "unsupported configuration (head_size/n_terms/dtype not built for gfx950)";
    case DTA_ERR_LAUNCH: return "HIP launch failed";
    case DTA_ERR_DROPOUT: return "attention dropout p must lie in [0, 1)";
  }
  return "unknown error";
}

int dta_supported(int32_t dtype, int32_t head_size, int32_t n_terms, int32_t dv) {
  return attn_supported(dtype, head_size, n_terms, dv) ? 1 : 0;
}

int dta_attn_fwd(const dta_attn_fwd_args* a, void* stream) {
  if (!a) return DTA_ERR_INVALID;
  if (!ok_dims(a->dtype, a->B, a->T, a->H, a->n_terms, a->head_size, a->dv)) return DTA_ERR_INVALID;
  FwdParams p{};
  if (!drop_params(a->dropout_p, a->dropout_seed, p.drop_thr, p.drop_scale, p.drop_seed_lo, p.drop_seed_hi))
    return DTA_ERR_DROPOUT;
  if (!attn_supported(a->dtype, a->head_size, a->n_terms, a->dv)) return DTA_ERR_UNSUPPORTED;
  if ((int64_t)a->B * a->T == 0) return DTA_OK;
  if (!ok_tensor(a->q, a->dtype, true) || !ok_tensor(a->k, a->dtype, true) || !ok_tensor(a->v, a->dtype, false) ||
      !ok_tensor(a->o, a->dtype, false) || !ok_obr(a->obr, a->obr_dtype, a->dtype) || !a->lse || !a->coef)
    return DTA_ERR_INVALID;
  p.ob16 = a->obr_dtype == DTA_F16;
  p.q = t5(a->q); p.k = t5(a->k); p.v = t5(a->v); p.o = t5(a->o); p.obr = t5(a->obr);
  p.lse = a->lse; p.coef = a->coef;
  p.B = a->B; p.T = a->T; p.H = a->H; p.N = a->n_terms; p.HS = a->head_size; p.DV = a->dv;
  p.sl2 = a->scale * kLog2e;
  p.cst = a->n_terms;
  if (a->rope_freqs) {
    if (a->head_size % 2 || ((uintptr_t)a->rope_freqs & 15) || !ok_tensor(a->q_rot, a->dtype, true)) return DTA_ERR_INVALID;
    p.rope = a->rope_freqs;
    p.qrot = t5(a->q_rot);
  }
  p.stamps = stamp_buf();
  return status(launch_attn_fwd(a->dtype, p, (hipStream_t)stream));
}

// dK/dV launches (branch groups) a backward of this shape runs at the default caps: more than
// one means dV is summed across groups (in dv_f32 when given)
int dta_attn_bwd_dkdv_groups(int32_t dtype, int32_t head_size, int32_t n_terms, int32_t dv, int32_t group_max_dkdv) {
  // a negative cap is invalid here as in dta_attn_bwd
  if (!attn_supported(dtype, head_size, n_terms, dv) || group_max_dkdv < 0) return 0;
  const int cap = group_max_dkdv > 0 ? group_max_dkdv : bwd_group_cap(dtype, head_size, n_terms, true);
  int n = 0;
  for (int g0 = 0, ng; g0 < n_terms; g0 += ng, ++n) ng = branch_group(dtype, head_size, n_terms - g0, dv, cap);
  return n;
}

size_t dta_attn_bwd_dcoef_partial_bytes(int32_t B, int32_t T, int32_t H, int32_t n_terms) {
  return (size_t)H * n_terms * B * ((T + 31) / 32) * 4;
}

size_t dta_attn_bwd_workspace_bytes(int32_t B, int32_t T, int32_t H, int32_t n_terms, int32_t head_size) {
  const size_t delta = (size_t)n_terms * B * H * T * 4;
  const size_t dq = (size_t)B * T * H * n_terms * head_size * 4;
  return delta + dq;
}

int dta_attn_bwd(const dta_attn_bwd_args* a, void* stream) {
  if (!a) return DTA_ERR_INVALID;
  if (!ok_dims(a->dtype, a->B, a->T, a->H, a->n_terms, a->head_size, a->dv)) return DTA_ERR_INVALID;
  BwdParams p{};
  if (!drop_params(a->dropout_p, a->dropout_seed, p.drop_thr, p.drop_scale, p.drop_seed_lo, p.drop_seed_hi))
    return DTA_ERR_DROPOUT;
  if (!attn_supported(a->dtype, a->head_size, a->n_terms, a->dv)) return DTA_ERR_UNSUPPORTED;
  if (!a->dcoef) return DTA_ERR_INVALID;
  hipStream_t st = (hipStream_t)stream;
  const int stages = a->stages ? a->stages : (DTA_BWD_PRE | DTA_BWD_DQ | DTA_BWD_DKDV);
  // (with dcoef_partial the DQ stage's ordered reduce overwrites every dcoef entry: nothing to zero)
  if ((stages & DTA_BWD_PRE) && !a->dcoef_partial) {
    if (hipMemsetAsync(a->dcoef, 0, sizeof(float) * a->H * a->n_terms, st)) return DTA_ERR_LAUNCH;
  }
  if ((int64_t)a->B * a->T == 0) return DTA_OK;
  if (!ok_tensor(a->q, a->dtype, true) || !ok_tensor(a->k, a->dtype, true) || !ok_tensor(a->v, a->dtype, false) ||
      !ok_obr(a->obr, a->obr_dtype, a->dtype) || !ok_tensor(a->dout, a->dtype, false) ||
      !ok_tensor(a->dk, a->dtype, true) || !ok_tensor(a->dv_out, a->dtype, false) ||
      !a->lse || !a->coef || !a->delta)
    return DTA_ERR_INVALID;
  if (a->dq.ptr ? !ok_tensor(a->dq, a->dtype, true) : !aligned_ptr(a->dq_f32)) return DTA_ERR_INVALID;
  p.q = t5(a->q); p.k = t5(a->k); p.v = t5(a->v); p.obr = t5(a->obr); p.dout = t5(a->dout);
  p.ob16 = a->obr_dtype == DTA_F16;
  p.dq = t5(a->dq); p.dk = t5(a->dk); p.dv = t5(a->dv_out);
  p.lse = a->lse; p.delta = a->delta; p.coef = a->coef; p.dcoef = a->dcoef;
  p.dq32 = a->dq.ptr ? nullptr : a->dq_f32;
  if (a->rope_freqs && (a->head_size % 4 || reinterpret_cast<uintptr_t>(a->rope_freqs) % 16)) return DTA_ERR_INVALID;
  p.rope = a->rope_freqs;
  if (a->dcoef_partial && !aligned_ptr(a->dcoef_partial)) return DTA_ERR_INVALID;
  if (a->dv_f32 && !aligned_ptr(a->dv_f32)) return DTA_ERR_INVALID;
  if (a->lse_c && !aligned_ptr(a->lse_c)) return DTA_ERR_INVALID;
  // |c_i| folded into the key-major kernel's probabilities: 16-bit plans without dropout
  p.lsec = (a->lse_c && a->dtype != DTA_F32 && !p.drop_thr) ? a->lse_c : nullptr;
  p.dcoef_part = a->dcoef_partial;
  p.B = a->B; p.T = a->T; p.H = a->H; p.N = a->n_terms; p.HS = a->head_size; p.DV = a->dv;
  p.scale = a->scale; p.sl2 = a->scale * kLog2e;
  p.cst = a->n_terms; p.br0 = 0; p.dv_acc = 0;
  p.stamps = stamp_buf();
  // branch groups [g0, g0 + ng): a native N runs as one group; otherwise each group's
  // branch-indexed operands are offset to its first branch (coef / dcoef rows keep the
  // stride cst = N), so the kernels see an ng-branch problem
  const int es = esize(a->dtype);
  const int64_t rowvec = (int64_t)p.B * p.H * p.T, nblk = (p.T + 31) / 32;
  auto group = [&](int g0, int ng) {
    BwdParams q = p;
    auto off = [&](T5& t) { t.p = (char*)t.p + (int64_t)g0 * t.si * es; };
    off(q.q); off(q.k); off(q.dk);
    q.obr.p = (char*)q.obr.p + (int64_t)g0 * q.obr.si * (p.ob16 ? 2 : 4);
    if (q.dq.p) off(q.dq);
    if (q.dq32) q.dq32 += (int64_t)g0 * p.HS;
    q.lse += g0 * rowvec; q.delta += g0 * rowvec; q.coef += g0; q.dcoef += g0;
    if (q.lsec) q.lsec += g0 * rowvec;
    if (q.dcoef_part) q.dcoef_part += g0 * (int64_t)p.B * nblk;
    q.N = ng; q.br0 = g0; q.dv_acc = g0 > 0; q.dv_last = g0 + ng == p.N;
    return q;
  };
  int e = 0;
  // the dK/dV grouping must see delta rows encoded for its own groups (see bwd_group_cap)
  if (a->group_max_dq < 0 || a->group_max_dkdv < 0) return DTA_ERR_INVALID;
  const int kcap = a->group_max_dkdv ? a->group_max_dkdv : bwd_group_cap(a->dtype, p.HS, p.N, true);
  int qcap = a->group_max_dq ? a->group_max_dq : bwd_group_cap(a->dtype, p.HS, p.N, false);
  // beyond 64 branches the group-start masks do not fit: both stages take the dK/dV grouping
  if (p.N > 64) qcap = kcap;
  // with dropout the delta rows hold delta_i itself (no group encoding): nothing to re-base
  const bool rebase = qcap != kcap && !p.drop_thr;
  const uint64_t qstarts = rebase ? group_starts(a->dtype, p.HS, p.N, p.DV, qcap) : 0;
  const uint64_t kstarts = rebase ? group_starts(a->dtype, p.HS, p.N, p.DV, kcap) : 0;
  if (stages & DTA_BWD_DQ) {
    // one dQ launch over every branch writes the delta rows straight in the dK/dV encoding
    const bool direct = DTA_DQ_KSTARTS && qstarts != kstarts && branch_group(a->dtype, p.HS, p.N, p.DV, qcap) == p.N;
    for (int g0 = 0, ng; g0 < p.N; g0 += ng) {
      ng = branch_group(a->dtype, p.HS, p.N - g0, p.DV, qcap);
      BwdParams q = group(g0, ng);
      q.kstarts = direct ? kstarts : 0;
      if ((e = launch_attn_dq(a->dtype, q, st))) return status(e);
    }
    if (p.dcoef_part &&
        (e = launch_dcoef_reduce(p.dcoef_part, p.dcoef, p.H, p.N, (int64_t)p.B * nblk, st)))
      return status(e);
    if (!direct && qstarts != kstarts && (e = launch_delta_rebase(p.delta, rowvec, p.N, qstarts, kstarts, st)))
      return status(e);
  }
  if (stages & DTA_BWD_DKDV) {
    // more than one dK/dV group: dV is summed in the fp32 workspace when the caller gave one
    const bool multi = branch_group(a->dtype, p.HS, p.N, p.DV, kcap) < p.N;
    for (int g0 = 0, ng; g0 < p.N; g0 += ng) {
      ng = branch_group(a->dtype, p.HS, p.N - g0, p.DV, kcap);
      BwdParams q = group(g0, ng);
      q.dv32 = multi ? a->dv_f32 : nullptr;
      if ((e = launch_attn_dkdv(a->dtype, q, st))) return status(e);
    }
  }
  return DTA_OK;
}

static int ln_common(const dta_ln_args* a, bool bwd) {
  if (!a || a->dtype < DTA_BF16 || a->dtype > DTA_F32 || a->rows < 0 || a->C <= 0) return DTA_ERR_INVALID;
  if (a->io_dtype != 0 && (a->dtype != DTA_F32 || (a->io_dtype - 1 != DTA_BF16 && a->io_dtype - 1 != DTA_F16)))
    return DTA_ERR_UNSUPPORTED;
  const int64_t v = 8;   // kernels move 8 elements per lane access
  if (a->C % v || a->C > 8192) return DTA_ERR_UNSUPPORTED;
  if (!aligned_ptr(a->x) || a->x_stride % v || !a->w || !a->mean || !a->rstd) return DTA_ERR_INVALID;
  if (!bwd && (!aligned_ptr(a->y) || a->y_stride % v || !a->b)) return DTA_ERR_INVALID;
  if (bwd && (!aligned_ptr(a->dy) || !aligned_ptr(a->dx) || a->dy_stride % v || a->dx_stride % v || !a->dw || !a->db))
    return DTA_ERR_INVALID;
  // residual fusion: the mixed fp32 / 16-bit path only, with aligned 8-element rows
  const bool fused = bwd ? (a->dres || a->dx16) : (a->res || a->xo);
  if (fused && a->io_dtype == 0) return DTA_ERR_UNSUPPORTED;
  if (!bwd && fused && (!aligned_ptr(a->res) || !aligned_ptr(a->xo) || a->res_stride % v || a->xo_stride % v))
    return DTA_ERR_INVALID;
  if (bwd && a->partial && !aligned_ptr(a->partial)) return DTA_ERR_INVALID;   // 16-byte partial rows
  if (bwd && a->dres && (!aligned_ptr(a->dres) || a->dres_stride % v)) return DTA_ERR_INVALID;
  if (bwd && a->dx16 && (!aligned_ptr(a->dx16) || a->dx16_stride % v)) return DTA_ERR_INVALID;
  return DTA_OK;
}

static LnParams ln_params(const dta_ln_args* a) {
  LnParams p{};
  p.rows = a->rows; p.C = a->C; p.eps = a->eps; p.out_scale = a->out_scale;
  p.x = a->x; p.xs = a->x_stride; p.y = a->y; p.ys = a->y_stride;
  p.w = a->w; p.b = a->b; p.mean = a->mean; p.rstd = a->rstd;
  p.dy = a->dy; p.dys = a->dy_stride; p.dx = a->dx; p.dxs = a->dx_stride;
  p.dw = a->dw; p.db = a->db;
  p.partial = a->partial;
  p.res = a->res; p.ress = a->res_stride; p.xo = a->xo; p.xos = a->xo_stride;
  p.dres = a->dres; p.dress = a->dres_stride; p.dx16 = a->dx16; p.dx16s = a->dx16_stride;
  return p;
}

int dta_ln_fwd(const dta_ln_args* a, void* stream) {
  if (int e = ln_common(a, false)) return e;
  if (a->io_dtype) return status(launch_ln_mixed(a->io_dtype - 1, ln_params(a), false, (hipStream_t)stream));
  return status(launch_ln(a->dtype, ln_params(a), false, (hipStream_t)stream));
}

size_t dta_ln_bwd_workspace_bytes(int64_t rows, int64_t C) { return (size_t)ln_bwd_workspace_floats(rows, C) * 4; }

int dta_ln_bwd(const dta_ln_args* a, void* stream) {
  if (int e = ln_common(a, true)) return e;
  if (a->io_dtype) return status(launch_ln_mixed(a->io_dtype - 1, ln_params(a), true, (hipStream_t)stream));
  return status(launch_ln(a->dtype, ln_params(a), true, (hipStream_t)stream));
}

int dta_rope(const dta_rope_args* a, void* stream) {
  if (!a || !ok_dims(a->dtype, a->B, a->T, a->H, a->n_terms, a->head_size, 1)) return DTA_ERR_INVALID;
  if (a->head_size % 8) return DTA_ERR_UNSUPPORTED;
  if ((int64_t)a->B * a->T == 0) return DTA_OK;
  const int src_dtype = a->src_f32 ? DTA_F32 : a->dtype;
  // the kernel reads the freqs table by 16-byte vectors (as the attention entry points require)
  if (!ok_tensor(a->src, src_dtype, true) || !ok_tensor(a->dst, a->dtype, true) || !aligned_ptr(a->freqs))
    return DTA_ERR_INVALID;
  RopeParams p{};
  p.src = t5(a->src); p.dst = t5(a->dst); p.freqs = a->freqs;
  p.B = a->B; p.T = a->T; p.H = a->H; p.N = a->n_terms; p.HS = a->head_size; p.inverse = a->inverse ? 1 : 0;
  return status(launch_rope(a->dtype, a->src_f32 != 0, p, (hipStream_t)stream));
}

static int swiglu_common(const dta_swiglu_args* a, bool bwd, SwigluParams& p) {
  if (!a || a->dtype < DTA_BF16 || a->dtype > DTA_F32 || a->rows < 0 || a->n < 0) return DTA_ERR_INVALID;
  if (a->n % 8) return DTA_ERR_UNSUPPORTED;
  auto ok = [](const void* q, int64_t st) { return aligned_ptr(q) && st % 8 == 0 && st >= 0; };
  if (!ok(a->a, a->a_stride) || !ok(a->b, a->b_stride)) return DTA_ERR_INVALID;
  if (!bwd && !ok(a->out, a->out_stride)) return DTA_ERR_INVALID;
  if (bwd && (!ok(a->dout, a->dout_stride) || !ok(a->da, a->da_stride) || !ok(a->db, a->db_stride)))
    return DTA_ERR_INVALID;
  p = SwigluParams{a->rows, a->n, a->a, a->a_stride, a->b, a->b_stride, a->out, a->out_stride,
                   a->dout, a->dout_stride, a->da, a->da_stride, a->db, a->db_stride};
  return DTA_OK;
}

int dta_swiglu_fwd(const dta_swiglu_args* a, void* stream) {
  SwigluParams p;
  if (int e = swiglu_common(a, false, p)) return e;
  return status(launch_swiglu(a->dtype, p, false, (hipStream_t)stream));
}

int dta_swiglu_bwd(const dta_swiglu_args* a, void* stream) {
  SwigluParams p;
  if (int e = swiglu_common(a, true, p)) return e;
  if (a->dbias) {
    if (!aligned_ptr(a->dbias) || !aligned_ptr(a->dbias_work)) return DTA_ERR_INVALID;
    if (a->rows == 0 || a->n == 0) return status(hipMemsetAsync(a->dbias, 0, sizeof(float) * 2 * a->n, (hipStream_t)stream));
    return status(launch_swiglu_bias(a->dtype, p, a->dbias, a->dbias_work, (hipStream_t)stream));
  }
  return status(launch_swiglu(a->dtype, p, true, (hipStream_t)stream));
}

size_t dta_swiglu_bwd_workspace_bytes(int64_t rows, int64_t n) {
  return rows < 0 || n < 0 ? 0 : (size_t)swiglu_bias_work_floats(rows, n) * 4;
}

int dta_accumulate_f32(int32_t dtype, int64_t n, const void* src, float* dst, void* stream) {
  if (dtype < DTA_BF16 || dtype > DTA_F32 || n < 0) return DTA_ERR_INVALID;
  if (n == 0) return DTA_OK;
  if (!aligned_ptr(src) || !aligned_ptr(dst)) return DTA_ERR_INVALID;
  return status(launch_accumulate(dtype, n, src, dst, (hipStream_t)stream));
}

int dta_cast_f32(int32_t dtype, int32_t B, int32_t T, int32_t H, int32_t n_terms, int32_t head_size,
                 const float* src, dta_tensor dst, void* stream) {
  if (!ok_dims(dtype, B, T, H, n_terms, head_size, 1) || head_size % 8) return DTA_ERR_INVALID;
  if ((int64_t)B * T == 0) return DTA_OK;
  if (!aligned_ptr(src) || !ok_tensor(dst, dtype, true)) return DTA_ERR_INVALID;
  return status(launch_cast(dtype, src, t5(dst), B, T, H, n_terms, head_size, (hipStream_t)stream));
}

static int64_t decode_splits(int32_t t_cap) { return (t_cap + DTA_DECODE_CHUNK - 1) / DTA_DECODE_CHUNK; }

size_t dta_attn_decode_workspace_bytes(int32_t B, int32_t H, int32_t n_terms, int32_t head_size, int32_t dv,
                                       int32_t t_cap) {
  const size_t single = (size_t)B * H * n_terms * t_cap * 4;
  const size_t split = (size_t)B * H * decode_splits(t_cap) * n_terms * (dv + 2) * 4;
  return single > split ? single : split;
}

int dta_attn_decode(const dta_attn_decode_args* a, void* stream) {
  if (!a || !ok_dims(a->dtype, a->B, 1, a->H, a->n_terms, a->head_size, a->dv)) return DTA_ERR_INVALID;
  if (a->head_size % 8 || a->head_size > 128 || a->n_terms > 4 || a->dv > 256) return DTA_ERR_UNSUPPORTED;
  if (a->length < 1 || a->t_cap < a->length) return DTA_ERR_INVALID;
  if ((int64_t)a->B * a->H == 0) return DTA_OK;
  // every operand is read or written by 16-byte vector accesses: full alignment checks on all four
  if (!ok_tensor(a->q, a->dtype, true) || !ok_tensor(a->k_cache, a->dtype, true) ||
      !ok_tensor(a->v_cache, a->dtype, false) || !ok_tensor(a->o, a->dtype, false) || !a->coef ||
      !aligned_ptr(a->workspace))
    return DTA_ERR_INVALID;
  DecodeParams p{};
  p.q = t5(a->q); p.k = t5(a->k_cache); p.v = t5(a->v_cache); p.o = t5(a->o);
  p.coef = a->coef; p.ws = a->workspace;
  p.B = a->B; p.H = a->H; p.N = a->n_terms; p.HS = a->head_size; p.DV = a->dv;
  p.L = a->length; p.ldw = a->t_cap; p.scale = a->scale; p.Ldev = a->length_dev;
  p.S = (int)decode_splits(a->length);
  p.ml = a->workspace + (int64_t)a->B * a->H * p.S * a->n_terms * a->dv;   // after the partial rows
  return status(launch_decode(a->dtype, p, (hipStream_t)stream));
}

}  // extern "C"
