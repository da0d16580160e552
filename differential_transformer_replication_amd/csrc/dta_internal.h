// dta_internal.h -- host-side parameter blocks shared between the C-ABI
// (dta_capi.cpp) and the per-dtype kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DTA_DQ_KSTARTS
#define DTA_DQ_KSTARTS 1   // attn_dq writes the delta rows in the dK/dV grouping's encoding when it holds every branch (no rebase launch)
#endif

namespace dta {

struct T5 {            // [b][t][h][i] element strides + base pointer
  void* p;
  int64_t sb, st, sh, si;
};

struct FwdParams {
  T5 q, k, v, o, obr;
  float* lse;
  const float* coef;
  int B, T, H, N, HS, DV;
  float sl2;           // scale * log2(e)
  unsigned long long* stamps;   // diagnostic builds (DTA_STAMPS) only: per-wave segment cycle sums
  uint32_t drop_thr;   // attention dropout: keep iff hash >= drop_thr (= p * 2^32); 0 = off
  float drop_scale;    // 1 / (1 - p)
  uint32_t drop_seed_lo, drop_seed_hi;
  int bsplit;          // launcher-internal: > 1 = branch-split launch of the N = 1 kernel
                       // (one branch of bsplit per workgroup; writes O_i and LSE_i only)
  int bseq;            // launcher-internal: > 1 = the N = 1 kernel runs bseq branches one after
                       // another per workgroup and writes O as well (no combine pass)
  int cst;             // row stride of coef [h][cst] (the call's total branch count)
  const float* rope;   // if set (ABI 5): q is un-rotated; the forward rotates Q_i at load
  T5 qrot;             //   (fp32 [T][HS/2][2] table) and stores the rotated rows here
  int ob16;            // O_i (obr) stored as fp16 instead of fp32 (ABI 6, 16-bit activations)
};

struct BwdParams {
  T5 q, k, v, obr, dout, dq, dk, dv;
  const float* lse;
  float* delta;        // written by attn_dq, read by attn_dkdv
  const float* coef;
  float* dcoef;        // accumulated by attn_dq (zeroed first)
  float* dq32;         // if set: dQ written as fp32 [b][t][h][i][d] instead of into dq
  const float* rope;   // if set: fp32 [T][HS/2][2] table; dQ / dK leave through the inverse rotation
  float* dcoef_part;   // if set: per-wave d(coef) partials [h][i][b][T/32] (no atomics), summed by dcoef_reduce
  int B, T, H, N, HS, DV;
  float sl2, scale;
  unsigned long long* stamps;   // as FwdParams::stamps
  uint32_t drop_thr;   // as FwdParams
  float drop_scale;
  uint32_t drop_seed_lo, drop_seed_hi;
  // branch groups (capi: a call whose N has no kernel plan runs as groups of branches
  // that have one; every branch-indexed pointer above is then offset to the group's
  // first branch br0):
  int cst;             // the call's total branch count: row stride of coef / dcoef
                       // [h][cst], of the d(coef) partials and of dq32; dropout's branch index
  int br0;             // the group's first branch (dropout mask key)
  int dv_acc;          // dK/dV kernel: add into dv instead of storing (groups after the first)
  float* dv32;         // optional fp32 [b][t][h][e] running dV sum across branch groups
  int dv_last;         // the last dK/dV group (with dv32: the one that writes dv)
  int ob16;            // obr holds fp16 O_i (ABI 6)
  float* lsec;         // optional (ABI 8 lse_c, 16-bit, no dropout): stored LSE_i + log2|c_i| rows
                       // [i][b][h][t], written by attn_dq, the S seeds of attn_dkdv (|c_i| folded into P)
  uint64_t kstarts;    // attn_dq run as one group, no dropout: the dK/dV grouping's starts (bit i), so the
                       // delta rows are written in that encoding and no rebase launch follows (0: own group)
};

// per-dtype launchers (dtype index: 0 bf16, 1 f16, 2 f32); return hipError_t
int launch_attn_fwd(int dtype, const FwdParams& p, hipStream_t st);
// dropout instantiations (attn_*_drop.hip): the same kernels with the mask compiled in
int launch_attn_fwd_drop(int dtype, const FwdParams& p, hipStream_t st);
int launch_attn_dq_drop(int dtype, const BwdParams& p, hipStream_t st);
int launch_attn_dkdv_drop(int dtype, const BwdParams& p, hipStream_t st);
int launch_attn_dq(int dtype, const BwdParams& p, hipStream_t st);
int launch_attn_dkdv(int dtype, const BwdParams& p, hipStream_t st);
bool attn_supported(int dtype, int hs, int n, int dv);   // any kernel path: native plan or branch groups
bool attn_native(int dtype, int hs, int n, int dv);      // an N-branch kernel plan is built

struct LnParams {
  int64_t rows, C;
  float eps, out_scale;
  const void* x; int64_t xs;
  void* y; int64_t ys;
  const float* w; const float* b;
  float* mean; float* rstd;
  const void* dy; int64_t dys;
  void* dx; int64_t dxs;
  float* dw; float* db;
  float* partial;      // optional [blocks][2][C] workspace: deterministic dw/db (no atomics)
  // residual fusion (mixed fp32 x / 16-bit y path only; NULL = off):
  const void* res; int64_t ress;   // fwd: x + res (res in y's dtype) is normalised ...
  float* xo; int64_t xos;          // ... and written here (fp32)
  const float* dres; int64_t dress;  // bwd: dx += dres (the residual branch's gradient)
  void* dx16; int64_t dx16s;       // bwd: dx also stored in y's dtype
};
int launch_ln_mixed(int y_dtype, const LnParams& p, bool bwd, hipStream_t st);   // x fp32, y / dy 16-bit
int ln_bwd_blocks(int64_t rows);
int64_t ln_bwd_workspace_floats(int64_t rows, int64_t C);

struct RopeParams {
  T5 src, dst;
  const float* freqs;
  int B, T, H, N, HS;
  int inverse;
};

#ifndef DTA_DECODE_CHUNK
#define DTA_DECODE_CHUNK 256   // keys per workgroup of the split-key decode plan
#endif

struct DecodeParams {
  T5 q, k, v, o;       // q/o: one row per (b, h) (st unused); k/v: the cache [b][t][h][i]
  const float* coef;   // [h][i]
  float* ws;           // single pass: fp32 [b][h][i][ldw]; split: partial rows [b][h][s][i][DV]
  float* ml;           // split path: fp32 [b][h][s][i][2] chunk (max, sum); null = single pass
  int B, H, N, HS, DV, L, ldw, S;   // L: length, or its upper bound when Ldev is set
  float scale;
  const int* Ldev;     // optional device length
};

int launch_decode(int dtype, const DecodeParams& p, hipStream_t st);
int launch_ln(int dtype, const LnParams& p, bool bwd, hipStream_t st);
int launch_rope(int dtype, bool src_f32, const RopeParams& p, hipStream_t st);
int launch_dcoef_reduce(const float* part, float* dcoef, int H, int N, int64_t per, hipStream_t st);
int launch_delta_rebase(float* delta, int64_t rows, int N, uint64_t from, uint64_t to, hipStream_t st);
int launch_cast(int dtype, const float* src, const T5& dst, int B, int T, int H, int N, int HS, hipStream_t st);

struct SwigluParams {
  int64_t rows, n;                       // rows x n elements, n % 8 == 0
  const void* a; int64_t as;             // gate pre-activation (row stride, elements)
  const void* b; int64_t bs;             // linear branch
  void* out; int64_t os;                 // forward output
  const void* dout; int64_t dos;         // backward: incoming gradient
  void* da; int64_t das;
  void* db; int64_t dbs;
};
int launch_swiglu(int dtype, const SwigluParams& p, bool bwd, hipStream_t st);
int launch_accumulate(int dtype, int64_t n, const void* src, float* dst, hipStream_t st);
int launch_swiglu_bias(int dtype, const SwigluParams& p, float* dbias, float* work, hipStream_t st);
int64_t swiglu_bias_work_floats(int64_t rows, int64_t n);

}  // namespace dta
