// elementwise.hip -- HBM-bound kernels around the attention core, gfx950.
//
//  * ln_fwd / ln_bwd   GroupLayerNorm over the concatenated heads (C' = H*dv)
//                      fused with the constant x(1 - 0.8) output scale
//                      (diff_transformer.py:15-20, 90-91).  One wave per row,
//                      16-byte vector loads, two-pass mean/variance in registers.
//  * rope              interleaved-pair rotary embedding of every Q_i / K_i and
//                      its inverse for the gradients (Ndiff_transformer.py:11-22).
//  * dcoef_reduce      dcoef[h][i] = sum of the dQ kernel's per-block partials of
//                      delta_i = <dO, O_i>  (d lambda, SURVEY semantic 5), fixed order.
//  * cast_f32          fp32 dQ accumulator -> activation dtype.
//  * swiglu / accumulate / swiglu_bias   the training step's fused elementwise passes.
// Every output is written once with non-temporal stores (DTA_EW_NT).
#include <type_traits>

#include "dta_common.h"
#include "dta_internal.h"

namespace dta {

template <class E> struct Vec8;
template <> struct Vec8<__bf16> { typedef bf16x8 t; };
template <> struct Vec8<_Float16> { typedef f16x8 t; };

// streaming policy of the row-wise kernels' activations (read once, written once):
// bit 0 = non-temporal loads, bit 1 = non-temporal stores.  One-process A/B at cfg2's
// GroupLayerNorm and cfg3's RoPE (profiles/r04_ab_ln_nt.json): nt stores 45.6 -> 41.7 us
// (ln_fwd, 6.44 TB/s), 90.3 -> 76.6 (ln_bwd), 51.3 -> 42.2 (rope, 7.15 TB/s); nt loads
// slower (52.6 us ln_fwd) with or without them.  Outputs bitwise equal.
#ifndef DTA_EW_NT
#define DTA_EW_NT 2
#endif
template <class V>
__device__ __forceinline__ V ldv(const V* p) {
  if constexpr (DTA_EW_NT & 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <class V>
__device__ __forceinline__ void stv(V* p, V v) {
  if constexpr (DTA_EW_NT & 2) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// load/store 8 consecutive elements as fp32
template <class E>
__device__ __forceinline__ void ld8(const E* p, float* f) {
  if constexpr (sizeof(E) == 2) {
    typename Vec8<E>::t v = ldv(reinterpret_cast<const typename Vec8<E>::t*>(p));
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
  } else {
    f32x4 a = ldv(reinterpret_cast<const f32x4*>(p)), b = ldv(reinterpret_cast<const f32x4*>(p + 4));
#pragma unroll
    for (int j = 0; j < 4; ++j) { f[j] = a[j]; f[j + 4] = b[j]; }
  }
}
template <class E>
__device__ __forceinline__ void st8(E* p, const float* f) {
  if constexpr (sizeof(E) == 2) {
    typename Vec8<E>::t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (E)f[j];
    stv(reinterpret_cast<typename Vec8<E>::t*>(p), v);
  } else {
    stv(reinterpret_cast<f32x4*>(p), f32x4{f[0], f[1], f[2], f[3]});
    stv(reinterpret_cast<f32x4*>(p + 4), f32x4{f[4], f[5], f[6], f[7]});
  }
}

// Sum over the 64 lanes, every lane gets the total: four DPP steps inside each 16-lane
// row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then
// v_permlane16_swap and v_permlane32_swap across rows -- all VALU, where __shfl_xor took
// six ds_bpermute round trips through the LDS, each behind an lgkmcnt(0) wait.
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_sum(float v) {
  v = dpp_add<0xB1>(v);      // quad_perm [1,0,3,2]
  v = dpp_add<0x4E>(v);      // quad_perm [2,3,0,1]
  v = dpp_add<0x141>(v);     // row_half_mirror
  v = dpp_add<0x140>(v);     // row_mirror
  const unsigned u = __float_as_uint(v);
  auto r16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
  const unsigned w = __float_as_uint(v);
  auto r32 = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}


// CH = 8-element chunks per lane (C <= 512*CH)
template <class E, int CH, class Y = E>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const E* x = reinterpret_cast<const E*>(p.x) + row * p.xs;
  float v[CH][8];
  float s = 0.f;
  // residual fusion (fp32 x, 16-bit y): v = x + res, stored to xo, then normalised
  constexpr bool MIXED = std::is_same<E, float>::value && sizeof(Y) == 2;
  const bool fuse = MIXED && p.res != nullptr;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < p.C) {
      ld8<E>(x + col, v[c]);
      if constexpr (MIXED) {
        if (fuse) {
          float r[8];
          ld8<Y>(reinterpret_cast<const Y*>(p.res) + row * p.ress + col, r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] += r[j];
          st8<float>(p.xo + row * p.xos + col, v[c]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    }
  }
  const float inv_c = 1.f / (float)p.C;
  const float mean = wave_sum(s) * inv_c;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < p.C) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[c][j] - mean; ss += d * d; }
    }
  }
  const float var = wave_sum(ss) * inv_c;
  const float rstd = 1.f / sqrtf(var + p.eps);
  if (lane == 0) { p.mean[row] = mean; p.rstd[row] = rstd; }
  Y* y = reinterpret_cast<Y*>(p.y) + row * p.ys;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < p.C) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = fmaf((v[c][j] - mean) * rstd, p.w[col + j], p.b[col + j]) * p.out_scale;
      st8<Y>(y + col, o);
    }
  }
}

// Backward: dx per row plus per-column dw/db partial sums.  Each wave walks rows with
// a stride, the NEXT row's x / dy loads issued before the current row's math (two rows
// in flight per wave); the block's four waves combine their column partials in LDS.
// Partials go either to p.partial ([block][2][C], plain stores; ln_bwd_reduce then
// sums them in a fixed order -- bitwise reproducible) or, without a workspace,
// straight to dw/db by atomics.
template <class E> struct Raw8 { typedef s16x8 t; };
template <> struct Raw8<float> { typedef f32x4 t[2]; };

template <class E>
__device__ __forceinline__ void raw_ld(const E* p, s16x8& v) { v = ldv(reinterpret_cast<const s16x8*>(p)); }
template <class E>
__device__ __forceinline__ void raw_cvt(const s16x8& v, float* f) {
  const typename Vec8<E>::t w = __builtin_bit_cast(typename Vec8<E>::t, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (float)w[j];
}

template <class E, int CH>
__global__ __launch_bounds__(256) void ln_bwd_kernel(LnParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float dwp[CH][8], dbp[CH][8], wv[CH][8];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dwp[c][j] = 0.f; dbp[c][j] = 0.f;
      wv[c][j] = col < p.C ? p.w[col + j] * p.out_scale : 0.f;
    }
  }
  const float inv_c = 1.f / (float)p.C;
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t row = (int64_t)blockIdx.x * 4 + wave;
  // 16-bit rows stay packed in registers until used; fp32 rows are loaded as floats
  constexpr bool P16 = sizeof(E) == 2;
  s16x8 xr[P16 ? CH : 1], dr[P16 ? CH : 1];
  auto load = [&](int64_t r) {
    if constexpr (P16) {
      const E* x = reinterpret_cast<const E*>(p.x) + r * p.xs;
      const E* dy = reinterpret_cast<const E*>(p.dy) + r * p.dys;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int col = (c * 64 + lane) * 8;
        if (col < p.C) { raw_ld<E>(x + col, xr[c]); raw_ld<E>(dy + col, dr[c]); }
      }
    }
  };
  if (row < p.rows) load(row);
  for (; row < p.rows; row += stride) {
    float xv[CH][8], dv[CH][8];
    if constexpr (P16) {
#pragma unroll
      for (int c = 0; c < CH; ++c) { raw_cvt<E>(xr[c], xv[c]); raw_cvt<E>(dr[c], dv[c]); }
      if (row + stride < p.rows) load(row + stride);          // next row in flight during this row's math
    } else {
      const E* x = reinterpret_cast<const E*>(p.x) + row * p.xs;
      const E* dy = reinterpret_cast<const E*>(p.dy) + row * p.dys;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int col = (c * 64 + lane) * 8;
        if (col < p.C) { ld8<E>(x + col, xv[c]); ld8<E>(dy + col, dv[c]); }
      }
    }
    const float mean = p.mean[row], rstd = p.rstd[row];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < p.C) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (xv[c][j] - mean) * rstd;
          const float dys = dv[c][j] * p.out_scale;
          dwp[c][j] = fmaf(dys, xh, dwp[c][j]);
          dbp[c][j] += dys;
          const float g = dv[c][j] * wv[c][j];
          xv[c][j] = xh;
          dv[c][j] = g;
          sg += g;
          sgx = fmaf(g, xh, sgx);
        }
      }
    }
    const float mg = wave_sum(sg) * inv_c, mgx = wave_sum(sgx) * inv_c;
    E* dx = reinterpret_cast<E*>(p.dx) + row * p.dxs;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < p.C) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (dv[c][j] - mg - xv[c][j] * mgx);
        st8<E>(dx + col, o);
      }
    }
  }
  // column partials: reduce the 4 waves through LDS, then one value per column per block
  __shared__ float red[2][4][512];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][wave][(lane * 8 + j)] = dwp[c][j];
      red[1][wave][(lane * 8 + j)] = dbp[c][j];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 1024; e += 256) {
      const int which = e >> 9, k = e & 511;
      const int col = c * 512 + k;
      if (col < p.C) {
        const float sum = red[which][0][k] + red[which][1][k] + red[which][2][k] + red[which][3][k];
        if (p.partial) p.partial[((int64_t)blockIdx.x * 2 + which) * p.C + col] = sum;
        else atomicAdd((which ? p.db : p.dw) + col, sum);
      }
    }
  }
}

// Backward, one workgroup per row at a time (DTA_LN_BWD_ROWBLOCK, default): the four
// waves split the row's columns (thread t owns 8-column chunks t, t+256, ...), so a
// thread's dw/db column partials are only 16*CHB registers and need no cross-wave
// reduction; the row sums (sum g, sum g*xhat) cross waves through a parity-double-
// buffered LDS slot, one barrier per row.  The x / dy of the rows PD groups ahead are
// loaded before the current row's math (a register ring of PD + 1 rows): with 512
// workgroups (2 per CU, capped so the column partials stay small) one row ahead left
// ~16 KB in flight per CU; three rows ahead took cfg2's ln_bwd 72.6 -> 68.5 us
// (profiles/r06o_ab_ln_prefetch_depth.json).  ~114 VGPRs at C = 2048, where the
// wave-per-row kernel above holds 222.
#ifndef DTA_LN_BWD_RPI
#define DTA_LN_BWD_RPI 1         // rows per barrier (each workgroup step)
#endif
#ifndef DTA_LN_BWD_PD
#define DTA_LN_BWD_PD 3          // row groups in flight ahead of the one being computed (1..5)
#endif
// (rows wider than 2048 columns keep one row ahead: they already hold CHB times the bytes in
// flight per row, and three rows of them cost 206-512 registers, a wave per SIMD or spills)
template <class E, int CHB, class Y = E, int RPI = DTA_LN_BWD_RPI, int PD = (CHB == 1 ? DTA_LN_BWD_PD : 1)>
__global__ __launch_bounds__(256) void ln_bwd_rb_kernel(LnParams p) {
  static_assert(PD >= 1 && PD <= 5, "prefetch depth");
  constexpr int NSL = PD + 1;      // register slots of raw rows
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  float dwp[CHB][8], dbp[CHB][8];
#pragma unroll
  for (int c = 0; c < CHB; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) { dwp[c][j] = 0.f; dbp[c][j] = 0.f; }
  const float inv_c = 1.f / (float)p.C;
  __shared__ float red[2][RPI][4][2];
  // raw (unconverted) vectors of 8 elements: one s16x8 for 16-bit, two f32x4 for fp32
  constexpr bool P16 = sizeof(E) == 2, Y16 = sizeof(Y) == 2;
  typedef typename std::conditional<P16, s16x8, f32x4>::type RT;
  typedef typename std::conditional<Y16, s16x8, f32x4>::type RY;
  constexpr int NR = P16 ? 1 : 2, NY = Y16 ? 1 : 2;
  RT xr[NSL][RPI][CHB][NR];
  RY dr[NSL][RPI][CHB][NY];
  float mr[NSL][RPI], rr[NSL][RPI];
  const int64_t stride = gridDim.x;
  // rows r0 + q*stride, q < RPI; past the last row the last row is re-read (masked in the
  // math): a load behind a branch would leave the wait counters unknown at the join
  auto load = [&](auto S, int64_t r0) {
    constexpr int s = decltype(S)::value;
#pragma unroll
    for (int q = 0; q < RPI; ++q) {
      const int64_t r = min(r0 + q * stride, p.rows - 1);
      // the row statistics first: a load issued after the next row's prefetch would make
      // its wait (vmcnt counts in order) drain that prefetch too
      mr[s][q] = p.mean[r];
      rr[s][q] = p.rstd[r];
    }
#pragma unroll
    for (int q = 0; q < RPI; ++q) {
      const int64_t r = min(r0 + q * stride, p.rows - 1);
      const E* x = reinterpret_cast<const E*>(p.x) + r * p.xs;
      const Y* dy = reinterpret_cast<const Y*>(p.dy) + r * p.dys;
      // unconditional loads (lanes past C read column 0, masked in the math)
#pragma unroll
      for (int c = 0; c < CHB; ++c) {
        const int col0 = (c * 256 + t) * 8;
        const int col = col0 < p.C ? col0 : 0;
#pragma unroll
        for (int k = 0; k < NR; ++k) xr[s][q][c][k] = ldv(reinterpret_cast<const RT*>(x + col + k * 4));
#pragma unroll
        for (int k = 0; k < NY; ++k) dr[s][q][c][k] = ldv(reinterpret_cast<const RY*>(dy + col + k * 4));
      }
    }
  };
  auto cvt = [&](auto T16, const auto& v, float* f) {
    using V = decltype(T16);
    if constexpr (sizeof(V) == 2) {
      raw_cvt<V>(v[0], f);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) { f[j] = v[0][j]; f[j + 4] = v[1][j]; }
    }
  };
  int par = 0;
  // this thread's LN weights, the same for every row: loaded once (a per-row load issued
  // behind the next row's prefetch would drain it at its wait)
  float wv[CHB][8];
#pragma unroll
  for (int c = 0; c < CHB; ++c) {
    const int col = (c * 256 + t) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) wv[c][j] = col < p.C ? p.w[col + j] : 0.f;
  }
  auto body = [&](auto S, int64_t r0) {
    constexpr int s = decltype(S)::value;
    if (r0 + PD * RPI * stride < p.rows)                       // the rows PD groups ahead in flight
      load(std::integral_constant<int, (s + PD) % NSL>{}, r0 + PD * RPI * stride);
    float xh[RPI][CHB][8], g[RPI][CHB][8];
#pragma unroll
    for (int q = 0; q < RPI; ++q) {
      const bool live = r0 + q * stride < p.rows;      // workgroup-uniform
      const float mean = mr[s][q], rstd = rr[s][q];
      float sg = 0.f, sgx = 0.f;
#pragma unroll
      for (int c = 0; c < CHB; ++c) {
        const bool ok = live && (c * 256 + t) * 8 < p.C;
        float xv[8], dv[8];
        cvt(E{}, xr[s][q][c], xv);
        cvt(Y{}, dr[s][q][c], dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[q][c][j] = ok ? (xv[j] - mean) * rstd : 0.f;
          const float dys = ok ? dv[j] * p.out_scale : 0.f;
          dwp[c][j] = fmaf(dys, xh[q][c][j], dwp[c][j]);
          dbp[c][j] += dys;
          g[q][c][j] = dys * wv[c][j];
          sg += g[q][c][j];
          sgx = fmaf(g[q][c][j], xh[q][c][j], sgx);
        }
      }
      sg = wave_sum(sg);
      sgx = wave_sum(sgx);
      if (lane == 0) { red[par][q][wave][0] = sg; red[par][q][wave][1] = sgx; }
    }
    // LDS-only barrier: __syncthreads() would also wait for the next rows' prefetch
    __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int q = 0; q < RPI; ++q) {
      const int64_t r = r0 + q * stride;
      if (r >= p.rows) break;
      const float rstd = rr[s][q];
      const float mg = (red[par][q][0][0] + red[par][q][1][0] + red[par][q][2][0] + red[par][q][3][0]) * inv_c;
      const float mgx = (red[par][q][0][1] + red[par][q][1][1] + red[par][q][2][1] + red[par][q][3][1]) * inv_c;
      E* dx = reinterpret_cast<E*>(p.dx) + r * p.dxs;
#pragma unroll
      for (int c = 0; c < CHB; ++c) {
        const int col = (c * 256 + t) * 8;
        if (col < p.C) {
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = rstd * (g[q][c][j] - mg - xh[q][c][j] * mgx);
          if constexpr (std::is_same<E, float>::value && Y16) {
            if (p.dres) {                        // residual fusion: + the residual branch's gradient
              float d[8];
              ld8<float>(p.dres + r * p.dress + col, d);
#pragma unroll
              for (int j = 0; j < 8; ++j) o[j] += d[j];
            }
            if (p.dx16) st8<Y>(reinterpret_cast<Y*>(p.dx16) + r * p.dx16s + col, o);
          }
          st8<E>(dx + col, o);
        }
      }
    }
    par ^= 1;
  };
  int64_t r = blockIdx.x;
  if (r < p.rows) load(std::integral_constant<int, 0>{}, r);
  if constexpr (PD >= 2) if (r + RPI * stride < p.rows) load(std::integral_constant<int, 1>{}, r + RPI * stride);
  if constexpr (PD >= 3) if (r + 2 * RPI * stride < p.rows) load(std::integral_constant<int, 2>{}, r + 2 * RPI * stride);
  if constexpr (PD >= 4) if (r + 3 * RPI * stride < p.rows) load(std::integral_constant<int, 3>{}, r + 3 * RPI * stride);
  if constexpr (PD >= 5) if (r + 4 * RPI * stride < p.rows) load(std::integral_constant<int, 4>{}, r + 4 * RPI * stride);
  // slot s of the ring serves row groups s, s + NSL, ...: the loop unrolled NSL times
  auto run = [&](auto S) -> bool {
    body(S, r);
    r += RPI * stride;
    return r < p.rows;
  };
  while (r < p.rows) {
    if (!run(std::integral_constant<int, 0>{})) break;
    if (!run(std::integral_constant<int, 1>{})) break;
    if constexpr (NSL > 2) if (!run(std::integral_constant<int, 2 % NSL>{})) break;
    if constexpr (NSL > 3) if (!run(std::integral_constant<int, 3 % NSL>{})) break;
    if constexpr (NSL > 4) if (!run(std::integral_constant<int, 4 % NSL>{})) break;
    if constexpr (NSL > 5) if (!run(std::integral_constant<int, 5 % NSL>{})) break;
  }
#pragma unroll
  for (int c = 0; c < CHB; ++c) {
    const int col = (c * 256 + t) * 8;
    if (col < p.C) {
      if (p.partial) {
        float* pw = p.partial + ((int64_t)blockIdx.x * 2) * p.C + col;
        float* pb = pw + p.C;
        *reinterpret_cast<f32x4*>(pw) = f32x4{dwp[c][0], dwp[c][1], dwp[c][2], dwp[c][3]};
        *reinterpret_cast<f32x4*>(pw + 4) = f32x4{dwp[c][4], dwp[c][5], dwp[c][6], dwp[c][7]};
        *reinterpret_cast<f32x4*>(pb) = f32x4{dbp[c][0], dbp[c][1], dbp[c][2], dbp[c][3]};
        *reinterpret_cast<f32x4*>(pb + 4) = f32x4{dbp[c][4], dbp[c][5], dbp[c][6], dbp[c][7]};
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { atomicAdd(p.dw + col + j, dwp[c][j]); atomicAdd(p.db + col + j, dbp[c][j]); }
      }
    }
  }
}

// dw / db += the column sums of the per-block partials, in a fixed order: pass 1 sums
// each of kLnChunks contiguous runs of blocks per column (many threads in flight),
// pass 2 adds the kLnChunks run sums in order
constexpr int kLnChunks = 32;
__global__ __launch_bounds__(256) void ln_bwd_reduce1_kernel(const float* part, int nblk, int64_t C, float* part2) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;      // over 2 * C
  if (e >= 2 * C) return;
  const int which = (int)(e / C);
  const int64_t col = e % C;
  const int per = (nblk + kLnChunks - 1) / kLnChunks;
  const int b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  float s = 0.f;
#pragma unroll 8
  for (int b = b0; b < b1; ++b) s += part[((int64_t)b * 2 + which) * C + col];
  part2[(int64_t)blockIdx.y * 2 * C + e] = s;
}
__global__ __launch_bounds__(256) void ln_bwd_reduce2_kernel(const float* part2, int64_t C, float* dw, float* db) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= 2 * C) return;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < kLnChunks; ++j) s += part2[(int64_t)j * 2 * C + e];
  const int64_t col = e % C;
  (e >= C ? db : dw)[col] += s;
}
// The two passes above in ONE launch: a workgroup owns 4*QD consecutive entries of the
// [2][C] partial row (QD lanes x 4 floats) and one thread row per chunk of blocks
// (256 / QD chunks), each summing its run of blocks with 16-byte loads; the chunk sums
// meet in LDS and 4*QD threads add them in chunk order -- a fixed order, so dw / db stay
// bitwise reproducible (QD = 8: the same order as reduce1 + reduce2, bitwise equal to
// them).  Saves the second launch, its gap and the part2 round trip (C' is a multiple of
// 8: quads never straddle dw / db).
#ifndef DTA_LN_REDUCE_QD
#define DTA_LN_REDUCE_QD 8
#endif
template <int QD>
__global__ __launch_bounds__(256) void ln_bwd_reduce_kernel(const float* part, int nblk, int64_t C, float* dw, float* db) {
  constexpr int NCH = 256 / QD, W = 4 * QD;
  const int t = threadIdx.x, q = t % QD, j = t / QD;
  const int64_t e0 = (int64_t)blockIdx.x * W + q * 4;
  const int per = (nblk + NCH - 1) / NCH;
  const int b0 = j * per, b1 = min(nblk, b0 + per);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (e0 < 2 * C) {
#pragma unroll 16
    for (int b = b0; b < b1; ++b) s += *reinterpret_cast<const f32x4*>(part + (int64_t)b * 2 * C + e0);
  }
  __shared__ float red[NCH][W + 1];
#pragma unroll
  for (int k = 0; k < 4; ++k) red[j][q * 4 + k] = s[k];
  __syncthreads();
  if (t < W) {
    const int64_t e = (int64_t)blockIdx.x * W + t;
    if (e < 2 * C) {
      float r = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) r += red[c][t];
      const int64_t col = e % C;
      (e >= C ? db : dw)[col] += r;
    }
  }
}
#ifndef DTA_LN_REDUCE_ONE
#define DTA_LN_REDUCE_ONE 1      // the one-launch ordered reduce (0: reduce1 + reduce2)
#endif
static void ln_bwd_reduce(const LnParams& p, int nblk, hipStream_t st) {
  if (DTA_LN_REDUCE_ONE) {
    constexpr int W = 4 * DTA_LN_REDUCE_QD;
    hipLaunchKernelGGL(ln_bwd_reduce_kernel<DTA_LN_REDUCE_QD>, dim3((unsigned)((2 * p.C + W - 1) / W)), dim3(256), 0, st,
                       p.partial, nblk, p.C, p.dw, p.db);
  } else {
    float* part2 = p.partial + (int64_t)nblk * 2 * p.C;
    const unsigned g = (unsigned)((2 * p.C + 255) / 256);
    hipLaunchKernelGGL(ln_bwd_reduce1_kernel, dim3(g, kLnChunks), dim3(256), 0, st, p.partial, nblk, p.C, part2);
    hipLaunchKernelGGL(ln_bwd_reduce2_kernel, dim3(g), dim3(256), 0, st, part2, p.C, p.dw, p.db);
  }
}


struct RopeDiv { FastDiv row, T, per_row, N; uint32_t rowlen; };

// one thread = 4 rotation pairs (8 elements); the 64-bit index decomposition of the first
// version (five int64 div/mod per thread) cost more VALU than the HBM time of its 32 bytes
template <class E, class S>
__global__ __launch_bounds__(256) void rope_kernel(RopeParams p, RopeDiv dv) {
  const uint32_t total = (uint32_t)p.B * p.T * p.H * p.N * (p.HS / 8);
  for (uint32_t idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
    const uint32_t row = dv.row.div(idx), within = idx - row * dv.rowlen;
    const uint32_t b = dv.T.div(row), t = row - b * p.T;
    const uint32_t hi = dv.per_row.div(within), c = within - hi * dv.per_row.d;
    const uint32_t h = dv.N.div(hi), i = hi - h * p.N;
    const S* src = reinterpret_cast<const S*>(p.src.p) + b * p.src.sb + (int64_t)t * p.src.st + h * p.src.sh + i * p.src.si + c * 8;
    E* dst = reinterpret_cast<E*>(p.dst.p) + b * p.dst.sb + (int64_t)t * p.dst.st + h * p.dst.sh + i * p.dst.si + c * 8;
    float x[8], o[8];
    ld8<S>(src, x);
    const float* f = p.freqs + ((int64_t)t * (p.HS / 2) + c * 4) * 2;
    const f32x4 f0 = *reinterpret_cast<const f32x4*>(f), f1 = *reinterpret_cast<const f32x4*>(f + 4);
    const float fr[8] = {f0[0], f0[1], f0[2], f0[3], f1[0], f1[1], f1[2], f1[3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float cs = fr[2 * j], sn = p.inverse ? -fr[2 * j + 1] : fr[2 * j + 1];
      const float a = x[2 * j], bb = x[2 * j + 1];
      o[2 * j] = a * cs - bb * sn;          // (a + ib)(cos + i sin)
      o[2 * j + 1] = a * sn + bb * cs;
    }
    st8<E>(dst, o);
  }
}


template <class E>
__global__ __launch_bounds__(256) void cast_f32_kernel(const float* src, T5 dst, int B, int T, int H, int N, int HS) {
  const int per_row = HS / 8;
  const int64_t total = (int64_t)B * T * H * N * per_row;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    int64_t r = idx;
    const int c = r % per_row; r /= per_row;
    const int i = r % N; r /= N;
    const int h = r % H; r /= H;
    const int t = r % T; const int b = (int)(r / T);
    float v[8];
    ld8<float>(src + idx * 8, v);
    st8<E>(reinterpret_cast<E*>(dst.p) + b * dst.sb + (int64_t)t * dst.st + h * dst.sh + i * dst.si + c * 8, v);
  }
}

// ---------------------------------------------------------------- hosts ---
static inline int grid_for(int64_t items) {
  int64_t g = (items + 255) / 256;
  return (int)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}

#ifndef DTA_LN_BWD_ROWBLOCK
#define DTA_LN_BWD_ROWBLOCK 1
#endif
// blocks of the LN backward: enough waves in flight to cover HBM latency, few enough
// that the per-block column partials stay small (dta_ln_bwd_workspace_bytes)
#ifndef DTA_LN_BWD_MAXBLK
#define DTA_LN_BWD_MAXBLK 512    // workgroups of the backward: occupancy vs partial rows to reduce (1024: +2%, r04_ab_ln_rpi_blocks.json)
#endif
int ln_bwd_blocks(int64_t rows) { return (int)std::min<int64_t>((rows + 7) / 8, DTA_LN_BWD_MAXBLK); }
int64_t ln_bwd_workspace_floats(int64_t rows, int64_t C) { return ((int64_t)ln_bwd_blocks(rows) + kLnChunks) * 2 * C; }

template <class E>
int ln_launch(const LnParams& p, bool bwd, hipStream_t st) {
  const int64_t ch = (p.C + 511) / 512;
  const int fwd_grid = (int)((p.rows + 3) / 4);
  const int bwd_grid = ln_bwd_blocks(p.rows);
#define DTA_LN(CH_)                                                                    \
  if (ch <= CH_) {                                                                     \
    if (bwd) {                                                                         \
      if (DTA_LN_BWD_ROWBLOCK && CH_ <= 16 && (CH_ + 3) / 4 * 2048 >= p.C)             \
        hipLaunchKernelGGL((ln_bwd_rb_kernel<E, (CH_ + 3) / 4>), dim3(bwd_grid), dim3(256), 0, st, p); \
      else                                                                             \
        hipLaunchKernelGGL((ln_bwd_kernel<E, CH_>), dim3(bwd_grid), dim3(256), 0, st, p); \
      if (p.partial) ln_bwd_reduce(p, bwd_grid, st);                                   \
    } else {                                                                           \
      hipLaunchKernelGGL((ln_fwd_kernel<E, CH_>), dim3(fwd_grid), dim3(256), 0, st, p); \
    }                                                                                  \
    return (int)hipGetLastError();                                                     \
  }
  DTA_LN(1) DTA_LN(2) DTA_LN(4) DTA_LN(8) DTA_LN(16)
#undef DTA_LN
  return -2;
}

// fp32 x / dx with 16-bit y / dy (block-per-row backward only)
template <class Y>
int ln_launch_mixed(const LnParams& p, bool bwd, hipStream_t st) {
  const int64_t ch = (p.C + 511) / 512;
  const int fwd_grid = (int)((p.rows + 3) / 4);
  const int bwd_grid = ln_bwd_blocks(p.rows);
#define DTA_LNM(CH_)                                                                             \
  if (ch <= CH_) {                                                                               \
    if (bwd) {                                                                                   \
      hipLaunchKernelGGL((ln_bwd_rb_kernel<float, (CH_ + 3) / 4, Y>), dim3(bwd_grid), dim3(256), 0, st, p); \
      if (p.partial) ln_bwd_reduce(p, bwd_grid, st);                                             \
    } else {                                                                                     \
      hipLaunchKernelGGL((ln_fwd_kernel<float, CH_, Y>), dim3(fwd_grid), dim3(256), 0, st, p);  \
    }                                                                                            \
    return (int)hipGetLastError();                                                               \
  }
  DTA_LNM(1) DTA_LNM(2) DTA_LNM(4) DTA_LNM(8) DTA_LNM(16)
#undef DTA_LNM
  return -2;
}

int launch_ln_mixed(int y_dtype, const LnParams& p, bool bwd, hipStream_t st) {
  if (p.rows == 0) return 0;
  switch (y_dtype) {
    case 0: return ln_launch_mixed<__bf16>(p, bwd, st);
    case 1: return ln_launch_mixed<_Float16>(p, bwd, st);
  }
  return -2;
}

int launch_ln(int dtype, const LnParams& p, bool bwd, hipStream_t st) {
  if (p.rows == 0) return 0;
  switch (dtype) {
    case 0: return ln_launch<__bf16>(p, bwd, st);
    case 1: return ln_launch<_Float16>(p, bwd, st);
    case 2: return ln_launch<float>(p, bwd, st);
  }
  return -2;
}

int launch_rope(int dtype, bool src_f32, const RopeParams& p, hipStream_t st) {
  const int64_t items = (int64_t)p.B * p.T * p.H * p.N * (p.HS / 8);
  if (items == 0) return 0;
  if (items >= (1ll << 31) || p.HS % 8) return -2;
  RopeDiv dv;
  dv.rowlen = (uint32_t)(p.H * p.N * (p.HS / 8));
  dv.row = FastDiv(dv.rowlen);
  dv.T = FastDiv((uint32_t)p.T);
  dv.per_row = FastDiv((uint32_t)(p.HS / 8));
  dv.N = FastDiv((uint32_t)p.N);
  dim3 g(grid_for(items));
#define DTA_R(E_)                                                                         \
  if (src_f32) hipLaunchKernelGGL((rope_kernel<E_, float>), g, dim3(256), 0, st, p, dv);   \
  else hipLaunchKernelGGL((rope_kernel<E_, E_>), g, dim3(256), 0, st, p, dv);
  switch (dtype) {
    case 0: DTA_R(__bf16) break;
    case 1: DTA_R(_Float16) break;
    case 2: DTA_R(float) break;
    default: return -2;
  }
#undef DTA_R
  return (int)hipGetLastError();
}

// dcoef[h][i] = sum of the dQ kernel's per-wave partials part[h][i][0..per), in order
__global__ __launch_bounds__(256) void dcoef_reduce_kernel(const float* part, float* dcoef, int64_t per) {
  const float* src = part + (int64_t)blockIdx.x * per;
  float s = 0.f;
  for (int64_t t = threadIdx.x; t < per; t += 256) s += src[t];
  s = wave_sum(s);
  __shared__ float w4[4];
  if ((threadIdx.x & 63) == 0) w4[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) dcoef[blockIdx.x] = (w4[0] + w4[1]) + (w4[2] + w4[3]);
}

int launch_dcoef_reduce(const float* part, float* dcoef, int H, int N, int64_t per, hipStream_t st) {
  hipLaunchKernelGGL(dcoef_reduce_kernel, dim3(H * N), dim3(256), 0, st, part, dcoef, per);
  return (int)hipGetLastError();
}

// attn_dq leaves each dQ branch group's delta rows relative to the group's first branch a
// (-delta_a, then delta_a - delta_i); re-base them onto the dK/dV grouping (capi.hip
// bwd_group_cap).  Bit i of from / to: a group starts at branch i.  delta is [N][rows];
// one thread per row decodes to delta_i and re-encodes in place, in branch order.
__global__ __launch_bounds__(256) void delta_rebase_kernel(float* delta, int64_t rows, int N,
                                                           uint64_t from, uint64_t to) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < rows; r += (int64_t)gridDim.x * 256) {
    float head = 0.f;
    for (int i = 0; i < N; ++i) {
      float* d = delta + i * rows + r;
      const float v = *d;
      if ((from >> i) & 1) head = -v;
      *d = ((from >> i) & 1) ? head : head - v;
    }
    for (int i = 0; i < N; ++i) {
      float* d = delta + i * rows + r;
      const float v = *d;
      if ((to >> i) & 1) head = v;
      *d = ((to >> i) & 1) ? -head : head - v;
    }
  }
}

int launch_delta_rebase(float* delta, int64_t rows, int N, uint64_t from, uint64_t to, hipStream_t st) {
  const int64_t blocks = (rows + 255) / 256;
  hipLaunchKernelGGL(delta_rebase_kernel, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(256), 0, st,
                     delta, rows, N, from, to);
  return (int)hipGetLastError();
}

// ---- dst += (float)src (fp32 master-gradient accumulation).  HBM-bound: 8 elements
// per thread and step (16-byte loads of 16-bit src), grid-stride, scalar tail.
template <class E>
__global__ __launch_bounds__(256) void accumulate_kernel(int64_t n, const E* __restrict__ src, float* __restrict__ dst) {
  const int64_t n8 = n / 8, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += stride) {
    float a[8];
    ld8<E>(src + i * 8, a);
    f32x4 d0 = *reinterpret_cast<const f32x4*>(dst + i * 8), d1 = *reinterpret_cast<const f32x4*>(dst + i * 8 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { d0[j] += a[j]; d1[j] += a[4 + j]; }
    *reinterpret_cast<f32x4*>(dst + i * 8) = d0;
    *reinterpret_cast<f32x4*>(dst + i * 8 + 4) = d1;
  }
  for (int64_t i = n8 * 8 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] += (float)src[i];
}

int launch_accumulate(int dtype, int64_t n, const void* src, float* dst, hipStream_t st) {
  const int64_t items = (n + 7) / 8;
  const dim3 g((unsigned)std::min<int64_t>((items + 255) / 256, 256 * 16));
  switch (dtype) {
    case 0: hipLaunchKernelGGL(accumulate_kernel<__bf16>, g, dim3(256), 0, st, n, (const __bf16*)src, dst); break;
    case 1: hipLaunchKernelGGL(accumulate_kernel<_Float16>, g, dim3(256), 0, st, n, (const _Float16*)src, dst); break;
    case 2: hipLaunchKernelGGL(accumulate_kernel<float>, g, dim3(256), 0, st, n, (const float*)src, dst); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// ---- SwiGLU (diff_transformer.py / Ndiff_transformer.py / control.py SwiGLU.forward):
// out = silu(a) * b with a = linear_gate(x), b = linear_xform(x), and its backward
// da = dout * b * silu'(a), db = dout * silu(a), silu'(a) = s (1 + a (1 - s)), s = sigmoid(a).
// One pass each (PyTorch runs silu, mul, mul-backward and silu-backward as separate
// passes); rows of a/b/out/dout/da/db may be strided views (row length n).  fp32 math.
template <class E>
__device__ __forceinline__ float silu_f(float a, float& sg) {
  sg = 1.f / (1.f + __expf(-a));
  return a * sg;
}
template <class E>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(SwigluParams p) {
  const int64_t per_row = p.n / 8, total = p.rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / per_row, c = (i % per_row) * 8;
    float a[8], b[8], o[8];
    ld8<E>(reinterpret_cast<const E*>(p.a) + r * p.as + c, a);
    ld8<E>(reinterpret_cast<const E*>(p.b) + r * p.bs + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sg;
      o[j] = silu_f<E>(a[j], sg) * b[j];
    }
    st8<E>(reinterpret_cast<E*>(p.out) + r * p.os + c, o);
  }
}
template <class E>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(SwigluParams p) {
  const int64_t per_row = p.n / 8, total = p.rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / per_row, c = (i % per_row) * 8;
    float a[8], b[8], d[8], da[8], db[8];
    ld8<E>(reinterpret_cast<const E*>(p.a) + r * p.as + c, a);
    ld8<E>(reinterpret_cast<const E*>(p.b) + r * p.bs + c, b);
    ld8<E>(reinterpret_cast<const E*>(p.dout) + r * p.dos + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sg;
      const float sl = silu_f<E>(a[j], sg);
      db[j] = d[j] * sl;
      da[j] = d[j] * b[j] * (sg * (1.f + a[j] * (1.f - sg)));
    }
    st8<E>(reinterpret_cast<E*>(p.da) + r * p.das + c, da);
    st8<E>(reinterpret_cast<E*>(p.db) + r * p.dbs + c, db);
  }
}

// Backward with the column sums of dA | dB (the packed gate / xform Linears' bias
// gradient, diff_transformer.py:95-105 under autocast: the sum over rows of the
// gradients as stored): each block owns 2048 columns x SWIGLU_RB rows, sums the
// rounded values in fp32 and writes its partials [row block][2n]; a second kernel adds
// the row blocks in a fixed order (bitwise reproducible, no atomics).
constexpr int SWIGLU_RB = 128;
template <class E>
__global__ __launch_bounds__(256) void swiglu_bwd_bias_kernel(SwigluParams p, float* part) {
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= p.n) return;
  const int64_t r0 = (int64_t)blockIdx.y * SWIGLU_RB, r1 = min(r0 + SWIGLU_RB, p.rows);
  float sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sa[j] = 0.f; sb[j] = 0.f; }
#pragma unroll 2
  for (int64_t r = r0; r < r1; ++r) {
    float a[8], b[8], d[8], da[8], db[8];
    ld8<E>(reinterpret_cast<const E*>(p.a) + r * p.as + c, a);
    ld8<E>(reinterpret_cast<const E*>(p.b) + r * p.bs + c, b);
    ld8<E>(reinterpret_cast<const E*>(p.dout) + r * p.dos + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sg;
      const float sl = silu_f<E>(a[j], sg);
      db[j] = (float)(E)(d[j] * sl);
      da[j] = (float)(E)(d[j] * b[j] * (sg * (1.f + a[j] * (1.f - sg))));
      sa[j] += da[j];
      sb[j] += db[j];
    }
    st8<E>(reinterpret_cast<E*>(p.da) + r * p.das + c, da);
    st8<E>(reinterpret_cast<E*>(p.db) + r * p.dbs + c, db);
  }
  float* pa = part + (int64_t)blockIdx.y * 2 * p.n + c;
  st8<float>(pa, sa);
  st8<float>(pa + p.n, sb);
}
// the column sums of the nblk partial rows, in a fixed order, in two passes: pass 1 sums each
// of kSwChunks contiguous runs of partial rows (every load of a run in flight together),
// pass 2 adds the run sums in order.  (One pass with one thread per column walked all
// 256 partial rows of cfg4 serially: 98 us per call, latency-bound.)
constexpr int kSwChunks = 16;
__global__ __launch_bounds__(256) void swiglu_bias_reduce1_kernel(const float* part, int nblk, int64_t n2, float* part2) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n2) return;
  const int per = (nblk + kSwChunks - 1) / kSwChunks;
  const int b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  float s = 0.f;
#pragma unroll 16
  for (int b = b0; b < b1; ++b) s += part[(int64_t)b * n2 + j];
  part2[(int64_t)blockIdx.y * n2 + j] = s;
}
__global__ __launch_bounds__(256) void swiglu_bias_reduce_kernel(const float* part2, int64_t n2, float* out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n2) return;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kSwChunks; ++c) s += part2[(int64_t)c * n2 + j];
  out[j] = s;
}
int64_t swiglu_bias_work_floats(int64_t rows, int64_t n) {
  return ((rows + SWIGLU_RB - 1) / SWIGLU_RB + kSwChunks) * 2 * n;
}

int launch_swiglu_bias(int dtype, const SwigluParams& p, float* dbias, float* work, hipStream_t st) {
  const int nblk = (int)((p.rows + SWIGLU_RB - 1) / SWIGLU_RB);
  const dim3 g((unsigned)((p.n / 8 + 255) / 256), (unsigned)nblk);
  switch (dtype) {
    case 0: hipLaunchKernelGGL(swiglu_bwd_bias_kernel<__bf16>, g, dim3(256), 0, st, p, work); break;
    case 1: hipLaunchKernelGGL(swiglu_bwd_bias_kernel<_Float16>, g, dim3(256), 0, st, p, work); break;
    case 2: hipLaunchKernelGGL(swiglu_bwd_bias_kernel<float>, g, dim3(256), 0, st, p, work); break;
    default: return -1;
  }
  float* part2 = work + (int64_t)nblk * 2 * p.n;
  const unsigned gx = (unsigned)((2 * p.n + 255) / 256);
  hipLaunchKernelGGL(swiglu_bias_reduce1_kernel, dim3(gx, kSwChunks), dim3(256), 0, st, work, nblk, 2 * p.n, part2);
  hipLaunchKernelGGL(swiglu_bias_reduce_kernel, dim3(gx), dim3(256), 0, st, part2, 2 * p.n, dbias);
  return (int)hipGetLastError();
}

int launch_swiglu(int dtype, const SwigluParams& p, bool bwd, hipStream_t st) {
  const int64_t items = p.rows * (p.n / 8);
  if (items == 0) return 0;
  dim3 g(grid_for(items));
#define DTA_SW(E_)                                                                       \
  if (bwd) hipLaunchKernelGGL(swiglu_bwd_kernel<E_>, g, dim3(256), 0, st, p);            \
  else hipLaunchKernelGGL(swiglu_fwd_kernel<E_>, g, dim3(256), 0, st, p);
  switch (dtype) {
    case 0: DTA_SW(__bf16) break;
    case 1: DTA_SW(_Float16) break;
    case 2: DTA_SW(float) break;
    default: return -2;
  }
#undef DTA_SW
  return (int)hipGetLastError();
}

int launch_cast(int dtype, const float* src, const T5& dst, int B, int T, int H, int N, int HS, hipStream_t st) {
  const int64_t items = (int64_t)B * T * H * N * (HS / 8);
  if (items == 0) return 0;
  dim3 g(grid_for(items));
  switch (dtype) {
    case 0: hipLaunchKernelGGL(cast_f32_kernel<__bf16>, g, dim3(256), 0, st, src, dst, B, T, H, N, HS); break;
    case 1: hipLaunchKernelGGL(cast_f32_kernel<_Float16>, g, dim3(256), 0, st, src, dst, B, T, H, N, HS); break;
    case 2: hipLaunchKernelGGL(cast_f32_kernel<float>, g, dim3(256), 0, st, src, dst, B, T, H, N, HS); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

}  // namespace dta
