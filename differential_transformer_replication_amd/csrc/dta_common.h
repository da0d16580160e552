// dta_common.h -- shared device helpers for the gfx950 differential-attention
// kernels: element traits, MFMA fragment I/O, wave reductions.
//
// All matrix work uses 32x32 MFMA tiles (64-lane waves):
//   bf16 / f16 : v_mfma_f32_32x32x16_{bf16,f16}  (K = 16 per instruction)
//   f32        : v_mfma_f32_32x32x2_f32          (K = 2, exact fp32; parity builds)
// The C/D accumulator layout is the same for every dtype on gfx950:
//   lane l, register r  ->  row (r&3) + 8*(r>>2) + 4*(l>>5),  column l&31.
// A/B operand maps (lane l, half h = l>>5):
//   16-bit: A[row l&31][k = 8h + j], B[k = 8h + j][col l&31], j = 0..7
//   f32   : A[row l&31][k = h],      B[k = h][col l&31]
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dta {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int rowof(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }

// combine lane l with lane l^32 (the two halves that hold the same column):
// one v_permlane32_swap (VALU) instead of an LDS bpermute round trip
__device__ __forceinline__ float wave_max_halves(float v) {
  const unsigned u = __float_as_uint(v);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float wave_sum_halves(float v) {
  const unsigned u = __float_as_uint(v);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// XCD-aware workgroup order: blocks are dealt round-robin over the 8 XCDs;
// remap the linear id so each XCD receives a contiguous range (neighbouring
// tiles of one (batch, head) then share that XCD's L2).  Bijective for any
// count (cdna_hip_programming.md T1).  Speed only -- never correctness.
__device__ __forceinline__ int xcd_remap(int id, int n) {
  const int q = n / 8, r = n % 8, x = id % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
}

// Dispatch order of the attention grids (grid x = work rank, y / z = head, chunk, batch):
// the work rank r (0 = the workgroups with the most causal tiles) varies slowest and the
// (y, z) index fastest.  Blocks are dealt round-robin over the 8 XCDs, so every XCD starts
// on its longest workgroups and ends on its shortest (longest-processing-time first: no
// long workgroup is left running alone at the end of the grid), and, when gridDim.y *
// gridDim.z is a multiple of 8, all workgroups of one (y, z) land on one XCD (its L2).
// Speed only -- never correctness.
#ifndef DTA_LPT
#define DTA_LPT 1
#endif
// DTA_LPT_GROUP = G > 0 (default 4): each XCD walks its (y, z) pairs G at a time,
// longest-first inside a group, so only about 2G pairs' K/V (forward, dQ) or Q/dO
// (dK/dV) are live in that XCD's L2 at once instead of all of them (needs gridDim.y *
// gridDim.z % 8 == 0; blocks are dealt to XCD id % 8).  One-process A/B at cfg2
// (profiles/r03_lpt_group_ab.json): fwd+dq+dkdv 3.052 -> 2.891 ms (G = 1 / 2 / 3 / 6 / 8:
// 3.140 / 3.001 / 3.081 / 2.926 / 2.912); fabric reads per launch fwd 2575 -> 734 MB,
// dq 2929 -> 1258, dK/dV 3146 -> 867; cfg3 N=3 1.231 -> 1.211, cfg5 unchanged.  0 = the
// ungrouped longest-first order.
#ifndef DTA_LPT_GROUP
#define DTA_LPT_GROUP 4
#endif
// Between 8 and 16 pairs per XCD the walk takes two equal groups instead of groups of
// DTA_LPT_GROUP (cfg3's 12 pairs: 4 + 4 + 4 -> 6 + 6; one-process A/B profiles/r05zc_ab_lpt_groups.json:
// cfg3 N = 3 fwd+dq+dkdv 1.099 -> 1.060 ms, N = 4 1.381 -> 1.344; cfg2's 16 pairs keep groups of
// 4, its 2 x 8 measured equal).
#ifndef DTA_LPT_HALVES
#define DTA_LPT_HALVES 1
#endif
__device__ __forceinline__ void lpt_order(int& r, int& y, int& z, int& id) {
  id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int nyz = gridDim.y * gridDim.z;
  if (DTA_LPT && DTA_LPT_GROUP > 0 && nyz % 8 == 0) {
    const int xcd = id & 7, s = id >> 3;            // s-th block this XCD receives
    const int per = nyz >> 3, R = gridDim.x;        // pairs per XCD, work ranks
    const int G = (DTA_LPT_HALVES && per > 8 && per < 16) ? (per + 1) / 2 : DTA_LPT_GROUP;
    const int g = s / (R * G);
    const int gsz = min(G, per - g * G);
    const int t = s - g * R * G;
    r = t / gsz;
    const int pair = xcd + 8 * (g * G + t % gsz);
    y = pair % gridDim.y;
    z = pair / gridDim.y;
    return;
  }
  if (DTA_LPT) {
    r = id / nyz;
    const int rest = id - r * nyz;
    y = rest % gridDim.y;
    z = rest / gridDim.y;
  } else {
    const int lin = xcd_remap(id, gridDim.x * gridDim.y * gridDim.z);
    r = lin % gridDim.x;
    y = (lin / gridDim.x) % gridDim.y;
    z = lin / (gridDim.x * gridDim.y);
    id = lin;
  }
}

template <class E> struct Ops;

// ----------------------------------------------------------- 16-bit types ---
template <class E, class V8, class V4>
struct Ops16 {
  using elem = E;
  using frag = V8;                    // 8 elements = 4 VGPRs
  static constexpr int KSTEP = 16;    // k per MFMA
  static constexpr int KH = 8;        // k elements per lane half
  static constexpr int VEC = 8;       // elements per 16-byte global access

  __device__ static float to_f(E x) { return (float)x; }
  __device__ static E from_f(float x) { return (E)x; }

  // A or B operand from a row-major image: row pointer at k = 0.
  __device__ static frag row(const E* rowp, int s, int h) {
    return *reinterpret_cast<const frag*>(rowp + s * KSTEP + h * KH);
  }
  // 4 rows x 16 columns -> lane i of each 16-lane group gets column i
  // (ds_read_b64_tr_b16).  base: element (row0, col0) of the 4x(32) strip.
  __device__ static V4 tr4(const E* base, int stride, int lane) {
    const int i = lane & 15;
    const E* p = base + (i >> 2) * stride + ((lane >> 4) & 1) * 16 + (i & 3) * 4;
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
    return __builtin_bit_cast(V4, v);
  }
  // Transposed operand whose k order matches an accumulator packed by pack():
  // element j <-> k row 16s + 8(j>>2) + 4h + (j&3) of the 32-row block at base.
  __device__ static frag tr_perm(const E* base, int stride, int s, int h, int lane) {
    V4 lo = tr4(base + (16 * s + 4 * h) * stride, stride, lane);
    V4 hi = tr4(base + (16 * s + 8 + 4 * h) * stride, stride, lane);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
  // Transposed operand in natural k order: element j <-> k row KSTEP*s + 8h + j.
  __device__ static frag tr_nat(const E* base, int stride, int s, int h, int lane) {
    V4 lo = tr4(base + (16 * s + 8 * h) * stride, stride, lane);
    V4 hi = tr4(base + (16 * s + 8 * h + 4) * stride, stride, lane);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
  // accumulator registers 8s..8s+7 -> operand fragment of k-step s
  template <int S>
  __device__ static frag pack(const f32x16& a) {
    frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (E)a[8 * S + j];
    return f;
  }
  __device__ static frag zero() { return frag{}; }
  __device__ static frag load_global(const E* p) { return *reinterpret_cast<const frag*>(p); }
};

template <> struct Ops<__bf16> : Ops16<__bf16, bf16x8, bf16x4> {
  __device__ static f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Ops<_Float16> : Ops16<_Float16, f16x8, f16x4> {
  __device__ static f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

// ------------------------------------------------------------------ fp32 ---
template <> struct Ops<float> {
  using elem = float;
  using frag = float;
  static constexpr int KSTEP = 2;
  static constexpr int KH = 1;
  static constexpr int VEC = 4;

  __device__ static float to_f(float x) { return x; }
  __device__ static float from_f(float x) { return x; }
  __device__ static f32x16 mma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  __device__ static float row(const float* rowp, int s, int h) { return rowp[2 * s + h]; }
  __device__ static float tr_perm(const float* base, int stride, int s, int h, int lane) {
    return base[((s & 3) + 8 * (s >> 2) + 4 * h) * stride + (lane & 31)];
  }
  __device__ static float tr_nat(const float* base, int stride, int s, int h, int lane) {
    return base[(2 * s + h) * stride + (lane & 31)];
  }
  template <int S>
  __device__ static float pack(const f32x16& a) { return a[S]; }
  __device__ static float zero() { return 0.f; }
  __device__ static float load_global(const float* p) { return *p; }
};

// Row padding (in elements) of LDS images.  16-bit: one 16-byte slot, which
// makes the 32-distinct-row ds_read_b128 pattern conflict-free for every
// head size; fp32: one element (odd stride) for the scalar reads.
template <class E> struct Pad { static constexpr int v = 8; };
template <> struct Pad<float> { static constexpr int v = 1; };

// Copy VEC contiguous elements global -> LDS (zero when !valid).
template <class E>
__device__ __forceinline__ void stage_vec(E* dst, const E* src, bool valid) {
  if constexpr (sizeof(E) == 2) {
    s16x8 v = valid ? *reinterpret_cast<const s16x8*>(src) : s16x8{};
    *reinterpret_cast<s16x8*>(dst) = v;     // 16-bit images keep 16-byte aligned rows
  } else {
    f32x4 v = valid ? *reinterpret_cast<const f32x4*>(src) : f32x4{};
    dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2]; dst[3] = v[3];   // odd-stride rows
  }
}

// Store 4 consecutive accumulator values (registers 4g..4g+3) as elements.
template <class E>
__device__ __forceinline__ void store4(E* dst, float a, float b, float c, float d) {
#ifndef DTA_ATTN_NT
#define DTA_ATTN_NT 0          // 1: the attention epilogues' global stores non-temporal
#endif
  if constexpr (sizeof(E) == 2) {
    typedef E v4 __attribute__((ext_vector_type(4)));
    v4 v = {(E)a, (E)b, (E)c, (E)d};
    if constexpr (DTA_ATTN_NT) __builtin_nontemporal_store(v, reinterpret_cast<v4*>(dst));
    else *reinterpret_cast<v4*>(dst) = v;
  } else {
    if constexpr (DTA_ATTN_NT) __builtin_nontemporal_store(f32x4{a, b, c, d}, reinterpret_cast<f32x4*>(dst));
    else *reinterpret_cast<f32x4*>(dst) = f32x4{a, b, c, d};
  }
}

// O_i (obr) elements: fp32, or fp16 (ABI 6, `h`) -- element offsets from the base
__device__ __forceinline__ void store_ob4(void* base, int64_t off, bool h, float a, float b, float c, float d) {
  if (h) store4<_Float16>(reinterpret_cast<_Float16*>(base) + off, a, b, c, d);
  else store4<float>(reinterpret_cast<float*>(base) + off, a, b, c, d);
}
__device__ __forceinline__ void load_ob8(const void* base, int64_t off, bool h, float (&o)[8]) {
  if (h) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const h8 v = *reinterpret_cast<const h8*>(reinterpret_cast<const _Float16*>(base) + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (float)v[j];
  } else {
#ifndef DTA_OBR_LOAD_NT
#define DTA_OBR_LOAD_NT 0      // A/B: attn_dq's reads of the fp32 O_i (read once) non-temporal
#endif
    const f32x4* pa = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(base) + off);
    const f32x4 a = DTA_OBR_LOAD_NT ? __builtin_nontemporal_load(pa) : *pa;
    const f32x4 b = DTA_OBR_LOAD_NT ? __builtin_nontemporal_load(pa + 1) : pa[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[j] = a[j]; o[4 + j] = b[j]; }
  }
}

template <class E>
__device__ __forceinline__ void store4_lds(E* dst, float a, float b, float c, float d) {
  if constexpr (sizeof(E) == 2) {
    typedef E v4 __attribute__((ext_vector_type(4)));
    v4 v = {(E)a, (E)b, (E)c, (E)d};
    *reinterpret_cast<v4*>(dst) = v;
  } else {
    dst[0] = a; dst[1] = b; dst[2] = c; dst[3] = d;
  }
}

constexpr float LOG2E = 1.4426950408889634f;

// 32-bit division by a launch constant: q = (umulhi(x, m) + x) >> s, exact for x < 2^31
// (round-up multiplier; the element index of a launch stays below 2^31 on this path)
struct FastDiv {
  uint32_t d, m, s;
  FastDiv() = default;
  explicit FastDiv(uint32_t d_) : d(d_), m(0), s(0) {
    while ((1ull << s) < d) ++s;
    m = (uint32_t)((((1ull << s) - d) << 32) / d + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t x) const { return (__umulhi(x, m) + x) >> s; }
};

}  // namespace dta
