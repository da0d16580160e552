// decode.hip -- one-query-row differential attention over a KV cache, gfx950.
//
// The reference's generate() (diff_transformer.py:177-185, Ndiff_transformer.py
// generate, control.py:163-171) re-runs the whole prefix for every new token.
// With a KV cache only the new token's row of the attention is needed:
//   o = sum_i coef[h][i] * softmax(q_i K_i[0:L]^T * scale) V[0:L]
// This is HBM-bound (each cached K_i / V row is read once per token), so the
// kernel is plain vector code, not MFMA: one workgroup per (b, h), four waves.
//   phase 1  every thread scores whole keys (16-byte K loads, q_i in LDS),
//            scores -> fp32 workspace, per-branch block max
//   phase 2  e = exp(s - m_i) in place, per-branch block sum l_i
//   phase 3  w_j = sum_i coef_i e_ij / l_i (the combined map row)
//   phase 4  o[e] = sum_j w_j V[j][e]: threads own a column, key groups stride
//            (coalesced V rows), LDS reduction over the groups.
// The split-key plan below is the one used for the standard head sizes.
// Algorithmic bytes per (b, h) and token: L * (N*hs + dv) * sizeof(E).
#include "dta_common.h"
#include "dta_internal.h"

namespace dta {

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

#ifndef DTA_DEC_NT
#define DTA_DEC_NT 0       // 1: the K/V cache stream read with non-temporal loads
#endif
template <class E, bool NT = false>
__device__ __forceinline__ void ld8f(const E* p, float* f) {
  if constexpr (sizeof(E) == 2) {
    typedef E v8 __attribute__((ext_vector_type(8)));
    const v8 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const v8*>(p)) : *reinterpret_cast<const v8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
  } else {
    const f32x4* q = reinterpret_cast<const f32x4*>(p);
    const f32x4 a = NT ? __builtin_nontemporal_load(q) : q[0], b = NT ? __builtin_nontemporal_load(q + 1) : q[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { f[j] = a[j]; f[j + 4] = b[j]; }
  }
}

__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide reduction of NB per-thread values (all threads get the result)
template <int NB, bool MAX>
__device__ __forceinline__ void block_reduce(float (&v)[NB], float* red) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const float r = MAX ? wmax(v[i]) : wsum(v[i]);
    if (lane == 0) red[wave * NB + i] = r;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    float r = red[i];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) r = MAX ? fmaxf(r, red[w * NB + i]) : r + red[w * NB + i];
    v[i] = r;
  }
  __syncthreads();
}

// The valid length: the device value when given, clamped to [0, L] (L = the host
// upper bound the grid and workspace were sized for), so a bad device length can
// never index past the cache, the workspace or the combine's LDS weights.
__device__ __forceinline__ int clamp_len(const DecodeParams& p) {
  return p.Ldev ? min(max(*p.Ldev, 0), p.L) : p.L;
}

template <class E, int N>
__global__ __launch_bounds__(kThreads) void decode_kernel(DecodeParams p) {
  __shared__ float qs[N * 128];
  __shared__ float red[kWaves * N];
  __shared__ float part[kThreads];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int HS = p.HS, DV = p.DV, L = clamp_len(p);
  const E* gq = reinterpret_cast<const E*>(p.q.p) + b * p.q.sb + h * p.q.sh;
  for (int x = tid; x < N * HS; x += kThreads) qs[x] = (float)gq[(x / HS) * p.q.si + x % HS];
  __syncthreads();

  float* ws = p.ws + ((int64_t)b * p.H + h) * N * p.ldw;     // [i][ldw]
  const E* gk = reinterpret_cast<const E*>(p.k.p) + b * p.k.sb + h * p.k.sh;
  float m[N];
#pragma unroll
  for (int i = 0; i < N; ++i) m[i] = -INFINITY;
  for (int j = tid; j < L; j += kThreads) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const E* kr = gk + (int64_t)j * p.k.st + i * p.k.si;
      float s = 0.f;
      for (int d = 0; d < HS; d += 8) {
        float f[8];
        ld8f<E>(kr + d, f);
#pragma unroll
        for (int u = 0; u < 8; ++u) s = fmaf(qs[i * HS + d + u], f[u], s);
      }
      s *= p.scale;
      ws[i * p.ldw + j] = s;
      m[i] = fmaxf(m[i], s);
    }
  }
  block_reduce<N, true>(m, red);

  float l[N];
#pragma unroll
  for (int i = 0; i < N; ++i) l[i] = 0.f;
  for (int j = tid; j < L; j += kThreads)
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const float e = __expf(ws[i * p.ldw + j] - m[i]);
      ws[i * p.ldw + j] = e;
      l[i] += e;
    }
  block_reduce<N, false>(l, red);

  float c[N];
#pragma unroll
  for (int i = 0; i < N; ++i) c[i] = p.coef[h * N + i] / l[i];
  for (int j = tid; j < L; j += kThreads) {
    float w = 0.f;
#pragma unroll
    for (int i = 0; i < N; ++i) w = fmaf(c[i], ws[i * p.ldw + j], w);
    ws[j] = w;                                  // row 0 now holds the combined map row
  }
  __threadfence_block();
  __syncthreads();

  // phase 4: G key groups x DV columns
  const int G = kThreads / DV;
  const int g = tid / DV, e = tid % DV;
  const E* gv = reinterpret_cast<const E*>(p.v.p) + b * p.v.sb + h * p.v.sh + e;
  float acc = 0.f;
  if (g < G)
    for (int j = g; j < L; j += G) acc = fmaf(ws[j], (float)gv[(int64_t)j * p.v.st], acc);
  part[tid] = acc;
  __syncthreads();
  if (tid < DV) {
    float o = 0.f;
    for (int x = 0; x < G; ++x) o += part[x * DV + tid];
    E* go = reinterpret_cast<E*>(p.o.p) + b * p.o.sb + h * p.o.sh;
    go[tid] = (E)o;
  }
}

// ---- split-key path (flash-decoding): fills the chip when B*H is small ------
// Grid (S, H, B): workgroup s owns keys [s*kChunk, (s+1)*kChunk).  It writes,
// per branch i, the chunk's max m_i, sum l_i = sum_j exp(s_ij - m_i) and the
// un-normalised row acc_i = sum_j exp(s_ij - m_i) V_j (fp32).  decode_combine
// rescales the S partials to the global max and applies coef_i / L_i.
// K rows are read by LPR = HS/8 lanes each (one 16-byte load per lane), V rows
// by DV/8 lanes each, so every wave-level load is a run of whole rows.
// kChunk: keys per split workgroup.  DTA_DECODE_CHUNK (256) sizes the workspace
// (the most splits); launches with >= kWideGrid workgroups use 2x chunks, which
// halves the partials (A/B: +4.5% at B=8 H=16 L=32768, slower on smaller grids)
constexpr int kWideGrid = 8192;

template <class E, int N, int HS, int DV, int kChunk>
__global__ __launch_bounds__(kThreads) void decode_split_kernel(DecodeParams p) {
  constexpr int LPR = HS / 8;                 // lanes per K row
  constexpr int KPW = 64 / LPR;               // keys per wave per load
  constexpr int VPR = DV / 8;                 // lanes per V row
  constexpr int G = kThreads / VPR;           // V row groups
  constexpr int KPT = kChunk / kThreads;      // keys per thread in the softmax phase
  static_assert(kChunk % kThreads == 0, "chunk must be a multiple of the workgroup");
  __shared__ float sc[N][kChunk];
  __shared__ float red[kWaves * N];
  __shared__ float part[G][N][DV + 4];
  const int s = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = s * kChunk, L = clamp_len(p);
  if (j0 >= L) return;                         // grid sized for an upper bound (uniform exit)
  const int nk = min(kChunk, L - j0);

  // phase 1: scores of this chunk into LDS
  {
    const int sub = lane % LPR, kr = lane / LPR;
    const E* gq = reinterpret_cast<const E*>(p.q.p) + b * p.q.sb + h * p.q.sh + sub * 8;
    float q[N][8];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      ld8f<E>(gq + i * p.q.si, q[i]);
#pragma unroll
      for (int u = 0; u < 8; ++u) q[i][u] *= p.scale;
    }
    const E* gk = reinterpret_cast<const E*>(p.k.p) + b * p.k.sb + h * p.k.sh + sub * 8;
    for (int jj = wave * KPW + kr; jj < kChunk; jj += kWaves * KPW) {
      const bool ok = jj < nk;
      const E* kp = gk + (int64_t)(j0 + (ok ? jj : 0)) * p.k.st;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        float f[8];
        ld8f<E, DTA_DEC_NT>(kp + i * p.k.si, f);
        float d = 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) d = fmaf(q[i][u], f[u], d);
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
        if (sub == 0) sc[i][jj] = ok ? d : -INFINITY;
      }
    }
  }
  __syncthreads();

  // phase 2: chunk max / exp / sum per branch (thread = key)
  float m[N], l[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    m[i] = sc[i][tid];
#pragma unroll
    for (int r = 1; r < KPT; ++r) m[i] = fmaxf(m[i], sc[i][tid + r * kThreads]);
  }
  block_reduce<N, true>(m, red);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    l[i] = 0.f;
#pragma unroll
    for (int r = 0; r < KPT; ++r) {
      const int j = tid + r * kThreads;
      const float e = j < nk ? __expf(sc[i][j] - m[i]) : 0.f;
      sc[i][j] = e;
      l[i] += e;
    }
  }
  block_reduce<N, false>(l, red);        // its barriers also publish sc

  // phase 3: acc_i = sum_j e_ij V_j (thread = 8 columns of one row group)
  const int g = tid / VPR, c0 = (tid % VPR) * 8;
  const E* gv = reinterpret_cast<const E*>(p.v.p) + b * p.v.sb + h * p.v.sh + c0;
  float acc[N][8];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[i][u] = 0.f;
  for (int jj = g; jj < nk; jj += G) {
    float f[8];
    ld8f<E, DTA_DEC_NT>(gv + (int64_t)(j0 + jj) * p.v.st, f);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const float e = sc[i][jj];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[i][u] = fmaf(e, f[u], acc[i][u]);
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int u = 0; u < 8; ++u) part[g][i][c0 + u] = acc[i][u];
  __syncthreads();
  const int64_t row = ((int64_t)b * p.H + h) * p.S + s;      // partial index
  float* wacc = p.ws + row * N * DV;
  for (int x = tid; x < N * DV; x += kThreads) {
    const int i = x / DV, c = x % DV;
    float a = 0.f;
#pragma unroll
    for (int gg = 0; gg < G; ++gg) a += part[gg][i][c];
    wacc[x] = a;
  }
  if (tid < N) {
    p.ml[row * N * 2 + tid * 2] = m[tid];
    p.ml[row * N * 2 + tid * 2 + 1] = l[tid];
  }
}

constexpr int kMaxPartials = 2048;            // S * N per (b, h) for the combine's LDS weights

template <class E, int N, int kChunk>
__global__ __launch_bounds__(kThreads) void decode_combine_kernel(DecodeParams p) {
  __shared__ float wgt[kMaxPartials];          // [s][i] = coef_i / L_i * exp(m_is - M_i)
  __shared__ float red[kWaves * N];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int64_t row0 = ((int64_t)b * p.H + h) * p.S;       // partial stride: the launch's S
  const int S = min((clamp_len(p) + kChunk - 1) / kChunk, p.S);  // chunks written this call
  const float* ml = p.ml + row0 * N * 2;
  float M[N], Ls[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    M[i] = -INFINITY;
    for (int s = tid; s < S; s += kThreads) M[i] = fmaxf(M[i], ml[s * N * 2 + i * 2]);
  }
  block_reduce<N, true>(M, red);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    Ls[i] = 0.f;
    for (int s = tid; s < S; s += kThreads) {
      const float e = __expf(ml[s * N * 2 + i * 2] - M[i]);
      wgt[s * N + i] = e;
      Ls[i] += ml[s * N * 2 + i * 2 + 1] * e;
    }
  }
  block_reduce<N, false>(Ls, red);             // barriers also publish wgt
  E* go = reinterpret_cast<E*>(p.o.p) + b * p.o.sb + h * p.o.sh;
  const float* a = p.ws + row0 * N * p.DV;
  float c[N];
#pragma unroll
  for (int i = 0; i < N; ++i) c[i] = p.coef[h * N + i] / Ls[i];
  for (int col = tid; col < p.DV; col += kThreads) {
    float o = 0.f;
#pragma unroll 4
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int i = 0; i < N; ++i) o = fmaf(c[i] * wgt[s * N + i], a[((int64_t)s * N + i) * p.DV + col], o);
    go[col] = (E)o;
  }
}

// Chunk size is chosen from the cache capacity (ldw = t_cap), not from the
// current length, so the eager path (length = pos + 1) and the graph path
// (length = t_cap, device length) launch the same chunks and reduce in the same
// order: their outputs are bitwise equal at every position.
template <class E, int N, int HS, int DV>
int split_launch(const DecodeParams& p0, hipStream_t st) {
  constexpr int C = DTA_DECODE_CHUNK;
  const int64_t s_cap = (p0.ldw + C - 1) / C;
  const bool wide = s_cap * p0.H * p0.B >= kWideGrid;
  const int chunk = wide ? 2 * C : C;
  // the combine keeps one LDS weight per (chunk, branch): gate on the chunk actually launched
  if (((int64_t)p0.ldw + chunk - 1) / chunk * N > kMaxPartials) return 1;
  DecodeParams p = p0;
  p.S = (p0.L + chunk - 1) / chunk;            // same partial layout as C-key chunks, fewer rows used
  if (wide) {
    hipLaunchKernelGGL((decode_split_kernel<E, N, HS, DV, 2 * C>), dim3(p.S, p.H, p.B), dim3(kThreads), 0, st, p);
    hipLaunchKernelGGL((decode_combine_kernel<E, N, 2 * C>), dim3(p.H, p.B), dim3(kThreads), 0, st, p);
  } else {
    hipLaunchKernelGGL((decode_split_kernel<E, N, HS, DV, C>), dim3(p.S, p.H, p.B), dim3(kThreads), 0, st, p);
    hipLaunchKernelGGL((decode_combine_kernel<E, N, C>), dim3(p.H, p.B), dim3(kThreads), 0, st, p);
  }
  return (int)hipGetLastError();
}

template <class E, int N>
int split_dispatch(const DecodeParams& p, hipStream_t st) {
  if (p.HS == 32 && p.DV == 64) return split_launch<E, N, 32, 64>(p, st);
  if (p.HS == 64 && p.DV == 128) return split_launch<E, N, 64, 128>(p, st);
  if (p.HS == 128 && p.DV == 256) return split_launch<E, N, 128, 256>(p, st);
  if (N == 1 && p.HS == 64 && p.DV == 64) return split_launch<E, N, 64, 64>(p, st);
  if (N == 1 && p.HS == 128 && p.DV == 128) return split_launch<E, N, 128, 128>(p, st);
  return 1;    // no split plan: caller uses the single-pass kernel
}

template <class E>
int decode_launch(const DecodeParams& p, hipStream_t st) {
  if (p.ml) {
    int e = 1;
    switch (p.N) {
      case 1: e = split_dispatch<E, 1>(p, st); break;
      case 2: e = split_dispatch<E, 2>(p, st); break;
      case 3: e = split_dispatch<E, 3>(p, st); break;
      case 4: e = split_dispatch<E, 4>(p, st); break;
    }
    if (e != 1) return e;
  }
  dim3 g(p.H, p.B);
  switch (p.N) {
    case 1: hipLaunchKernelGGL((decode_kernel<E, 1>), g, dim3(kThreads), 0, st, p); break;
    case 2: hipLaunchKernelGGL((decode_kernel<E, 2>), g, dim3(kThreads), 0, st, p); break;
    case 3: hipLaunchKernelGGL((decode_kernel<E, 3>), g, dim3(kThreads), 0, st, p); break;
    case 4: hipLaunchKernelGGL((decode_kernel<E, 4>), g, dim3(kThreads), 0, st, p); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

}  // namespace

int launch_decode(int dtype, const DecodeParams& p, hipStream_t st) {
  if ((int64_t)p.B * p.H == 0) return 0;
  switch (dtype) {
    case 0: return decode_launch<__bf16>(p, st);
    case 1: return decode_launch<_Float16>(p, st);
    case 2: return decode_launch<float>(p, st);
  }
  return -2;
}

}  // namespace dta
