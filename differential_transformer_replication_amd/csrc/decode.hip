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
// Algorithmic bytes per (b, h) and token: L * (N*hs + dv) * sizeof(E).
#include "dta_common.h"
#include "dta_internal.h"

namespace dta {

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

template <class E>
__device__ __forceinline__ void ld8f(const E* p, float* f) {
  if constexpr (sizeof(E) == 2) {
    typedef E v8 __attribute__((ext_vector_type(8)));
    const v8 v = *reinterpret_cast<const v8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
  } else {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
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

template <class E, int N>
__global__ __launch_bounds__(kThreads) void decode_kernel(DecodeParams p) {
  __shared__ float qs[N * 128];
  __shared__ float red[kWaves * N];
  __shared__ float part[kThreads];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int HS = p.HS, DV = p.DV, L = p.L;
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

template <class E>
int decode_launch(const DecodeParams& p, hipStream_t st) {
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
