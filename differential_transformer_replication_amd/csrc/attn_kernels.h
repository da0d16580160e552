// attn_kernels.h -- fused N-branch causal differential attention, gfx950.
//
//   O = sum_i c[h][i] * softmax_causal(Q_i K_i^T * scale) V        (all heads)
//
// Replaces DiffHead/MultiHeadDiffAttention's per-head eager loop
// (diff_transformer.py:57-72, 89) and AlternatingDiffHead's branch loop
// (Ndiff_transformer.py:102-125).  Three kernels, all flash-style loops whose
// tiles arrive in LDS by LDS-DMA (global_load_lds, one 1 KiB piece per wave
// instruction) into double buffers, so the next tile streams in while MFMAs
// consume the current one:
//
//  attn_fwd   query-major.  Workgroup = NW waves x 32 query rows of one
//             (b, h, dv-chunk).  Scores transposed (S^T = K Q^T: key in
//             registers, query on the lane) so each query row's online
//             softmax lives in one lane pair and P^T is directly the B operand
//             of O^T += V^T P^T.  V^T comes from the row-major V tile through
//             ds_read_b64_tr_b16.  Writes O, the per-branch normalised O_i and
//             the per-branch log2-sum-exp.
//  attn_dq    query-major backward for dQ (no atomics):
//             S^T_i = K_i Q_i^T, dP^T = V dO^T, dS^T_i = c_i P^T_i (dP^T - delta_i),
//             dQ_i^T += K_i^T dS^T_i.  Also computes delta_i = <dO, O_i> per row
//             (written for attn_dkdv) and d(coef) = sum delta_i.
//  attn_dkdv  key-major backward: S_i = Q_i K_i^T, dP = dO V^T (key on the lane),
//             dK_i^T += Q_i^T dS_i, dV^T += dO^T (sum_i c_i P_i).
//
// LDS images are rows of 16-byte chunks with an XOR swizzle (swz<ROWB>) that
// makes both access kinds conflict-free: 32-distinct-row ds_read_b128 operand
// reads and 4-row x 32-column ds_read_b64_tr_b16 transposed reads.  LDS-DMA
// writes lane-linearly, so the swizzle is applied to the per-lane SOURCE
// address and to every read (cdna_hip_programming.md rule 21).
#pragma once
#include "dta_common.h"
#include "dta_internal.h"

#include <type_traits>
#include <utility>

#ifndef DTA_STAMPS
#define DTA_STAMPS 0
#endif

namespace dta {

// In-kernel cycle stamps (diagnostic builds, -DDTA_STAMPS=1; cdna_hip_programming.md
// 7 'In-kernel stamps'): per-wave sums of the cycles between named points of the
// tile loop, written once per wave to FwdParams/BwdParams::stamps.  The stamp's own
// lgkmcnt(0) serialises LDS reads, so a stamped build is read for its SHARES only.
template <int NSEG_ = 8>
struct Stamps {
  // 32-bit sums (a wave's segment totals stay far below 2^32 cycles), and fewer segments
  // where SGPRs are short: 8 64-bit sums cost the dK/dV plan enough SGPRs to spill its DMA
  // offsets to scratch, which then serialised every LDS-DMA issue behind a scratch reload
  // and inflated its 'dma_issue' share (round 6)
  static constexpr int NSEG = NSEG_;
  unsigned t = 0, s[NSEG] = {};
  __device__ __forceinline__ static unsigned now() {
    unsigned long long v;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : : "memory");
    __builtin_amdgcn_sched_barrier(0);
    return (unsigned)v;
  }
  __device__ __forceinline__ void start() { if constexpr (DTA_STAMPS) t = now(); }
  template <int J>
  __device__ __forceinline__ void lap() {
    if constexpr (DTA_STAMPS) {
      const unsigned n = now();
      s[J] += n - t;
      t = n;
    }
  }
  __device__ __forceinline__ void flush(unsigned long long* out, int wave_id, int lane) {
    if constexpr (DTA_STAMPS) {
      if (out && lane == 0)
#pragma unroll
        for (int j = 0; j < 8; ++j) out[(int64_t)wave_id * 8 + j] = j < NSEG ? s[j] : 0;
    }
  }
};

// ------------------------------------------------------------ LDS images ---
// Image width for a logical width: LDS rows keep a power-of-two pitch (the XOR
// swizzle's domain), so head size 96 / value width 192 live in 128 / 256-column rows
// whose pad columns are staged but never read.
constexpr int img_cols(int c) {
  int p = 1;
  while (p < c) p <<= 1;
  return p;
}

template <int ROWB>
__device__ __forceinline__ int swz(int r) {
  if constexpr (ROWB >= 256) return ((r & 3) << 2) | ((r >> 2) & 3);
  else if constexpr (ROWB == 128) return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
  else if constexpr (ROWB == 64) return (r >> 2) & 3;
  else return (r >> 3) & 1;
}

template <class E, int COLS>
struct Img {
  static constexpr int ES = (int)sizeof(E);
  static constexpr int ROWB = COLS * ES;
  static constexpr int CPR = ROWB / 16;
  static_assert(ROWB >= 32 && (ROWB & (ROWB - 1)) == 0, "image rows must be a power of two >= 32 B");
  __device__ static int off(int r, int col) {   // element offset of (r, col)
    const int byte = col * ES;
    return (r * ROWB + ((((byte >> 4) ^ swz<ROWB>(r)) << 4) | (byte & 15))) / ES;
  }
  using O = Ops<E>;
  using frag = typename O::frag;
  // operand fragment of k-step s: row r, k = s*KSTEP + h*KH (+0..KH-1)
  __device__ static frag row(const E* img, int r, int s, int h) {
    if constexpr (ES == 2) return *reinterpret_cast<const frag*>(img + off(r, s * 16 + h * 8));
    else return img[off(r, 2 * s + h)];
  }
  // 4 rows r0..r0+3 x 16 columns per 16-lane group (ds_read_b64_tr_b16)
  template <class V4>
  __device__ static V4 tr4(const E* img, int r0, int cbase, int lane) {
    const int i = lane & 15;
    const E* p = img + off(r0 + (i >> 2), cbase + ((lane >> 4) & 1) * 16 + (i & 3) * 4);
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
    return __builtin_bit_cast(V4, v);
  }
  // transposed operand, k order matching an accumulator packed by pack<s>():
  // element j <-> row rbase + 16s + 8(j>>2) + 4h + (j&3), column cbase + (lane&31)
  __device__ static frag tr_perm(const E* img, int rbase, int s, int h, int cbase, int lane) {
    if constexpr (ES == 2) {
      typedef E v4 __attribute__((ext_vector_type(4)));
      v4 lo = tr4<v4>(img, rbase + 16 * s + 4 * h, cbase, lane);
      v4 hi = tr4<v4>(img, rbase + 16 * s + 8 + 4 * h, cbase, lane);
      return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    } else {
      return img[off(rbase + (s & 3) + 8 * (s >> 2) + 4 * h, cbase + (lane & 31))];
    }
  }
};

// Gradient through RoPE (Ndiff_transformer.py:11-22 backward), fused into the dQ / dK
// epilogues: the kernels differentiate w.r.t. the ROTATED Q_i / K_i, and the
// parameters' gradient is the conjugate rotation of that.  Registers 4g..4g+3 of a
// lane hold columns e..e+3 (e % 4 == 0) of one row: two interleaved pairs, whose
// [cos, sin] entries are 4 consecutive floats of the fp32 [T][hs/2][2] table.
__device__ __forceinline__ void rope_inv4(const float* rope, int64_t row, int hs, int e, float& a0, float& a1,
                                          float& a2, float& a3) {
  const f32x4 t = *reinterpret_cast<const f32x4*>(rope + (row * (hs >> 1) + (e >> 1)) * 2);
  const float b0 = fmaf(a0, t[0], a1 * t[1]), b1 = fmaf(a1, t[0], -a0 * t[1]);
  const float b2 = fmaf(a2, t[2], a3 * t[3]), b3 = fmaf(a3, t[2], -a2 * t[3]);
  a0 = b0; a1 = b1; a2 = b2; a3 = b3;
}

// Attention dropout (nn.Dropout on every softmax map, diff_transformer.py:66-67,
// Ndiff_transformer.py:114): element (q, k) of branch i of head h, batch b, is kept
// iff hash(b, h, i, q, k, seed) >= p * 2^32, and kept elements are scaled by 1/(1-p).
// The hash is counter-based (no state), so the forward and both backward kernels --
// and the tests' torch restatement -- regenerate the same mask from the seed.
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_key(uint32_t seed_lo, uint32_t seed_hi, int b, int h, int i, int H, int N) {
  return fmix32(seed_lo ^ fmix32((uint32_t)((b * H + h) * N + i) + seed_hi));
}
__device__ __forceinline__ float drop_mul(uint32_t key, int q, int k, uint32_t thr, float scale) {
  const uint32_t x = fmix32((key + (uint32_t)q * 0x9e3779b1u) ^ ((uint32_t)k * 0x7feb352du));
  return x >= thr ? scale : 0.f;
}

// ---- compile-time loops (asm immediates must be constants, not unrolled loop indices)
template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) { sfor_impl(f, std::make_integer_sequence<int, N>{}); }

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

// 16-bit transposed operand reads, issued by inline asm: the builtin carries no
// alias information, so the compiler guards every one of them with
// s_waitcnt vmcnt(0) -- draining the LDS-DMA ring each tile.  Waits for these
// reads are explicit (lgkm_pin).
//
// Addressing (derived from swz<ROWB>): for the 32-row block at row rbase and
// columns 32d..32d+31, the byte address of lane l's piece of the k-step-s
// fragment half x (x = 0: rows 16s+4h.., x = 1: rows 16s+8+4h..) is
//     (Ltr(l) ^ (64 d + 32 x)) + ROWB * (rbase + 16 s + 8 x)
// so one XOR per (d, x) and DS immediates carry the rest.
template <int ROWB>
__device__ __forceinline__ int tr_lane(int lane) {
  const int h = (lane >> 5) & 1, i = lane & 15, q = i >> 2;
  const int y = ((lane >> 4) & 1) * 2 + ((i & 3) >> 1);
  int L = (4 * h + q) * ROWB + 16 * (y ^ h) + 8 * (i & 1);
  if constexpr (ROWB >= 256) L += 64 * q;
  else if constexpr (ROWB == 128) L += 64 * (q >> 1);
  return L;
}
// operand row reads (ds_read_b128): row c32 of a 32-row block, k-step s:
//     R*ROWB + (Lrow(l) ^ 32 s)
template <int ROWB>
__device__ __forceinline__ int row_lane(int lane) {
  const int c = lane & 31, h = (lane >> 5) & 1;
  return c * ROWB + 16 * (h ^ swz<ROWB>(c));
}

typedef long long lds64;
// two fragments (k-steps s = 0, 1) of a 32x32 transposed operand block
template <int ROWB, int RB, int OFF = 0>
__device__ __forceinline__ void tr_issue(lds64 (&r)[4], unsigned a0, unsigned a1) {
  static_assert(OFF + ROWB * (RB + 24) < 65536, "DS immediate offset");
  asm volatile(
      "ds_read_b64_tr_b16 %0, %4 offset:%6\n\t"
      "ds_read_b64_tr_b16 %1, %5 offset:%7\n\t"
      "ds_read_b64_tr_b16 %2, %4 offset:%8\n\t"
      "ds_read_b64_tr_b16 %3, %5 offset:%9"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
      : "v"(a0), "v"(a1), "i"(OFF + ROWB * RB), "i"(OFF + ROWB * (RB + 8)), "i"(OFF + ROWB * (RB + 16)),
        "i"(OFF + ROWB * (RB + 24)));
}
// LDS byte address -> pointer; a constant added to the pointer (not to the address)
// folds into the DS instruction's immediate offset
__device__ __forceinline__ const __attribute__((address_space(3))) char* lds_ptr(unsigned a) {
  return reinterpret_cast<const __attribute__((address_space(3))) char*>((size_t)a);
}
template <class T>
__device__ __forceinline__ T lds_at(unsigned a, int off) {
  return *reinterpret_cast<const __attribute__((address_space(3))) T*>(lds_ptr(a) + off);
}
// retire every outstanding LDS read, then pin the asm results so no use of
// them can be scheduled above the wait (cdna_hip_programming.md 5.7 item 1)
template <int M>
__device__ __forceinline__ void lgkm_pin(lds64 (&r)[M][4]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(r[m][j]));
}
// Software-pipelined operand reads: ds_read_b128 by inline asm (invisible to the
// compiler's waitcnt pass) and counted waits.  lgkmcnt(N) with N = the number of OUR reads
// issued after the one being consumed is exact whatever else the compiler interleaves:
// LDS returns in order, so any other LDS / SMEM op only makes the wait longer.
typedef int i32x4 __attribute__((ext_vector_type(4)));
template <int OFF>
__device__ __forceinline__ void ds128(i32x4& r, unsigned a) {
  static_assert(OFF >= 0 && OFF < 65536, "DS immediate offset");
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
}
template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
}

// One score chain S[kb] += K[kb] Q^T over NSQ k-steps (32-row key blocks kb < NKB, K rows as
// the A operand) with every operand read D reads ahead of its MFMA.  Per k-step s: the Q
// fragment (QL: from LDS at bQ ^ 32 s + QOFF, else qreg[s]) then the NKB K fragments
// (bK ^ 32 s + KOFF + kb * 32 * KROWB).  bK / bQ: lane bases whose bits 5..6 are the lane's
// own (the XOR applies to them; the region offsets ride in DS immediates).
template <class E, int NSQ, int NKB, int QL, int D, int KOFF, int QOFF, int KROWB>
__device__ __forceinline__ void s_chain_pipe(f32x16 (&sa)[NKB], unsigned bK, unsigned bQ,
                                             const typename Ops<E>::frag* qreg) {
  using frag = typename Ops<E>::frag;
  constexpr int PER = NKB + QL, NR = NSQ * PER;
  // region offsets past the 16-bit DS immediate go into the base (they are multiples of a
  // tile, so the k-step XOR still applies after the add)
  constexpr bool KBIG = KOFF + NKB * 32 * KROWB >= 65536, QBIG = QOFF + 1024 >= 65536;
  bK += KBIG ? KOFF : 0;
  bQ += QBIG ? QOFF : 0;
  i32x4 kr[D + 1], qv[QL ? NSQ : 1];
  auto issue = [&](auto J) {
    constexpr int j = decltype(J)::value, st = j / PER, w = j % PER;
    if constexpr (QL && w == 0) ds128<(QBIG ? 0 : QOFF)>(qv[QL ? st : 0], bQ ^ (32 * st));
    else ds128<(KBIG ? 0 : KOFF) + (w - QL) * 32 * KROWB>(kr[(st * NKB + w - QL) % (D + 1)], bK ^ (32 * st));
  };
  sfor<(D < NR ? D : NR)>([&](auto J) { issue(J); });
  sfor<NSQ * NKB>([&](auto C) {
    constexpr int c = decltype(C)::value, st = c / NKB, kb = c % NKB;
    constexpr int j = st * PER + QL + kb;                                   // this K fragment's read
    constexpr int from = c == 0 ? D : ((c - 1) / NKB) * PER + QL + (c - 1) % NKB + D + 1;
    sfor<NR>([&](auto J2) {                                                   // reads (from, j + D]
      constexpr int j2 = decltype(J2)::value;
      if constexpr (j2 >= from && j2 <= j + D) issue(std::integral_constant<int, j2>{});
    });
    constexpr int issued = (j + D + 1 < NR ? j + D + 1 : NR);
    lgkm_wait<issued - 1 - j>();
    asm volatile("" : "+v"(kr[c % (D + 1)]));
    frag qb;
    if constexpr (QL) {
      asm volatile("" : "+v"(qv[QL ? st : 0]));
      qb = __builtin_bit_cast(frag, qv[QL ? st : 0]);
    } else {
      qb = qreg[st];
    }
    sa[kb] = Ops<E>::mma(__builtin_bit_cast(frag, kr[c % (D + 1)]), qb, sa[kb]);
  });
}

// lgkm_pin with CNT younger reads left in flight
template <int CNT, int M>
__device__ __forceinline__ void lgkm_pin_n(lds64 (&r)[M][4]) {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(CNT) : "memory");
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(r[m][j]));
}

// tr_issue through the compiler's own ds_read_b64_tr_b16 builtin: its waits are the
// compiler's.  An asm read's destination is "complete" to the compiler the moment the
// asm issues, so in a plan that spills, the register allocator may store or copy that
// destination before the data lands (the round-4 non-finite dQ of the 16-bit head size
// 128 N = 3 plan: 476-508 B/lane of scratch).  Plans that spill read through this
// instead (the builtin makes the compiler guard it with vmcnt(0), draining the ring's
// DMA: the cost of correctness there).
template <int ROWB, int RB, int OFF = 0>
__device__ __forceinline__ void tr_load(lds64 (&r)[4], unsigned a0, unsigned a1) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  auto rd = [](unsigned a) {
    return __builtin_bit_cast(lds64, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        reinterpret_cast<__attribute__((address_space(3))) v4s*>((size_t)a)));
  };
  r[0] = rd(a0 + OFF + ROWB * RB);
  r[1] = rd(a1 + OFF + ROWB * (RB + 8));
  r[2] = rd(a0 + OFF + ROWB * (RB + 16));
  r[3] = rd(a1 + OFF + ROWB * (RB + 24));
}

template <class E>
__device__ __forceinline__ typename Ops<E>::frag tr_frag(const lds64 (&r)[4], int s) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  const v4s lo = __builtin_bit_cast(v4s, r[2 * s]), hi = __builtin_bit_cast(v4s, r[2 * s + 1]);
  return __builtin_bit_cast(typename Ops<E>::frag, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Stage ROWS x COLS elements (rows row0.., clamped to rowmax; only the first
// VALID columns come from memory) into an image.  Whole-row 1 KiB pieces go by
// LDS-DMA; images with padded columns are staged through registers (zero-fill).
template <class E, int COLS, int ROWS, int VALID, int NTHR>
__device__ __forceinline__ void stage(E* img, const E* g, int64_t rs, int row0, int rowmax, int tid) {
  using I = Img<E, COLS>;
  constexpr int BYTES = ROWS * I::ROWB;
  if constexpr (VALID == COLS && BYTES % 1024 == 0) {
    constexpr int NI = BYTES / 1024;
    const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int j0 = 0; j0 < NI; j0 += NTHR / 64) {
      const int j = j0 + wave;
      if (NI % (NTHR / 64) == 0 || j < NI) {
        const int pb = j * 1024 + lane * 16;
        const int r = pb / I::ROWB;
        const int c = ((pb % I::ROWB) >> 4) ^ swz<I::ROWB>(r);
        const int row = min(row0 + r, rowmax);
        const char* src = reinterpret_cast<const char*>(g + (int64_t)row * rs) + c * 16;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(img) + j * 1024),
                                         16, 0, 0);
      }
    }
  } else {
    constexpr int CH = ROWS * I::CPR;
    for (int c = tid; c < CH; c += NTHR) {
      const int r = c / I::CPR, ch = c % I::CPR;
      const int row = row0 + r;
      const bool ok = row <= rowmax && ch * 16 < VALID * I::ES;
      s16x8 v = ok ? *reinterpret_cast<const s16x8*>(reinterpret_cast<const char*>(g + (int64_t)row * rs) + ch * 16)
                   : s16x8{};
      *reinterpret_cast<s16x8*>(reinterpret_cast<char*>(img) + r * I::ROWB + ((ch ^ swz<I::ROWB>(r)) << 4)) = v;
    }
  }
}

// RoPE at load (Ndiff_transformer.py:11-22, 104-109: interleaved pairs, rotation in fp32):
// fr = fp32 [T][HS/2][2] (cos, sin).  rope_frag rotates one operand fragment of query row t
// in registers (column col = the fragment's first k); rope_lds rotates ROWS staged rows of
// an LDS image in place and, with `write`, stores the rotated rows to gout (row stride
// ors) -- the copy the backward reads.
template <class E>
__device__ __forceinline__ void rope_frag(typename Ops<E>::frag& f, const float* fr, int t, int col, int HS, int hf) {
  if constexpr (sizeof(E) == 2) {
    const float* q = fr + ((int64_t)t * (HS / 2) + col / 2) * 2;
    const f32x4 a = *reinterpret_cast<const f32x4*>(q), b = *reinterpret_cast<const f32x4*>(q + 4);
    const float cs[4] = {a[0], a[2], b[0], b[2]}, sn[4] = {a[1], a[3], b[1], b[3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = (float)f[2 * j], y = (float)f[2 * j + 1];
      f[2 * j] = (E)(x * cs[j] - y * sn[j]);
      f[2 * j + 1] = (E)(x * sn[j] + y * cs[j]);
    }
  } else {
    // fp32 fragments: k = 2s + hf, so a pair's two elements sit in lanes l and l ^ 32
    const float* q = fr + ((int64_t)t * (HS / 2) + col / 2) * 2;
    const float c = q[0], sn = q[1];
    const float other = __shfl_xor(f, 32, 64);
    f = hf == 0 ? f * c - other * sn : other * sn + f * c;
  }
}
template <class E, int COLS, int ROWS, int VALID, int NTHR>
__device__ __forceinline__ void rope_lds(E* img, const float* fr, int row0, int T, E* gout, int64_t ors, bool write,
                                         int tid) {
  using I = Img<E, COLS>;
  constexpr int V = 16 / (int)sizeof(E);
  typedef E vec __attribute__((ext_vector_type(V)));
  for (int x = tid; x < ROWS * I::CPR; x += NTHR) {
    const int r = x / I::CPR, ch = x % I::CPR;
    if (ch * V >= VALID) continue;
    const int t = min(row0 + r, T - 1);
    vec* a = reinterpret_cast<vec*>(reinterpret_cast<char*>(img) + r * I::ROWB + ((ch ^ swz<I::ROWB>(r)) << 4));
    vec v = *a;
    const float* q = fr + ((int64_t)t * (VALID / 2) + ch * V / 2) * 2;
#pragma unroll
    for (int j = 0; j < V / 2; ++j) {
      const float c = q[2 * j], sn = q[2 * j + 1];
      const float xx = (float)v[2 * j], yy = (float)v[2 * j + 1];
      v[2 * j] = (E)(xx * c - yy * sn);
      v[2 * j + 1] = (E)(xx * sn + yy * c);
    }
    *a = v;
    if (write && row0 + r < T) *reinterpret_cast<vec*>(gout + (int64_t)(row0 + r) * ors + ch * V) = v;
  }
}

// Multiply n elements of an LDS array by s in place (16 bytes per lane and step; n
// a multiple of 16 / sizeof(E)).  Every thread of the block calls it between barriers.
template <class E, int NTHR>
__device__ __forceinline__ void scale_lds(E* a, int n, float s, int tid) {
  constexpr int V = 16 / (int)sizeof(E);
  typedef E vec __attribute__((ext_vector_type(V)));
  for (int e = tid * V; e < n; e += NTHR * V) {
    vec x = *reinterpret_cast<vec*>(a + e);
#pragma unroll
    for (int j = 0; j < V; ++j) x[j] = (E)((float)x[j] * s);
    *reinterpret_cast<vec*>(a + e) = x;
  }
}

// Per-row fp32 vectors (LSE / delta) of NR rows x N branches by 4-byte LDS-DMA.
// src layout [i][b][h][t]: branch stride bs; dst [i][NR] (padded to 64-float pieces).
template <int N, int NR, int NTHR>
__device__ __forceinline__ void stage_rows(float* dst, const float* src, int64_t bs, int row0, int rowmax, int tid) {
  constexpr int TOT = N * NR;
  constexpr int NI = (TOT + 63) / 64;
  const int wave = tid >> 6, lane = tid & 63;
  for (int j = wave; j < NI; j += NTHR / 64) {
    const int e = j * 64 + lane;
    const int i = min(e / NR, N - 1), r = e % NR;
    const float* s = src + i * bs + min(row0 + r, rowmax);
    __builtin_amdgcn_global_load_lds(s, (__attribute__((address_space(3))) void*)(dst + j * 64), 4, 0, 0);
  }
}

// LDS-DMA pieces one wave issues for a stage<> / stage_rows<> call (its j loop)
template <int NI, int NW>
__device__ __forceinline__ int pieces(int wave) { return NI / NW + (wave < NI % NW ? 1 : 0); }
template <class E, int COLS, int ROWS, int VALID, int NW>
__device__ __forceinline__ int stage_pieces(int wave) {
  constexpr int BYTES = ROWS * Img<E, COLS>::ROWB;
  if constexpr (VALID == COLS && BYTES % 1024 == 0) return pieces<BYTES / 1024, NW>(wave);
  else return 0;                  // register path: its loads are retired by the LDS writes
}
template <int N, int NR, int NW>
__device__ __forceinline__ int rows_pieces(int wave) { return pieces<(N * NR + 63) / 64, NW>(wave); }

// s_waitcnt vmcnt(n) for a wave-uniform n.  Issued through the builtin (not
// inline asm) so the compiler's wait-count tracking sees it.
__device__ __forceinline__ void wait_vm(int n) {
#define DTA_VM(k) case k: __builtin_amdgcn_s_waitcnt(((k) & 15) | (((k) >> 4) << 14) | (7 << 4) | (15 << 8)); break;
  switch (n) {
    DTA_VM(0) DTA_VM(1) DTA_VM(2) DTA_VM(3) DTA_VM(4) DTA_VM(5) DTA_VM(6) DTA_VM(7) DTA_VM(8) DTA_VM(9)
    DTA_VM(10) DTA_VM(11) DTA_VM(12) DTA_VM(13) DTA_VM(14) DTA_VM(15) DTA_VM(16) DTA_VM(17) DTA_VM(18)
    DTA_VM(19) DTA_VM(20) DTA_VM(21) DTA_VM(22) DTA_VM(23) DTA_VM(24) DTA_VM(25) DTA_VM(26) DTA_VM(27)
    DTA_VM(28) DTA_VM(29) DTA_VM(30) DTA_VM(31)
    default: __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
  }
#undef DTA_VM
}

// Workgroup barrier that retires this wave's LDS reads but leaves LDS-DMA (vmcnt)
// in flight -- __syncthreads() would drain every outstanding DMA.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0) only
  __builtin_amdgcn_s_barrier();
}

// Waves per SIMD a launch can keep resident given its LDS footprint (workgroups
// per CU x waves per workgroup / 4 SIMDs), capped at the 2 the 256-register plans
// target.  Where the LDS already limits a kernel to one wave per SIMD, its launch
// bound says so and the wave gets the whole 512-entry register file (VGPRs +
// AGPRs) instead of spilling at 256.
constexpr int simd_waves(int nw, int bytes) {
  const int w = (160 * 1024 / bytes) * nw / 4;
  return w < 1 ? 1 : (w > 2 ? 2 : w);
}

// Ring depth for a per-tile footprint: as many stages (2..4) as the LDS leaves room for.
constexpr int ring_stages(int fixed_bytes, int tile_bytes) {
  return (fixed_bytes + 4 * tile_bytes <= 160 * 1024) ? 4 : (fixed_bytes + 3 * tile_bytes <= 160 * 1024) ? 3 : 2;
}

// one LDS-DMA piece: SZ bytes per lane from byte voff of the buffer [base, base + bytes)
// (zeros past its end) to lds + SZ * lane.  base, bytes and lds are wave-uniform.
// (The transfer size is a literal in each helper: the host pass of hipcc rejects
// a template-dependent size here.)
__device__ __forceinline__ void buf_lds16(const void* base, uint32_t bytes, char* lds, uint32_t voff) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}
__device__ __forceinline__ void buf_lds4(const void* base, uint32_t bytes, char* lds, uint32_t voff) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)lds, 4, voff, 0, 0, 0);
}

// One key tile of the query-major kernels -- K_i rows ([N][BN][HS] image) and V
// rows ([BN][DVC] image, columns from the V base given) -- by buffer_load ... lds
// with per-tile descriptors; rows past T read as zeros (masked as keys >= T).
// Wave w issues pieces u * NW + w; single-kind slots resolve at compile time.
template <class E, int HS, int N, int DVC, int BN, int NW>
struct KvRing {
  static constexpr int ES = (int)sizeof(E);
  static constexpr int HSP = img_cols(HS), DVP = img_cols(DVC);   // image widths
  static constexpr int KB = BN * HSP * ES, VB = BN * DVP * ES;
  static constexpr int PK = N * KB / 1024, PV = VB / 1024, NPC = PK + PV;
  static constexpr int MYP = (NPC + NW - 1) / NW;
  static constexpr bool ok = ES == 2 && HS >= 32 && KB % 1024 == 0 && VB % 1024 == 0;

  __device__ static int pieces(int wave) { return NPC / NW + (wave < NPC % NW ? 1 : 0); }
  // (pad chunks of a padded image read the row's first chunk: in bounds, never used)
  __device__ static uint32_t offk(int64_t st, int64_t si, int j, int lane) {
    using KI = Img<E, HSP>;
    const int i = j / (KB / 1024), pb = (j % (KB / 1024)) * 1024 + lane * 16;
    const int r = pb / KI::ROWB;
    int c = ((pb % KI::ROWB) >> 4) ^ swz<KI::ROWB>(r);
    if constexpr (HSP != HS) c = c * 16 < HS * ES ? c : 0;
    return (uint32_t)(r * (uint32_t)(st * ES) + (uint32_t)(i * si * ES) + c * 16);
  }
  __device__ static uint32_t offv(int64_t st, int j, int lane) {
    using VI = Img<E, DVP>;
    const int pb = (j - PK) * 1024 + lane * 16;
    const int r = pb / VI::ROWB;
    int c = ((pb % VI::ROWB) >> 4) ^ swz<VI::ROWB>(r);
    if constexpr (DVP != DVC) c = c * 16 < DVC * ES ? c : 0;
    return (uint32_t)(r * (uint32_t)(st * ES) + c * 16);
  }
  // this wave's pieces of one tile, source offsets computed per tile
  __device__ static void issue(const E* gk, int64_t kst, int64_t ksi, const E* gv, int64_t vst, int k0, int T,
                               E* kdst, E* vdst, int wave, int lane) {
    const int rows = max(0, T - k0);           // a tile past T reads (as zeros) nothing
    const E* bk = gk + (int64_t)k0 * kst;
    const E* bv = gv + (int64_t)k0 * vst;
    const uint32_t nk = (uint32_t)rows * (uint32_t)(kst * ES), nv = (uint32_t)rows * (uint32_t)(vst * ES);
    char* kd = reinterpret_cast<char*>(kdst);
    char* vd = reinterpret_cast<char*>(vdst);
    sfor<MYP>([&](auto U) {
      constexpr int u = decltype(U)::value;
      const int j = u * NW + wave;
      if constexpr ((u + 1) * NW <= PK) {
        buf_lds16(bk, nk, kd + j * 1024, offk(kst, ksi, j, lane));
      } else if constexpr (u * NW >= PK && (u + 1) * NW <= NPC) {
        buf_lds16(bv, nv, vd + (j - PK) * 1024, offv(vst, j, lane));
      } else {
        if (j < PK) buf_lds16(bk, nk, kd + j * 1024, offk(kst, ksi, j, lane));
        else if (j < NPC) buf_lds16(bv, nv, vd + (j - PK) * 1024, offv(vst, j, lane));
      }
    });
  }
  // the per-lane source offsets of this wave's pieces are the same for every tile:
  // computed once (VGPRs), a tile then costs only its two descriptors and M0 values
  __device__ static void offsets(int64_t kst, int64_t ksi, int64_t vst, int wave, int lane, uint32_t (&off)[MYP]) {
    sfor<MYP>([&](auto U) {
      constexpr int u = decltype(U)::value;
      const int j = u * NW + wave;
      if constexpr ((u + 1) * NW <= PK) off[u] = offk(kst, ksi, j, lane);
      else if constexpr (u * NW >= PK && (u + 1) * NW <= NPC) off[u] = offv(vst, j, lane);
      else off[u] = j < PK ? offk(kst, ksi, j, lane) : (j < NPC ? offv(vst, j, lane) : 0u);
    });
  }
  // piece u of this wave's share of one tile (a scheduled stream spreads them over its slots)
  template <int u>
  __device__ static void issue_one(const E* gk, int64_t kst, const E* gv, int64_t vst, int k0, int T, E* kdst,
                                   E* vdst, int wave, uint32_t off) {
    const int rows = max(0, T - k0);
    const int j = u * NW + wave;
    if constexpr ((u + 1) * NW <= PK) {
      buf_lds16(gk + (int64_t)k0 * kst, (uint32_t)rows * (uint32_t)(kst * ES), reinterpret_cast<char*>(kdst) + j * 1024, off);
    } else if constexpr (u * NW >= PK && (u + 1) * NW <= NPC) {
      buf_lds16(gv + (int64_t)k0 * vst, (uint32_t)rows * (uint32_t)(vst * ES), reinterpret_cast<char*>(vdst) + (j - PK) * 1024, off);
    } else {
      if (j < PK) buf_lds16(gk + (int64_t)k0 * kst, (uint32_t)rows * (uint32_t)(kst * ES), reinterpret_cast<char*>(kdst) + j * 1024, off);
      else if (j < NPC) buf_lds16(gv + (int64_t)k0 * vst, (uint32_t)rows * (uint32_t)(vst * ES), reinterpret_cast<char*>(vdst) + (j - PK) * 1024, off);
    }
  }
  __device__ static void issue_pre(const E* gk, int64_t kst, const E* gv, int64_t vst, int k0, int T, E* kdst,
                                   E* vdst, int wave, const uint32_t (&off)[MYP]) {
    const int rows = max(0, T - k0);
    const E* bk = gk + (int64_t)k0 * kst;
    const E* bv = gv + (int64_t)k0 * vst;
    const uint32_t nk = (uint32_t)rows * (uint32_t)(kst * ES), nv = (uint32_t)rows * (uint32_t)(vst * ES);
    char* kd = reinterpret_cast<char*>(kdst);
    char* vd = reinterpret_cast<char*>(vdst);
    sfor<MYP>([&](auto U) {
      constexpr int u = decltype(U)::value;
      const int j = u * NW + wave;
      if constexpr ((u + 1) * NW <= PK) {
        buf_lds16(bk, nk, kd + j * 1024, off[u]);
      } else if constexpr (u * NW >= PK && (u + 1) * NW <= NPC) {
        buf_lds16(bv, nv, vd + (j - PK) * 1024, off[u]);
      } else {
        if (j < PK) buf_lds16(bk, nk, kd + j * 1024, off[u]);
        else if (j < NPC) buf_lds16(bv, nv, vd + (j - PK) * 1024, off[u]);
      }
    });
  }
};

// K/V descriptors cover [row base, T rows): every branch's K columns inside one
// row stride, V's DV columns too, extents within the 32-bit record count.
template <class P>
inline bool kv_layout_ok(const P& p, int es) {
  const int64_t ks = p.k.st, vs = p.v.st;
  if (ks <= 0 || vs <= 0 || p.k.si < 0) return false;
  if ((int64_t)(p.N - 1) * p.k.si + p.HS > ks || p.DV > vs) return false;
  return (int64_t)p.T * ks * es < (1ll << 31) && (int64_t)p.T * vs * es < (1ll << 31);
}

// Row constants as an extra MFMA k-step (bf16, no dropout): each query row's constants
// ride in the score and dP chains instead of one VALU op per element.  A = a "ones"
// fragment (k = 0, 1 set), B = the row's constant split into two bf16 halves (hi, lo:
// 16 significant bits), so every accumulator starts at that constant:
//   S'_i = (sl2 Q_i) K_i^T - LSE_i      (Q_i pre-scaled by sl2 once per workgroup)
//   dP'  = dO V^T - delta_0
// P_i = exp2(S'_i) with no fma; dS_0 / c_0 = P_0 dP', dS_i / c_i = P_i (dP' + delta_0 -
// delta_i); c_i and the softmax scale are applied once in the dQ epilogue.
#ifndef DTA_FWD_IGLP
#define DTA_FWD_IGLP -1          // A/B: __builtin_amdgcn_iglp_opt(k) in the tile loop (-1 = off); k = 0: no effect on any kernel (r06u), 1: compiler out of memory
#endif
#ifndef DTA_DQ_IGLP
#define DTA_DQ_IGLP -1
#endif
#ifndef DTA_DKDV_IGLP
#define DTA_DKDV_IGLP -1
#endif
#ifndef DTA_DQ_SEED
#define DTA_DQ_SEED 1
#endif
#ifndef DTA_DQ_PIPE
#define DTA_DQ_PIPE 3
#endif
#ifndef DTA_FWD_PIPE
#define DTA_FWD_PIPE 3
#endif
#ifndef DTA_FWD_TR_EARLY
#define DTA_FWD_TR_EARLY 0       // A/B: the forward's first d-block V^T reads issued before the last softmax
#endif
#ifndef DTA_FWD_SEED
#define DTA_FWD_SEED 0           // A/B: forward Q_i pre-scaled by scale*log2e, S seeded with -m by one MFMA (FAST tiles): r06e cfg2 fwd 0.874 -> 0.854 ms, but the bf16 Q*scale rounding moved the forward LSE / O_i off the backward kernels and broke the d(coef) / large-logit bars (r06f): off
#endif
#ifndef DTA_FWD_PK
#define DTA_FWD_PK 0             // A/B: the forward's exp arguments and row sums as packed fp32 pairs (v_pk_*): 161 -> 102 VALU issues, fwd +0.3..0.7% (r06p2): off
#endif
#ifndef DTA_FWD_FAST
#define DTA_FWD_FAST 1
#endif
#ifndef DTA_DKDV_FUSE1
#define DTA_DKDV_FUSE1 1
#endif
template <class E>
__device__ __forceinline__ typename Ops<E>::frag seed_frag(float v, int hf) {
  typename Ops<E>::frag f = Ops<E>::zero();
  const E hi = (E)v;
  const E lo = (E)(v - (float)hi);
  if (hf == 0) { f[0] = hi; f[1] = lo; }
  return f;
}

// ---------------------------------------------------------------- forward ---
// Paired workgroups: 4-wave workgroups sized to 80 KB of LDS, two per CU, so the two
// waves sharing a SIMD belong to different workgroups (different barriers) instead of
// one 8-wave workgroup whose SIMD partners run in lockstep (MI355X_MICROARCH.md, two
// waves per SIMD).  cfg2: dK/dV 1.499 -> 1.406 ms; forward / dQ with branch 0's Q rows
// in registers and 64-key tiles: fwd 1.004 -> 0.978, dQ 1.115 -> 1.013 ms.
constexpr int ring_stages_lim(int fixed_bytes, int tile_bytes, int lim) {
  return (fixed_bytes + 4 * tile_bytes <= lim) ? 4 : (fixed_bytes + 3 * tile_bytes <= lim) ? 3 : 2;
}

template <class E> struct FwdTile { static constexpr int BN = 64; };
template <> struct FwdTile<float> { static constexpr int BN = 32; };

// dv chunk per forward workgroup: keep N * DVC/2 accumulator VGPRs <= 128
// N * dv / 2 <= this many accumulator VGPRs: one workgroup takes the whole dv
constexpr int kFwdFullDv = 192;
template <int N, int DV, bool B16 = true>
struct FwdChunk {
  // 16-bit: N = 3 at dv = 128 takes the whole dv in one (one-wave-per-SIMD) workgroup
  // instead of two dv chunks that each redo QK^T and the softmax (fwd 0.523 -> 0.470 ms
  // at cfg3's shape); N = 4 spills that way
  static constexpr int cap = (B16 && N * DV / 2 <= kFwdFullDv) ? DV : (256 / N) / 32 * 32;
  static constexpr int DVC = DV <= cap ? DV : (cap >= 128 && DV % 128 == 0 ? 128 : (cap >= 64 ? 64 : 32));
};

#ifndef DTA_EPI_SKIP
#define DTA_EPI_SKIP 0           // measurement only (wrong results): 1 skips the attention kernels' output stores, 2 the forward's O_i stores
#endif
#ifndef DTA_FWD_BN32
#define DTA_FWD_BN32 0           // A/B: the paired forward plans with 32-key tiles
#endif
template <class E, int HS, int N, int DVC, int NW, bool QREG, int QRH = 0>
struct FwdCfg {
  // QRH > 0 (paired plan): the first QRH branches' Q rows stay in registers
  static constexpr bool PAIR = NW == 4 && !QREG && sizeof(E) == 2 && N * DVC / 2 <= 128;
  static constexpr int BN = (PAIR && (QRH == 0 || DTA_FWD_BN32)) ? 32 : FwdTile<E>::BN;
  static constexpr int BM = NW * 32;
  static constexpr int HSP = img_cols(HS), DVP = img_cols(DVC);     // LDS image widths
  static constexpr int nQ = QREG ? 0 : (N - QRH) * BM * HSP;
  static constexpr int nK = N * BN * HSP;
  static constexpr int nV = BN * DVP;
  static constexpr int NS = ring_stages_lim(nQ * (int)sizeof(E), (nK + nV) * (int)sizeof(E),
                                            PAIR ? 80 * 1024 : 160 * 1024);
  static constexpr int bytes = (nQ + NS * nK + NS * nV) * (int)sizeof(E);
  // rough VGPR count (accumulators, two key blocks of scores, P, Q fragments,
  // addresses); a plan that fits 256 keeps the two-waves-per-SIMD bound
  static constexpr int regs = N * DVC / 2 + N * 2 * 16 + N * 8 + (QREG ? N : QRH) * HS / 4 + 48;
  static constexpr int WPE = regs <= 256 ? 2 : simd_waves(NW, bytes);
};

// NP: no paired plan (the dropout instantiations: their extra registers spill it)
// Single-branch plans (the branch-split forward's workgroups, the control model) take the
// paired layout too: Q in registers, 64-key tiles, two 4-wave workgroups per CU instead of
// one 8-wave workgroup whose SIMD partners run in lockstep.  One-process A/B
// (profiles/r05c_ab_pair_n1.json, outputs bitwise equal): cfg3 N = 3 forward 0.398 ->
// 0.369 ms, N = 4 0.506 -> 0.484; control hs 64 forward 0.222 -> 0.199, dQ 0.273 -> 0.252;
// control hs 128 (cfg5) dQ 11.36 -> 10.73 ms but forward 8.60 -> 8.79, so the head size 128
// forward keeps the 8-wave plan.  DTA_PAIR_N1 = 0 (A/B builds) keeps 8 waves everywhere.
#ifndef DTA_PAIR_N1
#define DTA_PAIR_N1 1
#endif
template <class E, int HS, int N, int DV = 2 * HS, bool NP = false>
struct FwdPick {
  static constexpr int DVC = FwdChunk<N, DV, sizeof(E) == 2>::DVC;
  static constexpr int LIM = 160 * 1024;
  static constexpr int NWMAX = sizeof(E) == 2 ? 8 : 4;
  // widest workgroup with Q in LDS, else Q in registers
  // an 8-wave plan past ~280 registers spills at two waves per SIMD: take 4 waves
  static constexpr bool q8 = NWMAX >= 8 && FwdCfg<E, HS, N, DVC, 8, false>::bytes <= LIM &&
                             FwdCfg<E, HS, N, DVC, 8, false>::regs <= 280;
  static constexpr bool q4 = FwdCfg<E, HS, N, DVC, 4, false>::bytes <= LIM;
  // paired 4-wave plan with 64-key tiles and branch 0's Q in registers
  static constexpr int QRH = (q8 && (N >= 2 || (DTA_PAIR_N1 && HS <= 96)) &&
                              FwdCfg<E, HS, N, DVC, 4, false, 1>::bytes <= 80 * 1024) ? 1 : 0;
  static constexpr bool pair = !NP && QRH == 1 && q8 &&
                                FwdCfg<E, HS, N, DVC, 4, false, QRH>::PAIR &&
                                FwdCfg<E, HS, N, DVC, 4, false, QRH>::bytes <= 80 * 1024;
  static constexpr int QH = pair ? QRH : 0;
  static constexpr int NW = pair ? 4 : (q8 ? 8 : (q4 ? 4 : 4));
  static constexpr bool QREG = !(q8 || q4);
  static constexpr bool ok = FwdCfg<E, HS, N, DVC, NW, QREG, QH>::bytes <= LIM;
};

// Epilogue stores through an LDS bounce.  In the 32x32 accumulator layout a lane holds row
// (lane & 31), columns d*32 + 8g + 4hf + 0..3, so a direct store instruction writes 32 rows
// x 16 B per half-wave (32 cache lines); bounced through a per-wave LDS region (32 rows x 64
// fp32 = 8 KB, 16-byte chunks XOR-swizzled by row) every store instruction writes whole
// 256-byte row segments: 4 rows of 64 fp32, or 8 rows of 64 16-bit values.  A wave's own
// LDS accesses complete in order, so no wait sits between the write and the read.
// val(d, g) returns the lane's 4 values of column block d, group g; rows >= nrows are not
// stored.  dst: row 0, column 0 of the wave's tile; ld: row stride in OutT elements.
#ifndef DTA_FWD_BOUNCE
#define DTA_FWD_BOUNCE 1
#endif
#ifndef DTA_BWD_BOUNCE
#define DTA_BWD_BOUNCE 1
#endif
// Non-temporal bounced stores (whole 256-byte row segments, unlike the per-lane 16-byte stores
// that measured much slower NT in round 4): 1 = the fp32 ones -- the forward's O_i (537 MB at
// cfg2, read back once by attn_dq) and the dV sums -- so they stop evicting the operands the next
// kernels read from the Infinity Cache; 2 = every bounced store.  Step-interleaved A/B
// (profiles/r06i_ab_bounce_nt.json): cfg2 fwd + dq + dK/dV 2.879 -> 2.838 ms (1) / 2.835 (2),
// cfg3 N = 3 1.049 -> 1.034 / 1.037.  1 by default: the bf16 outputs (O, dQ, dK, dV) feed the
// very next kernels of a training step (GroupLN, the projection GEMMs).
#ifndef DTA_BOUNCE_NT
#define DTA_BOUNCE_NT 1
#endif
template <class OutT, int NDB, class Val>
__device__ __forceinline__ void bounce_store(float* reg, int lane, Val&& val, OutT* dst, int64_t ld, int nrows) {
  const int r = lane & 31, hf = lane >> 5;
#pragma unroll
  for (int h = 0; h < NDB / 2; ++h) {
#pragma unroll
    for (int dd = 0; dd < 2; ++dd)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = dd * 8 + 2 * g + hf;
        *reinterpret_cast<f32x4*>(reg + r * 64 + ((c ^ (r & 15)) << 2)) = val(2 * h + dd, g);
      }
    // the reads below take values other lanes wrote, and the next h rewrites the region:
    // pin the write -> read -> write order (a scheduling barrier only, no instruction; a
    // wave's LDS operations then complete in issue order)
    __builtin_amdgcn_wave_barrier();
    if constexpr (sizeof(OutT) == 4) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int rr = k * 4 + (lane >> 4), c = lane & 15;
        const f32x4 v = *reinterpret_cast<const f32x4*>(reg + rr * 64 + ((c ^ (rr & 15)) << 2));
        if (rr < nrows) {
          if constexpr (DTA_BOUNCE_NT >= 1) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst + rr * ld + h * 64 + c * 4));
          else *reinterpret_cast<f32x4*>(dst + rr * ld + h * 64 + c * 4) = v;
        }
      }
    } else {
      typedef OutT v8 __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int rr = k * 8 + (lane >> 3), c = (lane & 7) * 2;
        const f32x4 a = *reinterpret_cast<const f32x4*>(reg + rr * 64 + ((c ^ (rr & 15)) << 2));
        const f32x4 bq = *reinterpret_cast<const f32x4*>(reg + rr * 64 + (((c + 1) ^ (rr & 15)) << 2));
        const v8 v = {(OutT)a[0], (OutT)a[1], (OutT)a[2], (OutT)a[3], (OutT)bq[0], (OutT)bq[1], (OutT)bq[2], (OutT)bq[3]};
        if (rr < nrows) {
          if constexpr (DTA_BOUNCE_NT >= 2) __builtin_nontemporal_store(v, reinterpret_cast<v8*>(dst + rr * ld + h * 64 + c * 4));
          else *reinterpret_cast<v8*>(dst + rr * ld + h * 64 + c * 4) = v;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}
__device__ __forceinline__ bool t5_aligned16(const T5& t, int esize) {
  const int64_t m = 16 / esize;
  return (reinterpret_cast<uintptr_t>(t.p) & 15) == 0 && t.sb % m == 0 && t.st % m == 0 && t.sh % m == 0 &&
         t.si % m == 0;
}

// SEQ (N = 1 paired plans only): the workgroup runs p.bseq branches one after another over
// the same query block -- each branch's key loop, O_i and LSE_i as a branch-split
// workgroup would -- and keeps O = sum_i c_i O_i in registers across them, so the
// branch-split forward needs no combine pass (see launch_fwd_t).
template <class E, int HS, int N, int DVC, int NW, bool QREG, bool SRD, bool DROP, int QRH, bool SEQ = false>
__global__ __launch_bounds__(NW * 64, (FwdCfg<E, HS, N, DVC, NW, QREG, QRH>::PAIR ? 2 : FwdCfg<E, HS, N, DVC, NW, QREG, QRH>::WPE))
void attn_fwd_kernel(FwdParams p) {
  using O = Ops<E>;
  using frag = typename O::frag;
  using CF = FwdCfg<E, HS, N, DVC, NW, QREG, QRH>;
  constexpr int HSP = CF::HSP, DVP = CF::DVP;
  using QI = Img<E, HSP>;
  using KI = Img<E, HSP>;
  using VI = Img<E, DVP>;
  constexpr int NQR = QREG ? N : QRH;      // branches whose Q rows live in registers
  constexpr int BN = CF::BN, BM = CF::BM, NTHR = NW * 64;
  constexpr int KS = O::KSTEP;
  constexpr int NSQ = HS / KS;
  constexpr int NKB = BN / 32;
  constexpr int SPB = 32 / KS;
  constexpr int NDB = DVC / 32;
  constexpr float THR = 8.f;        // deferred-rescale threshold (log2 units): P <= 2^8

  extern __shared__ __attribute__((aligned(16))) char smem[];
  E* Qs = reinterpret_cast<E*>(smem);
  constexpr int NS = CF::NS;
  E* Kb = Qs + CF::nQ;              // [NS][N][BN][HSP]  ring
  E* Vb = Kb + NS * CF::nK;         // [NS][BN][DVP]

  // wave index is wave-uniform: make it provably so (SGPR), or every branch on it
  // becomes an exec-masked divergent branch
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tid = threadIdx.x, lane = tid & 63;
  int hf = lane >> 5, c32 = lane & 31;
  int bx, by, bz, lin;
  lpt_order(bx, by, bz, lin);                          // bx: work rank
  const int nch = p.DV / DVC;
  const int qt = gridDim.x - 1 - bx;                   // longest causal rows first
  // branch-split launch (N == 1 instantiation, p.bsplit branches per head): workgroup
  // (head, branch br) computes O_br and LSE_br only; a combine pass forms O
  const int nsp = (N == 1 && p.bsplit > 1) ? p.bsplit : 1;
  const int hv = by / nch, dc0 = (by % nch) * DVC;
  const int hh = nsp > 1 ? hv / nsp : hv, br = hv - hh * nsp;
  const int b = bz;
  const int T = p.T;
  const int q0 = qt * BM, qw0 = q0 + wave * 32;
  int qrow = qw0 + c32;

  static_assert(!SEQ || (N == 1 && QRH == 1 && DVC == 2 * HS && !DROP), "SEQ: N = 1 paired plans, whole dv");
  // the bounced epilogue (see bounce_store): 16-bit plans with whole 64-column passes, a
  // ring that holds a region per wave, fp32 O_i and 16-byte aligned outputs
  constexpr bool BNC = DTA_FWD_BOUNCE && sizeof(E) == 2 && NDB % 2 == 0 &&
                       NS * (CF::nK + CF::nV) * (int)sizeof(E) >= NW * 8192;
  const bool bnc = BNC && !p.ob16 && t5_aligned16(p.obr, 4) && (nsp > 1 || t5_aligned16(p.o, sizeof(E)));
  const int nseq = SEQ ? p.bseq : 1;
  const E* gq = reinterpret_cast<const E*>(p.q.p) + b * p.q.sb + hh * p.q.sh + br * p.q.si;
  const E* gk = reinterpret_cast<const E*>(p.k.p) + b * p.k.sb + hh * p.k.sh + br * p.k.si;
  const E* gv = reinterpret_cast<const E*>(p.v.p) + b * p.v.sb + hh * p.v.sh + dc0;
  const bool qrope = p.rope != nullptr;
  E* gqr = qrope ? reinterpret_cast<E*>(p.qrot.p) + b * p.qrot.sb + hh * p.qrot.sh + br * p.qrot.si : nullptr;

  float coef[N];
#pragma unroll
  for (int i = 0; i < N; ++i) coef[i] = nsp > 1 ? 1.f : p.coef[hh * p.cst + i];
  constexpr int NDBS = SEQ ? DVC / 32 : 1;
  f32x16 oacc[NDBS];                  // SEQ: sum_i c_i O_i over the branches done so far
#pragma unroll
  for (int d = 0; d < NDBS; ++d) oacc[d] = f32x16{};

  for (int sb = 0; sb < nseq; ++sb) {
  if constexpr (SEQ) {
    if (sb > 0) {
      gq += p.q.si; gk += p.k.si;
      if (qrope) gqr += p.qrot.si;
    }
    coef[0] = p.coef[hh * p.cst + sb];
  }
  const int brs = SEQ ? sb : br;      // this pass's branch index (LSE_i / O_i rows)
  frag qf[NQR > 0 ? NQR : 1][NQR > 0 ? NSQ : 1];
#pragma unroll
  for (int i = 0; i < NQR; ++i)
#pragma unroll
    for (int s = 0; s < NSQ; ++s)
      qf[i][s] = qrow < T ? O::load_global(gq + (int64_t)qrow * p.q.st + i * p.q.si + s * KS + hf * O::KH)
                          : O::zero();
#pragma unroll
  for (int i = NQR; i < N; ++i)
    stage<E, HSP, BM, HS, NTHR>(Qs + (i - NQR) * BM * HSP, gq + i * p.q.si, p.q.st, q0, T - 1, tid);
  // RoPE at load (p.rope, ABI 5): Q_i arrive un-rotated; the rows in registers turn here,
  // the LDS-staged ones once they land (first attempt); each rotated row is stored once to
  // p.qrot for the backward (by the dv chunk 0 workgroup), so the RoPE pass rotates K only
  bool qrot_pending = qrope && N > NQR;
  if (qrope) {
    const int tr = min(qrow, T - 1);
#pragma unroll
    for (int i = 0; i < NQR; ++i)
#pragma unroll
      for (int s = 0; s < NSQ; ++s) {
        rope_frag<E>(qf[i][s], p.rope, tr, s * KS + hf * O::KH, HS, hf);
        if (dc0 == 0 && qrow < T)
          *reinterpret_cast<frag*>(gqr + (int64_t)qrow * p.qrot.st + i * p.qrot.si + s * KS + hf * O::KH) = qf[i][s];
      }
  }

  // FSEED (see below; the same condition as FAST): the register-resident Q_i pre-scaled by
  // scale*log2e once, after the RoPE'd rows went to qrot; the LDS-resident ones after they land
  constexpr bool FSEED_Q = DTA_FWD_SEED && DTA_FWD_FAST && sizeof(E) == 2 && !DROP && N <= 2 &&
                           (CF::PAIR || CF::WPE >= 2);
  if constexpr (FSEED_Q) {
#pragma unroll
    for (int i = 0; i < NQR; ++i)
#pragma unroll
      for (int s = 0; s < NSQ; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[i][s][j] = (E)((float)qf[i][s][j] * p.sl2);
  }
  bool q_lds_unscaled = FSEED_Q && N > NQR;
  const int kend = min(T, q0 + BM);
  const int ntiles = (kend + BN - 1) / BN;
  using KR = KvRing<E, HS, N, DVC, BN, NW>;
  // this wave's per-lane DMA source offsets computed once (VGPRs): a tile then costs only
  // its two scalar descriptors and M0 (in-kernel stamps: fwd 0.979 -> 0.901 ms at cfg2)
  constexpr bool PRE = SRD;
  uint32_t doff[PRE ? KR::MYP : 1];
  if constexpr (PRE) KR::offsets(p.k.st, p.k.si, p.v.st, wave, lane, doff);
  auto stage_kv = [&](int kt, int buf) {
    const int k0 = kt * BN;
    if constexpr (PRE) {
      KR::issue_pre(gk, p.k.st, gv, p.v.st, k0, T, Kb + buf * CF::nK, Vb + buf * CF::nV, wave, doff);
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i)
        stage<E, HSP, BN, HS, NTHR>(Kb + (buf * N + i) * BN * HSP, gk + i * p.k.si, p.k.st, k0, T - 1, tid);
      stage<E, DVP, BN, DVC, NTHR>(Vb + buf * CF::nV, gv, p.v.st, k0, T - 1, tid);
    }
  };
  const int tile_pieces = SRD ? KR::pieces(wave)
                              : N * stage_pieces<E, HSP, BN, HS, NW>(wave) + stage_pieces<E, DVP, BN, DVC, NW>(wave);
  f32x16 acc[N][NDB];
  float m[N], l[N];
  const bool wave_live = qw0 < T;
  // FAST (16-bit, no dropout): after a workgroup's first key tile the reference m stays
  // fixed -- no per-tile row maximum, no rescale: P = exp2(S sl2 - m) straight off the
  // QK^T accumulators.  P may then exceed 1 by as much as the row maximum grew, and it is
  // packed to E for the PV operand, so the bound is the operand type's range: a lane whose
  // partial row sum (which bounds every P it packed) leaves [0, LSMAX] marks the workgroup,
  // which then re-runs its whole key loop on the per-tile-maximum path.  bf16 shares fp32's
  // exponent range: 2^60 (a row maximum that grew by ~55 log2 units past its first tile's,
  // or a non-finite score); fp16 saturates at 65504: 2^15.
  // (N <= 2 plans with two waves per SIMD: the one-wave 512-register plans and the hs = 32
  // N = 3 paired plan spill with it)
  constexpr bool FAST = DTA_FWD_FAST && sizeof(E) == 2 && !DROP && N <= 2 && (CF::PAIR || CF::WPE >= 2);
  constexpr float LSMAX = std::is_same<E, _Float16>::value ? 0x1p15f : 0x1p60f;
  float bad = 0.f;
  // SEED (with FAST): Q_i are pre-scaled by scale*log2e once (registers and LDS), so scores come
  // out of QK^T in log2 units, and on the fixed-reference tiles each branch's S accumulators
  // start at -m by one extra MFMA (a ones fragment times the row constant split into hi + lo
  // halves, as in attn_dq): P = exp2(S) needs no fma.  Entering those tiles each m moves to a value
  // the two halves represent exactly, so the seeded tiles, the earlier ones and the LSE agree.
  constexpr bool FSEED = DTA_FWD_SEED && FAST;
  static_assert(FSEED == FSEED_Q, "FSEED_Q restates FAST's condition");
  typename O::frag f_one = O::zero(), f_nm[FSEED ? N : 1];
  if constexpr (FSEED) { if (hf == 0) { f_one[0] = (E)1.f; f_one[1] = (E)1.f; } }
  auto mrep = [](float v) -> float {     // nearest value hi + lo (two E halves) represent
    const E hi = (E)v;
    return (float)hi + (float)(E)(v - (float)hi);
  };

  // per-lane LDS read bases kept in registers across the loop (see attn_dkdv_kernel)
  int LrK = 0, LtV = 0;      // set per attempt, after the ring prologue
  // key = k0 + kb*32 + rowof(r); masked when key > qrow or key >= T
  auto mask_scores = [&](int k0, f32x16 (&sa)[NKB]) {
    const int lim = min(qrow, T - 1) - k0 - 4 * hf;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) sa[kb][r] = (kb * 32 + (r & 3) + 8 * (r >> 2) > lim) ? -INFINITY : sa[kb][r];
  };
  // this lane's row maximum: two independent v_max3 chains
  auto row_max = [&](const f32x16 (&sa)[NKB]) -> float {
    float a = -INFINITY, b = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; r += 4) {
        a = fmaxf(fmaxf(a, sa[kb][r]), sa[kb][r + 1]);
        b = fmaxf(fmaxf(b, sa[kb][r + 2]), sa[kb][r + 3]);
      }
    return fmaxf(a, b);
  };
  // P = exp2(S * scale*log2e - m), row sums (two chains), packed to the PV operand;
  // with dropout the row sum keeps every element and the PV operand only the kept ones
  auto exp_pack = [&](int i, int k0, f32x16 (&sa)[NKB], frag (&pf)[NKB * SPB], bool seeded = false) -> float {
    const float mi = m[i];
    float ls0 = 0.f, ls1 = 0.f;
    // FSEED: scores already in log2 units (seeded tiles: already minus m)
    auto arg = [&](float v) { return FSEED ? (seeded ? v : v - mi) : fmaf(v, p.sl2, -mi); };
    if constexpr (DTA_FWD_PK && !FSEED) {
      // the argument fmas and the two row-sum chains as packed pairs (v_pk_fma_f32 /
      // v_pk_add_f32): element for element the scalar form's arithmetic, bitwise equal
      f32x2 ls2 = f32x2{0.f, 0.f};
      const f32x2 sl2v = f32x2{p.sl2, p.sl2}, nmv = f32x2{-mi, -mi};
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const f32x2 a2 = __builtin_elementwise_fma(f32x2{sa[kb][r], sa[kb][r + 1]}, sl2v, nmv);
          const float e0 = exp2_fast(a2[0]);
          const float e1 = exp2_fast(a2[1]);
          sa[kb][r] = e0;
          sa[kb][r + 1] = e1;
          ls2 += f32x2{e0, e1};
        }
      ls0 = ls2[0];
      ls1 = ls2[1];
    } else {
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float e0 = exp2_fast(arg(sa[kb][r]));
        const float e1 = exp2_fast(arg(sa[kb][r + 1]));
        sa[kb][r] = e0;
        sa[kb][r + 1] = e1;
        ls0 += e0;
        ls1 += e1;
      }
    }
    const float ls = ls0 + ls1;
    l[i] += ls;
    if constexpr (DROP) {
      const uint32_t key = drop_key(p.drop_seed_lo, p.drop_seed_hi, b, hh, br + i, p.H, nsp > 1 ? nsp : N);
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sa[kb][r] *= drop_mul(key, qrow, k0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf, p.drop_thr, p.drop_scale);
    }
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      if constexpr (SPB == 2) {
        pf[kb * 2 + 0] = O::template pack<0>(sa[kb]);
        pf[kb * 2 + 1] = O::template pack<1>(sa[kb]);
      } else {
#pragma unroll
        for (int s = 0; s < 16; ++s) pf[kb * SPB + s] = sa[kb][s];
      }
    }
    return ls;
  };
  // one branch's mask, max, deferred rescale (only when some row's max grew by > 2^THR), exp;
  // fast: exp against the fixed m, the lane's partial sum checked instead
  auto softmax_branch = [&](int i, int k0, auto MASKED, f32x16 (&sa)[NKB], frag (&pf)[NKB * SPB], auto FASTT) {
    if constexpr (decltype(MASKED)::value) mask_scores(k0, sa);
    if constexpr (decltype(FASTT)::value) {
      {
        const float ls = exp_pack(i, k0, sa, pf, FSEED);
        bad = (ls <= LSMAX) ? bad : 1.f;        // NaN / inf / past the operand range: re-run
        return;
      }
    }
    const float mx = wave_max_halves(row_max(sa)) * (FSEED ? 1.f : p.sl2);
    if (__any(mx > m[i] + THR)) {
      const float mnew = fmaxf(m[i], mx);
      const float alpha = exp2_fast(m[i] - mnew);
      m[i] = mnew;
      l[i] *= alpha;
#pragma unroll
      for (int d = 0; d < NDB; ++d) acc[i][d] *= alpha;
    }
    exp_pack(i, k0, sa, pf);
  };
  // DTA_FWD_TR_EARLY (single-branch 16-bit plans without dropout -- the N = 2 plan spills with it --
  // on the non-pipelined PV path): the first d-block's V^T
  // reads of the PV product are issued after the last branch's QK^T chain, ahead of its softmax
  // VALU, so their LDS latency hides behind it (16 more VGPRs live across it)
  constexpr bool FTRE = DTA_FWD_TR_EARLY && N == 1 && sizeof(E) == 2 && !DROP && !(DTA_FWD_PIPE > 0 && NKB == 1 && NDB > 1);
  lds64 rv0[NKB][4];        // (full size even when unused: referenced in a generic lambda)
  auto issue_v0 = [&](int kt) {
    if constexpr (FTRE) {
      const unsigned vb = lds_addr(Vb + (kt % NS) * CF::nV);
      const unsigned a0 = vb + LtV, a1 = vb + (LtV ^ 32);
      sfor<NKB>([&](auto KB) { tr_issue<VI::ROWB, 32 * decltype(KB)::value>(rv0[decltype(KB)::value], a0, a1); });
    }
  };
  // QK^T + online softmax of one key tile for every branch, P packed as the PV B operand
  auto phase_a = [&](int kt, auto MASKED, frag (&pf)[N][NKB * SPB], auto FASTT) {
    constexpr bool MASK = decltype(MASKED)::value;
    const int buf = kt % NS;
    const int k0 = kt * BN;
    const E* Kc = Kb + buf * CF::nK;
    f32x16 sa[N][NKB];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const E* Ki = Kc + i * BN * HSP;
      if constexpr (sizeof(E) == 2) {
        // row operands: byte R*ROWB + (Lrow ^ 32 s) for a 32-row block at row R
        const int Lr = LrK;
        const char* kbase = reinterpret_cast<const char*>(Ki);
        const char* qbase = reinterpret_cast<const char*>(Qs + (i >= NQR ? i - NQR : 0) * BM * HSP) + wave * 32 * QI::ROWB;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
          sa[i][kb] = (FSEED && decltype(FASTT)::value) ? O::mma(f_one, f_nm[FSEED ? i : 0], f32x16{}) : f32x16{};
        if constexpr (NSQ * (NKB + 1) <= 12 && QRH == 0) {
          // every operand read of this branch's S^T issued ahead of its MFMA chain,
          // so the chain waits on the LDS latency once instead of per k-step
          // (head sizes <= 64; at 128 the 24 fragments do not fit the registers)
          frag kfr[NKB][NSQ], qfr[NSQ];
#pragma unroll
          for (int s = 0; s < NSQ; ++s) {
            const int o = Lr ^ (32 * s);
            if (i < NQR) qfr[s] = qf[i < NQR ? i : 0][s];
            else qfr[s] = *reinterpret_cast<const frag*>(qbase + o);
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) kfr[kb][s] = *reinterpret_cast<const frag*>(kbase + kb * 32 * KI::ROWB + o);
          }
#pragma unroll
          for (int s = 0; s < NSQ; ++s)
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) sa[i][kb] = O::mma(kfr[kb][s], qfr[s], sa[i][kb]);
          if (i < NQR) __builtin_amdgcn_sched_group_barrier(0x100, NSQ * NKB, 0);
          else __builtin_amdgcn_sched_group_barrier(0x100, NSQ * (NKB + 1), 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NSQ * NKB, 0);
        } else if constexpr (DTA_FWD_PIPE > 0 && QI::ROWB == KI::ROWB && NKB == 1) {
          // operand reads DTA_FWD_PIPE reads ahead of the MFMAs (see s_chain_pipe); 32-key
          // tiles only: with 64-key tiles (cfg2) the paired plan sits at 252 VGPRs and the
          // pipelined chain measured slower (fwd 0.954 -> 1.008 ms), cfg5 0.97x
          sfor<N>([&](auto I_) {
            constexpr int ic = decltype(I_)::value;
            if (ic == i)
              s_chain_pipe<E, NSQ, NKB, (ic >= NQR ? 1 : 0), DTA_FWD_PIPE, ic * BN * HSP * (int)sizeof(E),
                           (ic >= NQR ? ic - NQR : 0) * BM * HSP * (int)sizeof(E), KI::ROWB>(
                  sa[ic], lds_addr(Kc) + Lr, lds_addr(Qs) + wave * 32 * QI::ROWB + Lr, qf[ic < NQR ? ic : 0]);
          });
        } else {
#pragma unroll
          for (int s = 0; s < NSQ; ++s) {
            const int o = Lr ^ (32 * s);
            frag qb;
            if (i < NQR) qb = qf[i < NQR ? i : 0][s];
            else qb = *reinterpret_cast<const frag*>(qbase + o);
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
              sa[i][kb] = O::mma(*reinterpret_cast<const frag*>(kbase + kb * 32 * KI::ROWB + o), qb, sa[i][kb]);
          }
        }
      } else {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
          sa[i][kb] = f32x16{};
#pragma unroll
          for (int s = 0; s < NSQ; ++s) {
            frag qb;
            if (i < NQR) qb = qf[i < NQR ? i : 0][s];
            else qb = QI::row(Qs + (i >= NQR ? i - NQR : 0) * BM * HSP, wave * 32 + c32, s, hf);
            sa[i][kb] = O::mma(KI::row(Ki, kb * 32 + c32, s, hf), qb, sa[i][kb]);
          }
        }
      }
      if (FTRE && i == N - 1) issue_v0(kt);
      softmax_branch(i, k0, MASKED, sa[i], pf[i], FASTT);
    }
  };
  // O_i^T += V^T P_i^T, one V fragment feeds every branch
  auto phase_b = [&](int kt, const frag (&pf)[N][NKB * SPB]) {
    const E* Vc = Vb + (kt % NS) * CF::nV;
    // the dropout plans spill (up to 128 B/lane): compiler-tracked V^T reads (see tr_load)
    constexpr bool SPILLS = DROP;
    if constexpr (sizeof(E) == 2 && DTA_FWD_PIPE > 0 && NKB == 1 && NDB > 1 && !SPILLS) {
      // the next d-block's V^T fragments read while this one's MFMAs run (32-key tiles:
      // 8 more VGPRs)
      const unsigned vb = lds_addr(Vc);
      const int Lv = LtV;
      lds64 r[2][NKB][4];
      auto issue = [&](auto D) {
        constexpr int d = decltype(D)::value;
        const unsigned a0 = vb + (Lv ^ (64 * d)), a1 = vb + (Lv ^ (64 * d + 32));
        sfor<NKB>([&](auto KB) { tr_issue<VI::ROWB, 32 * decltype(KB)::value>(r[d & 1][decltype(KB)::value], a0, a1); });
      };
      issue(std::integral_constant<int, 0>{});
      sfor<NDB>([&](auto D) {
        constexpr int d = decltype(D)::value;
        if constexpr (d + 1 < NDB) issue(std::integral_constant<int, d + 1>{});
        lgkm_pin_n<(d + 1 < NDB ? 4 * NKB : 0), NKB>(r[d & 1]);
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const frag va = tr_frag<E>(r[d & 1][kb], s);
#pragma unroll
            for (int i = 0; i < N; ++i) acc[i][d] = O::mma(va, pf[i][kb * 2 + s], acc[i][d]);
          }
      });
    } else if constexpr (sizeof(E) == 2) {
      const unsigned vb = lds_addr(Vc);
      const int Lv = LtV;
      sfor<NDB>([&](auto D) {
        constexpr int d = decltype(D)::value;
        lds64 r[NKB][4];
        const unsigned a0 = vb + (Lv ^ (64 * d)), a1 = vb + (Lv ^ (64 * d + 32));
        if constexpr (FTRE && d == 0) {
          lgkm_pin<NKB>(rv0);
#pragma unroll
          for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              const frag va = tr_frag<E>(rv0[kb], s);
#pragma unroll
              for (int i = 0; i < N; ++i) acc[i][d] = O::mma(va, pf[i][kb * 2 + s], acc[i][d]);
            }
          return;
        }
        if constexpr (SPILLS) {
          sfor<NKB>([&](auto KB) { tr_load<VI::ROWB, 32 * decltype(KB)::value>(r[decltype(KB)::value], a0, a1); });
        } else {
          sfor<NKB>([&](auto KB) { tr_issue<VI::ROWB, 32 * decltype(KB)::value>(r[decltype(KB)::value], a0, a1); });
          lgkm_pin<NKB>(r);
        }
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const frag va = tr_frag<E>(r[kb], s);
#pragma unroll
            for (int i = 0; i < N; ++i) acc[i][d] = O::mma(va, pf[i][kb * 2 + s], acc[i][d]);
          }
      });
    } else {
#pragma unroll
      for (int d = 0; d < NDB; ++d)
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
          for (int s = 0; s < SPB; ++s) {
            const frag va = VI::tr_perm(Vc, kb * 32, s, hf, d * 32, lane);
#pragma unroll
            for (int i = 0; i < N; ++i) acc[i][d] = O::mma(va, pf[i][kb * SPB + s], acc[i][d]);
          }
    }
  };

  // two loops over straight-line bodies: tiles strictly below the block's first
  // query row and inside T need no mask; the block's diagonal / tail tiles do
  // (one loop body with both variants behind a branch spills)
  Stamps<> st;
  auto step = [&](int kt, auto MASKED, auto FASTT) {
    // keep lane-derived addresses loop-variant: recomputed per tile instead of
    // hoisted into (spilled) registers across the whole loop
    asm volatile("" : "+v"(lane));
    if constexpr (sizeof(E) == 2) asm volatile("" : "+v"(LrK), "+v"(LtV));
    tid = (wave << 6) + lane; hf = lane >> 5; c32 = lane & 31;
    qrow = qw0 + c32;
    const bool live = wave_live && kt * BN <= qw0 + 31;
    st.lap<7>();
    if (kt + NS - 1 < ntiles) stage_kv(kt + NS - 1, (kt + NS - 1) % NS);
    st.lap<0>();
    if constexpr (DTA_FWD_IGLP >= 0) __builtin_amdgcn_iglp_opt(DTA_FWD_IGLP >= 0 ? DTA_FWD_IGLP : 0);   // A/B: LLVM's MFMA / LDS interleave strategy
    if (live) {
      frag pf[N][NKB * SPB];
      phase_a(kt, MASKED, pf, FASTT);
      st.lap<1>();
      phase_b(kt, pf);
      st.lap<2>();
    }
    // tile kt+1 must have landed; younger tiles may stay in flight
    wait_vm(tile_pieces * max(0, min(NS - 2, ntiles - 2 - kt)));
    st.lap<3>();
    lds_barrier();
    st.lap<4>();
  };
  // one pass over the key tiles: ring prologue, state reset, the unmasked then the masked
  // loop; with FAST every tile after the first runs without the per-tile maximum
  auto attempt = [&](bool safe) {
    for (int j = 0; j < NS - 1; ++j)
      if (j < ntiles) stage_kv(j, j);
    wait_vm(tile_pieces * max(0, min(NS - 1, ntiles) - 1));   // tile 0 (and the Q block) landed
    lds_barrier();
    if (qrot_pending) {
#pragma unroll
      for (int i = NQR; i < N; ++i)
        rope_lds<E, HSP, BM, HS, NTHR>(Qs + (i - NQR) * BM * HSP, p.rope, q0, T, gqr + i * p.qrot.si, p.qrot.st,
                                       dc0 == 0, tid);
      lds_barrier();
      qrot_pending = false;
    }
    if (q_lds_unscaled) {                    // FSEED: the LDS-resident Q_i, once
      scale_lds<E, NTHR>(Qs, CF::nQ, p.sl2, tid);
      lds_barrier();
      q_lds_unscaled = false;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      m[i] = -INFINITY;
      l[i] = 0.f;
#pragma unroll
      for (int d = 0; d < NDB; ++d) acc[i][d] = f32x16{};
    }
    if constexpr (sizeof(E) == 2) { LrK = row_lane<KI::ROWB>(lane); LtV = tr_lane<VI::ROWB>(lane); }
    st.start();
    const int nfull = min(ntiles, min((q0 + 1) / BN, T / BN));
    // per-tile-maximum tiles: all of them (safe, or no FAST), else the first one only
    const int kslow = (safe || !FAST) ? ntiles : min(1, ntiles);
    for (int kt = 0; kt < min(nfull, kslow); ++kt) step(kt, std::false_type{}, std::false_type{});
    for (int kt = nfull; kt < kslow; ++kt) step(kt, std::true_type{}, std::false_type{});
    if constexpr (FAST) {
      if constexpr (FSEED) {
        // the fixed reference moves to the nearest value the seed's two E halves represent (the
        // first tile's sums and accumulators follow it, a factor of 1 + O(2^-16)); one the halves
        // cannot hold (fp16 beyond 65504) sends the workgroup to the exact per-tile-maximum re-run
#pragma unroll
        for (int i = 0; i < N; ++i) {
          const float mr = mrep(m[i]);
          if (!(fabsf(mr) < INFINITY)) bad = 1.f;
          const float a = (fabsf(mr) < INFINITY) ? exp2_fast(m[i] - mr) : 1.f;
          l[i] *= a;
#pragma unroll
          for (int d = 0; d < NDB; ++d) acc[i][d] *= a;
          m[i] = (fabsf(mr) < INFINITY) ? mr : m[i];
          f_nm[i] = seed_frag<E>(-m[i], hf);
        }
      }
      for (int kt = kslow; kt < nfull; ++kt) step(kt, std::false_type{}, std::true_type{});
      for (int kt = max(kslow, nfull); kt < ntiles; ++kt) step(kt, std::true_type{}, std::true_type{});
    }
  };
  // one inlined copy of the loops: pass 1 (FAST) re-runs only a flagged workgroup
  for (int pass = 0; pass < (FAST ? 2 : 1); ++pass) {
    attempt(pass == 1);
    if constexpr (!FAST) break;
    if (pass == 1) break;
    // rows past T never count; the ring is idle (the last step drained it behind a barrier)
    int* flag = reinterpret_cast<int*>(Kb);
    const bool mine = __any(wave_live && qrow < T && bad != 0.f);
    if (lane == 0) flag[wave] = mine ? 1 : 0;
    lds_barrier();
    bool any = false;
#pragma unroll
    for (int w = 0; w < NW; ++w) any |= flag[w] != 0;
    lds_barrier();
    if (!any) break;
  }
  st.lap<5>();
  st.flush(p.stamps, lin * NW + wave, lane);

  if (!SEQ && !wave_live) return;
  if (DTA_EPI_SKIP == 1 && p.T != -7) return;
  if (bnc) {
    if (wave_live) {
      float inv[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const float lt = wave_sum_halves(l[i]);
        inv[i] = 1.f / lt;
        if (dc0 == 0 && hf == 0 && qrow < T)
          p.lse[(((int64_t)(brs + i) * p.B + b) * p.H + hh) * T + qrow] = -(m[i] + __builtin_log2f(lt));   // stored negated
      }
      float* reg = reinterpret_cast<float*>(Kb) + wave * 2048;    // the ring is idle
      const int nrows = min(32, T - qw0);
      float* gob0 = reinterpret_cast<float*>(p.obr.p) + b * p.obr.sb + (int64_t)qw0 * p.obr.st + hh * p.obr.sh +
                    brs * p.obr.si + dc0;
#pragma unroll
      for (int i = 0; i < N; ++i)
        bounce_store<float, NDB>(reg, lane, [&](int d, int g) {
          return f32x4{acc[i][d][4 * g] * inv[i], acc[i][d][4 * g + 1] * inv[i], acc[i][d][4 * g + 2] * inv[i],
                       acc[i][d][4 * g + 3] * inv[i]};
        }, gob0 + i * p.obr.si, p.obr.st, nrows);
      auto osum = [&](int d, int g) {
        f32x4 o = f32x4{};
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = fmaf(coef[i], acc[i][d][4 * g + j] * inv[i], o[j]);
        return o;
      };
      if constexpr (SEQ) {
#pragma unroll
        for (int d = 0; d < NDB; ++d)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 o = osum(d, g);
#pragma unroll
            for (int j = 0; j < 4; ++j) oacc[d < NDBS ? d : 0][4 * g + j] += o[j];
          }
      } else if (nsp == 1) {
        E* go0 = reinterpret_cast<E*>(p.o.p) + b * p.o.sb + (int64_t)qw0 * p.o.st + hh * p.o.sh + dc0;
        bounce_store<E, NDB>(reg, lane, osum, go0, p.o.st, nrows);
      }
    }
    if constexpr (SEQ) lds_barrier();       // the next branch's ring prologue overwrites the regions
  } else {
  if (!SEQ && qrow >= T) return;
  if (wave_live && qrow < T) {      // (SEQ: every lane stays for the next branch's barriers)
  float inv[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float lt = wave_sum_halves(l[i]);
    inv[i] = 1.f / lt;
    if (dc0 == 0 && hf == 0)
      p.lse[(((int64_t)(brs + i) * p.B + b) * p.H + hh) * T + qrow] = -(m[i] + __builtin_log2f(lt));   // stored negated
  }
  E* go = reinterpret_cast<E*>(p.o.p) + b * p.o.sb + (int64_t)qrow * p.o.st + hh * p.o.sh + dc0;
  // O_i saved for the backward's delta_i = <dO, O_i> (whose sums feed d(lambda)): fp32, or
  // fp16 (p.ob16: 2^-11, eight times bf16's resolution, half the bytes)
  const int64_t gob = b * p.obr.sb + (int64_t)qrow * p.obr.st + hh * p.obr.sh + brs * p.obr.si + dc0;
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int e = d * 32 + 8 * g + 4 * hf;
      float o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const float a0 = acc[i][d][4 * g + 0] * inv[i], a1 = acc[i][d][4 * g + 1] * inv[i];
        const float a2 = acc[i][d][4 * g + 2] * inv[i], a3 = acc[i][d][4 * g + 3] * inv[i];
        if (DTA_EPI_SKIP != 2 || p.T == -7) store_ob4(p.obr.p, gob + i * p.obr.si + e, p.ob16, a0, a1, a2, a3);
        o0 = fmaf(coef[i], a0, o0); o1 = fmaf(coef[i], a1, o1);
        o2 = fmaf(coef[i], a2, o2); o3 = fmaf(coef[i], a3, o3);
      }
      if constexpr (SEQ) {
        oacc[d < NDBS ? d : 0][4 * g + 0] += o0; oacc[d < NDBS ? d : 0][4 * g + 1] += o1;
        oacc[d < NDBS ? d : 0][4 * g + 2] += o2; oacc[d < NDBS ? d : 0][4 * g + 3] += o3;
      } else {
        if (nsp == 1) store4<E>(go + e, o0, o1, o2, o3);
      }
    }
  }
  }   // bnc
  }   // branches (SEQ)
  if constexpr (SEQ) {
    if (qw0 >= T) return;
    if (bnc) {
      E* go0 = reinterpret_cast<E*>(p.o.p) + b * p.o.sb + (int64_t)qw0 * p.o.st + hh * p.o.sh + dc0;
      bounce_store<E, NDBS>(reinterpret_cast<float*>(Kb) + wave * 2048, lane, [&](int d, int g) {
        return f32x4{oacc[d][4 * g], oacc[d][4 * g + 1], oacc[d][4 * g + 2], oacc[d][4 * g + 3]};
      }, go0, p.o.st, min(32, T - qw0));
      return;
    }
    if (qrow >= T) return;
    E* go = reinterpret_cast<E*>(p.o.p) + b * p.o.sb + (int64_t)qrow * p.o.st + hh * p.o.sh + dc0;
#pragma unroll
    for (int d = 0; d < NDBS; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4<E>(go + d * 32 + 8 * g + 4 * hf, oacc[d][4 * g], oacc[d][4 * g + 1], oacc[d][4 * g + 2], oacc[d][4 * g + 3]);
  }
}

// ------------------------------------------------------ backward: dQ ---
template <class E, int HS, int N, int DV, int NW, bool QREG, int QRH = 0, bool BN32 = false>
struct DqCfg {
  // QRH > 0 (paired plan): the first QRH branches' Q rows stay in registers, the
  // rest in LDS, so Q plus a 2-stage ring of 64-key tiles fits 80 KB
  static constexpr bool PAIR = NW == 4 && !QREG && sizeof(E) == 2;
  // BN32: 32-key tiles where no plan with 64-key tiles fits (N = 4 at head size >= 96)
  static constexpr int BN = (PAIR && QRH == 0) || BN32 ? 32 : FwdTile<E>::BN;
  static constexpr int BM = NW * 32;
  // LDS image widths: K rows at least 32 columns (the transposed reads of dQ = dS K take
  // 32-column blocks), every row a power-of-two pitch
  static constexpr int HSP = img_cols(HS < 32 ? 32 : HS), QP = img_cols(HS), DVP = img_cols(DV);
  static constexpr int nQ = QREG ? 0 : (N - QRH) * BM * QP;
  static constexpr int nK = N * BN * HSP;
  static constexpr int nV = BN * DVP;
  static constexpr int NS = ring_stages_lim(nQ * (int)sizeof(E), (nK + nV) * (int)sizeof(E),
                                            PAIR ? 80 * 1024 : 160 * 1024);
  static constexpr int bytes = (nQ + NS * nK + NS * nV) * (int)sizeof(E);
};

// N = 3 at head size 64 (cfg3): no 8-wave plan fits, so the dQ plan was one wave per
// SIMD (Q of all branches in registers, 160 AGPRs).  In the paired layout with 32-key
// tiles (branch 0's Q in registers, branches 1-2 in LDS, 72 KB, 252 VGPRs, no spill) it is
// faster: one-process A/B (profiles/r05g_ab_dq_pair3.json) cfg3 B=16 H=6 T=2048 dQ 0.414 ->
// 0.379 ms, B=8 H=16 T=4096 1.683 -> 1.329 ms.  DTA_DQ_PAIR3 = 0 (A/B builds) keeps one wave.
#ifndef DTA_DQ_EXPG
#define DTA_DQ_EXPG 4            // exps per group ahead of their products in the dQ softmax (r05u: 1 -> 4, cfg2 dQ 0.888 -> 0.867 ms)
#endif
#ifndef DTA_DQ_PAIR3
#define DTA_DQ_PAIR3 1
#endif
#ifndef DTA_DQ_TR_EARLY
#define DTA_DQ_TR_EARLY 0        // A/B: dQ's first d-block transposed K_i reads issued before the softmax VALU
#endif
#ifndef DTA_DKDV_TR_EARLY
#define DTA_DKDV_TR_EARLY 0      // A/B: dK/dV's transposed Q_i reads issued before the softmax VALU
#endif
#ifndef DTA_DQ_PK
#define DTA_DQ_PK 0              // A/B: dQ's dS math as packed fp32 pairs (v_pk_*): 120 -> 78 VALU issues per step, dq +1% (r06p): off
#endif
#ifndef DTA_DKDV_PK
#define DTA_DKDV_PK 0            // A/B: dK/dV's dS / dV-operand math as packed fp32 pairs (v_pk_*): 123 -> 101 VALU issues, dK/dV +2.8% (r06p): off
#endif
#ifndef DTA_DKDV_CFOLD
#define DTA_DKDV_CFOLD 1         // 0: never build the |c_i|-folded dK/dV instantiations (lse_c ignored)
#endif
#ifndef DTA_DQ_EARLY_RING
#define DTA_DQ_EARLY_RING 0      // A/B: the K/V ring's first stages issued before the delta_i prologue
#endif
#ifndef DTA_DQ_B32_N2
#define DTA_DQ_B32_N2 0          // A/B: the paired N = 2 dQ plan with 32-key tiles
#endif
template <class E, int HS, int N, int DV = 2 * HS, bool NP = false>
struct DqPick {
  static constexpr int LIM = 160 * 1024;
  static constexpr bool q8 = sizeof(E) == 2 && DqCfg<E, HS, N, DV, 8, false>::bytes <= LIM;
  // paired 4-wave plan with 64-key tiles and branch 0's Q in registers
  static constexpr int QRH = (q8 && (N >= 2 || DTA_PAIR_N1) &&
                              DqCfg<E, HS, N, DV, 4, false, 1>::bytes <= 80 * 1024) ? 1 : 0;
  // (head size >= 64: the hs = 32, N = 3 paired plan spills)
  static constexpr bool pair64 = !NP && QRH == 1 && q8 && HS >= 64 &&
                                 DqCfg<E, HS, N, DV, 4, false, QRH>::bytes <= 80 * 1024;
  // N >= 3 at head size 64, where no 8-wave plan fits: the paired layout with 32-key
  // tiles (branch 0's Q in registers) instead of one wave per SIMD (DTA_DQ_PAIR3)
  static constexpr bool pair32 = DTA_DQ_PAIR3 && !NP && !pair64 && sizeof(E) == 2 && N >= 3 && HS == 64 &&
                                 DqCfg<E, HS, N, DV, 4, false, 1, true>::bytes <= 80 * 1024;
  static constexpr bool pair = pair64 || pair32;
  static constexpr int NW = pair ? 4 : (q8 ? 8 : (sizeof(E) == 2 ? 4 : 2));
  static constexpr bool QREG = pair ? false : !q8;
  static constexpr int QH = pair ? 1 : 0;
  static constexpr bool B32 = pair32 || (DTA_DQ_B32_N2 && pair64 && N == 2) ||
                              DqCfg<E, HS, N, DV, NW, QREG, QH>::bytes > LIM;   // 32-key tiles
  static constexpr bool ok = DqCfg<E, HS, N, DV, NW, QREG, QH, B32>::bytes <= LIM;
};

template <class E, int HS, int N, int DV, int NW, bool QREG, bool OUTF32, bool SRD, bool DROP, int QRH, bool B32>
__global__ __launch_bounds__(NW * 64, simd_waves(NW, DqCfg<E, HS, N, DV, NW, QREG, QRH, B32>::bytes))
void attn_dq_kernel(BwdParams p) {
  using O = Ops<E>;
  using frag = typename O::frag;
  using CF = DqCfg<E, HS, N, DV, NW, QREG, QRH, B32>;
  constexpr int NQR = QREG ? N : QRH;      // branches whose Q rows live in registers
  constexpr int HSP = CF::HSP, QP = CF::QP, DVP = CF::DVP;
  using QI = Img<E, QP>;
  using KI = Img<E, HSP>;
  using VI = Img<E, DVP>;
  constexpr int BN = CF::BN, BM = CF::BM, NTHR = NW * 64;
  constexpr int KS = O::KSTEP;
  constexpr int NSQ = HS / KS, NSV = DV / KS;
  constexpr int NKB = BN / 32, SPB = 32 / KS, NHB = (HS + 31) / 32;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  E* Qs = reinterpret_cast<E*>(smem);   // [N][BM][QP] unless QREG
  constexpr int NS = CF::NS;
  E* Kb = Qs + CF::nQ;                  // [NS][N][BN][HSP]  ring
  E* Vb = Kb + NS * CF::nK;             // [NS][BN][DVP]

  // wave index is wave-uniform: make it provably so (SGPR), or every branch on it
  // becomes an exec-masked divergent branch
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tid = threadIdx.x, lane = tid & 63;
  int hf = lane >> 5, c32 = lane & 31;
  int bx, by, bz, lin;
  lpt_order(bx, by, bz, lin);                          // bx: work rank
  const int qt = gridDim.x - 1 - bx;                   // longest causal rows first
  const int hh = by, b = bz;
  const int T = p.T;
  const int q0 = qt * BM, qw0 = q0 + wave * 32;
  int qrow = qw0 + c32;
  const bool rowok = qrow < T;

  const E* gq = reinterpret_cast<const E*>(p.q.p) + b * p.q.sb + hh * p.q.sh;
  const E* gk = reinterpret_cast<const E*>(p.k.p) + b * p.k.sb + hh * p.k.sh;
  const E* gv = reinterpret_cast<const E*>(p.v.p) + b * p.v.sb + hh * p.v.sh;
  const E* gdo = reinterpret_cast<const E*>(p.dout.p) + b * p.dout.sb + hh * p.dout.sh;
  const int64_t gob = b * p.obr.sb + hh * p.obr.sh;   // O_i: fp32, or fp16 with p.ob16

  const int kend = min(T, q0 + BM);
  const int ntiles = (kend + BN - 1) / BN;
  using KR = KvRing<E, HS, N, DV, BN, NW>;
  static_assert(!SRD || (HSP == KR::HSP && DVP == KR::DVP), "descriptor staging fills the kernel's images");
  constexpr bool PRE = SRD && !DROP;  // DMA source offsets computed once (dropout: fewer spills without)
  uint32_t doff[PRE ? KR::MYP : 1];
  if constexpr (PRE) KR::offsets(p.k.st, p.k.si, p.v.st, wave, lane, doff);
  auto stage_kv = [&](int kt, int buf) {
    const int k0 = kt * BN;
    if constexpr (PRE) {
      KR::issue_pre(gk, p.k.st, gv, p.v.st, k0, T, Kb + buf * CF::nK, Vb + buf * CF::nV, wave, doff);
    } else if constexpr (SRD) {
      KR::issue(gk, p.k.st, p.k.si, gv, p.v.st, k0, T, Kb + buf * CF::nK, Vb + buf * CF::nV, wave, lane);
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i)
        stage<E, HSP, BN, HS, NTHR>(Kb + (buf * N + i) * BN * HSP, gk + i * p.k.si, p.k.st, k0, T - 1, tid);
      stage<E, DVP, BN, DV, NTHR>(Vb + buf * CF::nV, gv, p.v.st, k0, T - 1, tid);
    }
  };

  // (head size 128 at N >= 3 spills further with the seed fragments: it keeps the fmas)
  constexpr bool SEED = DTA_DQ_SEED && std::is_same<E, __bf16>::value && !DROP && SRD && !(HS >= 128 && N >= 3);
  // plans that spill (16-bit head size 128 at N >= 3: 84-508 B/lane of scratch; dropout
  // plans: up to 532 B/lane) read LDS only through compiler-tracked loads: no asm read
  // whose destination the allocator could spill before it lands (see tr_load)
  constexpr bool SPILLS = sizeof(E) == 2 && (DROP || (HS >= 128 && N >= 3) || (HS >= 192 && N >= 2));
  // DTA_DQ_EARLY_RING: the ring's first stages are issued before the per-row loads and the
  // delta_i reduction below, so their DMA overlaps the O_i reads instead of following them
  constexpr bool EARLY = DTA_DQ_EARLY_RING && SRD;
  if constexpr (EARLY)
    for (int j = 0; j < NS - 1; ++j)
      if (j < ntiles) stage_kv(j, j);
  // ---- per-row operands in registers: Q_i and dO rows (B operands), LSE, delta
  frag qf[NQR > 0 ? NQR : 1][NQR > 0 ? NSQ : 1], df[NSV];
  float coef[N], lse[N], del[N];
  float dhead = 0.f;                 // delta of the current dK/dV group's first branch (delta rows below)
  const int64_t rs = (((int64_t)0 * p.B + b) * p.H + hh) * T + qrow;     // [i][b][h][t], i = 0
  const int64_t bstride = (int64_t)p.B * p.H * T;
#pragma unroll
  for (int s = 0; s < NSV; ++s)
    df[s] = rowok ? O::load_global(gdo + (int64_t)qrow * p.dout.st + s * KS + hf * O::KH) : O::zero();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    coef[i] = p.coef[hh * p.cst + i];
    if (i < NQR) {
#pragma unroll
      for (int s = 0; s < NSQ; ++s)
        qf[i < NQR ? i : 0][s] = rowok ? O::load_global(gq + (int64_t)qrow * p.q.st + i * p.q.si + s * KS + hf * O::KH)
                                       : O::zero();
      if constexpr (SEED) {
#pragma unroll
        for (int s = 0; s < NSQ; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) qf[i < NQR ? i : 0][s][j] = (E)((float)qf[i < NQR ? i : 0][s][j] * p.sl2);
      }
    }
    lse[i] = rowok ? p.lse[rs + i * bstride] : 0.f;
    // ABI 8 lse_c: the stored LSE_i + log2|c_i| for attn_dkdv, which then seeds its scores with
    // it and gets |c_i| P_i out of its exp (c_i = 0: -inf, P = 0)
    if (p.lsec && rowok && hf == 0) p.lsec[rs + i * bstride] = lse[i] + __builtin_log2f(fabsf(coef[i]));
    // delta_i = <dO, O_i> over this row (flash-backward preprocess), both lane halves
    float d = 0.f;
    if (rowok) {
#pragma unroll
      for (int s = 0; s < NSV; ++s) {
        const int64_t o = gob + (int64_t)qrow * p.obr.st + i * p.obr.si + s * KS + hf * O::KH;
        if constexpr (sizeof(E) == 2) {
          float ov[8];
          load_ob8(p.obr.p, o, p.ob16, ov);
#pragma unroll
          for (int j = 0; j < 8; ++j) d = fmaf((float)df[s][j], ov[j], d);
        } else {
          d = fmaf(df[s], reinterpret_cast<const float*>(p.obr.p)[o], d);
        }
      }
    }
    d = wave_sum_halves(d);
    del[i] = d;
    // row constants for attn_dkdv, which folds c_i into its dK_i epilogue: without
    // dropout -delta_h (its dP accumulator's seed) at each dK/dV group's first branch h and
    // delta_h - delta_i after it -- h = 0 (this group), or the dK/dV grouping's starts
    // (p.kstarts, this launch holding every branch); with dropout delta_i
    const bool kstart = i == 0 || (DTA_DQ_KSTARTS && ((p.kstarts >> i) & 1));
    if (kstart) dhead = d;
    if (rowok && hf == 0) p.delta[rs + i * bstride] = DROP ? d : (kstart ? -d : dhead - d);
    // d(coef)[h][i] = sum over rows of delta_i: one atomic per wave
    float w = (rowok && hf == 0) ? d : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
    if (p.dcoef_part) {
      // one slot per (h, i, b, 32-row block): every slot written once, summed in order later
      if (lane == 0 && qw0 < T) p.dcoef_part[(((int64_t)hh * p.cst + i) * p.B + b) * ((T + 31) / 32) + qw0 / 32] = w;
    } else if (lane == 0 && qw0 < T) {
      atomicAdd(p.dcoef + hh * p.cst + i, w);
    }
  }

  if constexpr (!QREG) {
#pragma unroll
    for (int i = NQR; i < N; ++i)
      stage<E, QP, BM, HS, NTHR>(Qs + (i - NQR) * BM * QP, gq + i * p.q.si, p.q.st, q0, T - 1, tid);
  }
  const int tile_pieces = SRD ? KR::pieces(wave)
                              : N * stage_pieces<E, HSP, BN, HS, NW>(wave) + stage_pieces<E, DVP, BN, DV, NW>(wave);
  if constexpr (!EARLY)
    for (int j = 0; j < NS - 1; ++j)
      if (j < ntiles) stage_kv(j, j);
  // (EARLY: younger loads and stores follow the ring's pieces, so this waits for at least them)
  wait_vm(tile_pieces * max(0, min(NS - 1, ntiles) - 1));
  lds_barrier();
  // SEED: the LDS-resident Q_i rows pre-scaled by sl2 once; the seed fragments
  frag f_one = O::zero(), f_lse[SEED ? N : 1], f_dp = O::zero();
  float ddel[N];
  if constexpr (SEED) {
    if constexpr (!QREG && N > NQR) {
      scale_lds<E, NTHR>(Qs, CF::nQ, p.sl2, tid);
      lds_barrier();
    }
    if (hf == 0) { f_one[0] = (E)1.f; f_one[1] = (E)1.f; }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      f_lse[i] = seed_frag<E>(lse[i], hf);
      ddel[i] = del[0] - del[i];
    }
    f_dp = seed_frag<E>(-del[0], hf);
  }

  f32x16 dq[N][NHB];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int d = 0; d < NHB; ++d) dq[i][d] = f32x16{};
  const bool wave_live = qw0 < T;

  // unmasked loop, then the block's diagonal / tail tiles (see attn_fwd_kernel)
  // per-lane LDS read bases kept in registers across the loop (see attn_dkdv_kernel);
  // with dropout they are re-derived per step (fewer spills)
  int LrV = 0, LrK = 0, LrQ = 0, LtK = 0;
  // XA (see attn_dkdv_kernel): the ring slot's base added once per step, the k-step XOR after it
  constexpr int XMAX = 32 * ((NSV > NSQ ? NSV : NSQ) - 1) + 64 * (NHB - 1) + 32;
  constexpr int XM = XMAX < 256 ? 256 : (XMAX < 512 ? 512 : 1024);
  constexpr bool XA = !DROP && SRD && sizeof(E) == 2 && (CF::nQ * (int)sizeof(E)) % XM == 0 &&
                      (CF::nK * (int)sizeof(E)) % XM == 0 && (CF::nV * (int)sizeof(E)) % XM == 0;
  if constexpr (sizeof(E) == 2) {
    LrV = row_lane<VI::ROWB>(lane); LrK = row_lane<KI::ROWB>(lane); LrQ = row_lane<QI::ROWB>(lane);
    LtK = tr_lane<KI::ROWB>(lane);
  }
  Stamps<5> st;   // diagnostic builds only (DTA_STAMPS): dma_issue | dP | S,dS,dQ of every branch | wait_vm | barrier
  auto step = [&](int kt, auto MASKED) {
    constexpr bool MASK = decltype(MASKED)::value;
    // keep lane-derived addresses loop-variant: recomputed per tile instead of
    // hoisted into (spilled) registers across the whole loop
    asm volatile("" : "+v"(lane));
    if constexpr (!DROP && sizeof(E) == 2) {
      asm volatile("" : "+v"(LrV), "+v"(LrK), "+v"(LtK));
      if constexpr (QI::ROWB == KI::ROWB) LrQ = LrK;
      else asm volatile("" : "+v"(LrQ));
    } else if constexpr (sizeof(E) == 2) {
      LrV = row_lane<VI::ROWB>(lane); LrK = row_lane<KI::ROWB>(lane); LrQ = row_lane<QI::ROWB>(lane);
      LtK = tr_lane<KI::ROWB>(lane);
    }
    tid = (wave << 6) + lane; hf = lane >> 5; c32 = lane & 31;
    qrow = qw0 + c32;
    const int buf = kt % NS;
    if (kt + NS - 1 < ntiles) stage_kv(kt + NS - 1, (kt + NS - 1) % NS);
    st.lap<0>();
    if constexpr (DTA_DQ_IGLP >= 0) __builtin_amdgcn_iglp_opt(DTA_DQ_IGLP >= 0 ? DTA_DQ_IGLP : 0);   // A/B: LLVM's MFMA / LDS interleave strategy
    const int k0 = kt * BN;
    if (wave_live && k0 <= qw0 + 31) {
      const E* Kc = Kb + buf * CF::nK;
      const E* Vc = Vb + buf * CF::nV;
      unsigned bV = 0, bK = 0, tK = 0;
      if constexpr (XA) {
        bV = LrV + lds_addr(Vc); bK = LrK + lds_addr(Kc); tK = LtK + lds_addr(Kc);
      }
      {
        f32x16 dp[NKB];
        if constexpr (sizeof(E) == 2) {
          const int Lv = LrV;
          const char* vbase = reinterpret_cast<const char*>(Vc);
#pragma unroll
          for (int kb = 0; kb < NKB; ++kb) dp[kb] = SEED ? O::mma(f_one, f_dp, f32x16{}) : f32x16{};
          if constexpr (XA && DTA_DQ_PIPE > 0 && !SPILLS) {
            // V fragments read DTA_DQ_PIPE MFMAs ahead (k-step major, key block minor)
            constexpr int NIT = NSV * NKB, D = DTA_DQ_PIPE;
            i32x4 vb[D + 1];
            auto issue = [&](auto J) {
              constexpr int j = decltype(J)::value;
              ds128<(j % NKB) * 32 * VI::ROWB>(vb[j % (D + 1)], bV ^ (32 * (j / NKB)));
            };
            sfor<(D < NIT ? D : NIT)>([&](auto J) { issue(J); });
            sfor<NIT>([&](auto J) {
              constexpr int j = decltype(J)::value;
              if constexpr (j + D < NIT) issue(std::integral_constant<int, j + D>{});
              lgkm_wait<(j + D < NIT ? D : NIT - 1 - j)>();
              asm volatile("" : "+v"(vb[j % (D + 1)]));
              dp[j % NKB] = O::mma(__builtin_bit_cast(frag, vb[j % (D + 1)]), df[j / NKB], dp[j % NKB]);
            });
          } else
#pragma unroll
          for (int s = 0; s < NSV; ++s) {
            const int o = Lv ^ (32 * s);
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) {
              if constexpr (XA) dp[kb] = O::mma(lds_at<frag>(bV ^ (32 * s), kb * 32 * VI::ROWB), df[s], dp[kb]);
              else dp[kb] = O::mma(*reinterpret_cast<const frag*>(vbase + kb * 32 * VI::ROWB + o), df[s], dp[kb]);
            }
          }

        } else {
#pragma unroll
          for (int kb = 0; kb < NKB; ++kb) {
            dp[kb] = f32x16{};
#pragma unroll
            for (int s = 0; s < NSV; ++s) dp[kb] = O::mma(VI::row(Vc, kb * 32 + c32, s, hf), df[s], dp[kb]);
          }
        }
        st.lap<1>();
        sfor<N>([&](auto I_) {
          constexpr int i = decltype(I_)::value;
          const E* Ki = Kc + i * BN * HSP;
          f32x16 sa[NKB];
          if constexpr (XA && DTA_DQ_PIPE > 0 && !SPILLS) {
            // S'_i chain with its operand reads DTA_DQ_PIPE reads ahead of the MFMAs
            constexpr int QL = i >= NQR ? 1 : 0;
            constexpr int KOFF = i * BN * HSP * (int)sizeof(E), QOFF = (i >= NQR ? i - NQR : 0) * BM * QP * (int)sizeof(E);
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) sa[kb] = SEED ? O::mma(f_one, f_lse[SEED ? i : 0], f32x16{}) : f32x16{};
            s_chain_pipe<E, NSQ, NKB, QL, DTA_DQ_PIPE, KOFF, QOFF, KI::ROWB>(
                sa, bK, lds_addr(Qs) + wave * 32 * QI::ROWB + LrQ, qf[i < NQR ? i : 0]);
          } else if constexpr (sizeof(E) == 2) {
            const int Lr = LrK;
            const char* kbase = reinterpret_cast<const char*>(Ki);
            const char* qbase = reinterpret_cast<const char*>(Qs + (i >= NQR ? i - NQR : 0) * BM * QP) +
                                wave * 32 * QI::ROWB;
            const int Lq = LrQ;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) sa[kb] = SEED ? O::mma(f_one, f_lse[SEED ? i : 0], f32x16{}) : f32x16{};
#pragma unroll
            for (int s = 0; s < NSQ; ++s) {
              frag qb;
              if (i < NQR) qb = qf[i < NQR ? i : 0][s];
              else qb = *reinterpret_cast<const frag*>(qbase + (Lq ^ (32 * s)));
#pragma unroll
              for (int kb = 0; kb < NKB; ++kb) {
                if constexpr (XA)
                  sa[kb] = O::mma(lds_at<frag>(bK ^ (32 * s), (i * BN * HSP) * (int)sizeof(E) + kb * 32 * KI::ROWB), qb,
                                  sa[kb]);
                else
                  sa[kb] = O::mma(*reinterpret_cast<const frag*>(kbase + kb * 32 * KI::ROWB + (Lr ^ (32 * s))), qb, sa[kb]);
              }
            }
          } else {
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) {
              sa[kb] = f32x16{};
#pragma unroll
              for (int s = 0; s < NSQ; ++s) {
                frag qb;
                if (i < NQR) qb = qf[i < NQR ? i : 0][s];
                else qb = QI::row(Qs + (i >= NQR ? i - NQR : 0) * BM * QP, wave * 32 + c32, s, hf);
                sa[kb] = O::mma(KI::row(Ki, kb * 32 + c32, s, hf), qb, sa[kb]);
              }
            }
          }
          // DTA_DQ_TR_EARLY: the first d-block's transposed K_i reads of dQ_i issued here, ahead
          // of the softmax VALU below (16 more VGPRs live across it)
          constexpr bool TRE = DTA_DQ_TR_EARLY && sizeof(E) == 2 && !SPILLS;
          lds64 rk0[NKB][4];      // (full size even when unused: referenced in a generic lambda)
          if constexpr (TRE) {
            const unsigned kbse = lds_addr(Ki);
            const unsigned a0 = XA ? tK + (unsigned)(i * BN * HSP * (int)sizeof(E)) : kbse + LtK;
            const unsigned a1 = XA ? (tK ^ 32) + (unsigned)(i * BN * HSP * (int)sizeof(E)) : kbse + (LtK ^ 32);
            sfor<NKB>([&](auto KB) { tr_issue<KI::ROWB, 32 * decltype(KB)::value>(rk0[decltype(KB)::value], a0, a1); });
          }
          // dS^T = c_i P^T (dP^T - delta_i) = P^T * (c_i dP^T - c_i delta_i)
          const float li = lse[i], ci = coef[i], cdi = coef[i] * del[i];
          const int lim = min(qrow, T - 1) - k0 - 4 * hf;
          if constexpr (SEED) {
            // sa = S'_i (seeded with -LSE_i), dp = dP - delta_0: dS_i / c_i
            const float dd = ddel[i];
            // DTA_DQ_EXPG exps issued before their products: a product right behind its
            // exp waits a state on the transcendental result (s_nop)
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
              for (int r0 = 0; r0 < 16; r0 += DTA_DQ_EXPG) {
                float pr[DTA_DQ_EXPG];
#pragma unroll
                for (int u = 0; u < DTA_DQ_EXPG; ++u) {
                  const int r = r0 + u;
                  float arg = sa[kb][r];
                  if constexpr (MASK) arg = (kb * 32 + (r & 3) + 8 * (r >> 2) > lim) ? -INFINITY : arg;
                  pr[u] = exp2_fast(arg);
                }
                if constexpr (DTA_DQ_PK && DTA_DQ_EXPG % 2 == 0) {
                  // two rows per v_pk_mul_f32 / v_pk_add_f32 (same fp32 arithmetic per element)
#pragma unroll
                  for (int u = 0; u < DTA_DQ_EXPG; u += 2) {
                    const int r = r0 + u;
                    const f32x2 p2 = f32x2{pr[u], pr[u + 1]}, d2 = f32x2{dp[kb][r], dp[kb][r + 1]};
                    const f32x2 s2 = i == 0 ? p2 * d2 : p2 * (d2 + f32x2{dd, dd});
                    sa[kb][r] = s2[0];
                    sa[kb][r + 1] = s2[1];
                  }
                } else {
#pragma unroll
                  for (int u = 0; u < DTA_DQ_EXPG; ++u) {
                    const int r = r0 + u;
                    sa[kb][r] = i == 0 ? pr[u] * dp[kb][r] : pr[u] * (dp[kb][r] + dd);
                  }
                }
              }
          } else {
          uint32_t dkey = 0;
          if constexpr (DROP) dkey = drop_key(p.drop_seed_lo, p.drop_seed_hi, b, hh, p.br0 + i, p.H, p.cst);
#pragma unroll
          for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              float arg = fmaf(sa[kb][r], p.sl2, li);      // li = -LSE
              if constexpr (MASK) arg = (kb * 32 + (r & 3) + 8 * (r >> 2) > lim) ? -INFINITY : arg;
              // dropout: dA = c * mask/(1-p) * dP; dS = P (dA - c delta), delta from the dropped O_i
              float cm = ci;
              if constexpr (DROP)
                cm *= drop_mul(dkey, qrow, k0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf, p.drop_thr, p.drop_scale);
              sa[kb][r] = exp2_fast(arg) * fmaf(cm, dp[kb][r], -cdi);
            }
          }
          // dQ_i^T += K_i^T dS_i^T
          if constexpr (sizeof(E) == 2) {
            const unsigned kbse = lds_addr(Ki);
            const int Lk = LtK;
            sfor<NHB>([&](auto D) {
              constexpr int d = decltype(D)::value;
              lds64 r[NKB][4];
              const unsigned a0 = XA ? (tK ^ (64 * d)) + (unsigned)(i * BN * HSP * (int)sizeof(E)) : kbse + (Lk ^ (64 * d));
              const unsigned a1 = XA ? (tK ^ (64 * d + 32)) + (unsigned)(i * BN * HSP * (int)sizeof(E))
                                     : kbse + (Lk ^ (64 * d + 32));
              if constexpr (TRE && d == 0) {
                lgkm_pin<NKB>(rk0);
#pragma unroll
                for (int kb = 0; kb < NKB; ++kb) {
                  dq[i][d] = O::mma(tr_frag<E>(rk0[kb], 0), O::template pack<0>(sa[kb]), dq[i][d]);
                  dq[i][d] = O::mma(tr_frag<E>(rk0[kb], 1), O::template pack<1>(sa[kb]), dq[i][d]);
                }
                return;
              }
              if constexpr (SPILLS) {
                sfor<NKB>([&](auto KB) { tr_load<KI::ROWB, 32 * decltype(KB)::value>(r[decltype(KB)::value], a0, a1); });
              } else {
                sfor<NKB>([&](auto KB) { tr_issue<KI::ROWB, 32 * decltype(KB)::value>(r[decltype(KB)::value], a0, a1); });
                lgkm_pin<NKB>(r);
              }
#pragma unroll
              for (int kb = 0; kb < NKB; ++kb) {
                dq[i][d] = O::mma(tr_frag<E>(r[kb], 0), O::template pack<0>(sa[kb]), dq[i][d]);
                dq[i][d] = O::mma(tr_frag<E>(r[kb], 1), O::template pack<1>(sa[kb]), dq[i][d]);
              }
            });
          } else {
#pragma unroll
            for (int d = 0; d < NHB; ++d)
#pragma unroll
              for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int s = 0; s < SPB; ++s)
                  dq[i][d] = O::mma(KI::tr_perm(Ki, kb * 32, s, hf, d * 32, lane), sa[kb][s], dq[i][d]);
          }
        });
      }
    }
    st.lap<2>();
    wait_vm(tile_pieces * max(0, min(NS - 2, ntiles - 2 - kt)));
    st.lap<3>();
    lds_barrier();
    st.lap<4>();
  };
  st.start();
  const int nfull = min(ntiles, min((q0 + 1) / BN, T / BN));
  for (int kt = 0; kt < nfull; ++kt) step(kt, std::false_type{});
  for (int kt = nfull; kt < ntiles; ++kt) step(kt, std::true_type{});
  st.flush(p.stamps, lin * NW + wave, lane);

  if (qw0 >= T) return;
  if (DTA_EPI_SKIP == 1 && p.T != -7) return;
  // bounced epilogue (see bounce_store; the ring is idle): whole-row store instructions
  constexpr bool BNC = DTA_BWD_BOUNCE && sizeof(E) == 2 && NHB % 2 == 0 && CF::bytes >= NW * 8192;
  if constexpr (BNC) {
    if (OUTF32 || t5_aligned16(p.dq, sizeof(E))) {
      float* reg = reinterpret_cast<float*>(smem) + wave * 2048;
      const int nrows = min(32, T - qw0);
      const int rrow = min(qrow, T - 1);       // RoPE table row (rows past T are not stored)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const float sc = SEED ? p.scale * coef[i] : p.scale;
        auto val = [&](int d, int g) {
          float a0 = dq[i][d][4 * g] * sc, a1 = dq[i][d][4 * g + 1] * sc;
          float a2 = dq[i][d][4 * g + 2] * sc, a3 = dq[i][d][4 * g + 3] * sc;
          if (p.rope) rope_inv4(p.rope, rrow, HS, d * 32 + 8 * g + 4 * hf, a0, a1, a2, a3);
          return f32x4{a0, a1, a2, a3};
        };
        if constexpr (OUTF32)
          bounce_store<float, NHB>(reg, lane, val, p.dq32 + ((((int64_t)b * T + qw0) * p.H + hh) * p.cst + i) * HS,
                                   (int64_t)p.H * p.cst * HS, nrows);
        else
          bounce_store<E, NHB>(reg, lane, val, reinterpret_cast<E*>(p.dq.p) + b * p.dq.sb + (int64_t)qw0 * p.dq.st +
                                                   hh * p.dq.sh + i * p.dq.si, p.dq.st, nrows);
      }
      return;
    }
  }
  if (!rowok) return;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int d = 0; d < NHB; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int e = d * 32 + 8 * g + 4 * hf;
        if (e >= HS) continue;
        const float sc = SEED ? p.scale * coef[i] : p.scale;
        float a0 = dq[i][d][4 * g] * sc, a1 = dq[i][d][4 * g + 1] * sc;
        float a2 = dq[i][d][4 * g + 2] * sc, a3 = dq[i][d][4 * g + 3] * sc;
        if (p.rope) rope_inv4(p.rope, qrow, HS, e, a0, a1, a2, a3);
        if constexpr (OUTF32) {
          store4<float>(p.dq32 + ((((int64_t)b * T + qrow) * p.H + hh) * p.cst + i) * HS + e, a0, a1, a2, a3);
        } else {
          E* gdq = reinterpret_cast<E*>(p.dq.p) + b * p.dq.sb + (int64_t)qrow * p.dq.st + hh * p.dq.sh + i * p.dq.si;
          store4<E>(gdq + e, a0, a1, a2, a3);
        }
      }
}

// One query tile of the key-major backward -- Q_i rows, dO rows, LSE rows and
// (with DELTA) c*delta rows -- streamed into one ring stage by buffer_load ... lds.
// Stage layout: [N][BQ][HSP] Q image | [BQ][DVP] dO image | [NP] lse | [NP] c*delta
// (image widths padded to a power of two, img_cols).
// Every per-lane source offset is computed once (init); a tile then costs only
// scalar descriptor setup.  Rows past T read as zeros (and are masked).
template <class E, int HS, int N, int DV, int NW, bool DELTA, int BQ_ = 32, bool ROWS = true>
struct TileRing {
  static constexpr int ES = (int)sizeof(E), BQ = BQ_;
  static constexpr int NP = (N * BQ + 63) / 64 * 64;
  static constexpr int HSP = img_cols(HS), DVP = img_cols(DV);
  static constexpr int QB = BQ * HSP * ES, DB = BQ * DVP * ES;
  // ROWS = false: the LSE / delta row vectors are not staged (read from global memory)
  static constexpr int OFF_D = N * QB, OFF_L = OFF_D + DB, OFF_G = OFF_L + NP * 4;
  static constexpr int SB = ROWS ? OFF_G + NP * 4 : OFF_L;
  static constexpr int PQ = N * QB / 1024, PD = DB / 1024, PL = NP / 64;
  static constexpr int NPC = PQ + PD + (ROWS ? (DELTA ? 2 : 1) * PL : 0);     // DMA pieces per stage
  static constexpr int MYP = (NPC + NW - 1) / NW;                  // piece j goes to wave j % NW
  static constexpr bool ok = ES == 2 && HS >= 32 && QB % 1024 == 0 && DB % 1024 == 0;

  __device__ static int pieces(int wave) { return NPC / NW + (wave < NPC % NW ? 1 : 0); }

  // byte offset of lane's 16 (or 4) bytes of piece j from the tile's row base
  // (pad chunks of a padded image read the row's first chunk: in bounds, never used)
  __device__ static uint32_t offq(const BwdParams& p, int j, int lane) {           // j < PQ
    using QI = Img<E, HSP>;
    const int i = j / (QB / 1024), pb = (j % (QB / 1024)) * 1024 + lane * 16;
    const int r = pb / QI::ROWB;
    int c = ((pb % QI::ROWB) >> 4) ^ swz<QI::ROWB>(r);
    if constexpr (HSP != HS) c = c * 16 < HS * ES ? c : 0;
    return (uint32_t)(r * (uint32_t)(p.q.st * ES) + (uint32_t)(i * p.q.si * ES) + c * 16);
  }
  __device__ static uint32_t offd(const BwdParams& p, int j, int lane) {           // PQ <= j < PQ + PD
    using DI = Img<E, DVP>;
    const int pb = (j - PQ) * 1024 + lane * 16;
    const int r = pb / DI::ROWB;
    int c = ((pb % DI::ROWB) >> 4) ^ swz<DI::ROWB>(r);
    if constexpr (DVP != DV) c = c * 16 < DV * ES ? c : 0;
    return (uint32_t)(r * (uint32_t)(p.dout.st * ES) + c * 16);
  }
  __device__ static uint32_t offr(int j, int lane, int64_t bstride) {              // row-vector pieces
    const int e = ((j - PQ - PD) % PL) * 64 + lane;
    const int i = min(e / BQ, N - 1), r = e % BQ;
    return (uint32_t)((i * (uint32_t)bstride + r) * 4);
  }
  // Wave w issues pieces j = u * NW + w; a slot u whose NW pieces are all of one kind
  // is resolved at compile time (no per-piece scalar branching).
  // per-lane source offsets of this wave's pieces: the same for every tile (VGPRs, once)
  __device__ static void offsets(const BwdParams& p, int64_t bstride, int wave, int lane, uint32_t (&off)[MYP]) {
    sfor<MYP>([&](auto U) {
      constexpr int u = decltype(U)::value;
      const int j = u * NW + wave;
      if constexpr ((u + 1) * NW <= PQ) off[u] = offq(p, j, lane);
      else if constexpr (u * NW >= PQ && (u + 1) * NW <= PQ + PD) off[u] = offd(p, j, lane);
      else off[u] = j < PQ ? offq(p, j, lane) : (j < PQ + PD ? offd(p, j, lane) : (j < NPC ? offr(j, lane, bstride) : 0u));
    });
  }
  // gq / gdo: (b, h) bases; lse / delta: (b, h) row-vector bases of branch 0
  __device__ static void issue_pre(const BwdParams& p, const E* gq, const E* gdo, const float* lse, const float* delta,
                                   int64_t bstride, int q0, int T, char* st0, int wave, const uint32_t (&off)[MYP]) {
    const int rows = T - q0;
    const E* bq = gq + (int64_t)q0 * p.q.st;
    const E* bd = gdo + (int64_t)q0 * p.dout.st;
    const uint32_t nq = (uint32_t)rows * (uint32_t)(p.q.st * ES), nd = (uint32_t)rows * (uint32_t)(p.dout.st * ES);
    const uint32_t nl = (uint32_t)(((N - 1) * bstride + rows) * 4);
    sfor<MYP>([&](auto U) {
      constexpr int u = decltype(U)::value;
      const int j = u * NW + wave;
      if constexpr ((u + 1) * NW <= PQ) {
        buf_lds16(bq, nq, st0 + j * 1024, off[u]);
      } else if constexpr (u * NW >= PQ && (u + 1) * NW <= PQ + PD) {
        buf_lds16(bd, nd, st0 + OFF_D + (j - PQ) * 1024, off[u]);
      } else {
        if (j < PQ) buf_lds16(bq, nq, st0 + j * 1024, off[u]);
        else if (j < PQ + PD) buf_lds16(bd, nd, st0 + OFF_D + (j - PQ) * 1024, off[u]);
#ifndef DTA_DKDV_NOROWS_PROBE
        else if (j < PQ + PD + PL) buf_lds4(lse + q0, nl, st0 + OFF_L + (j - PQ - PD) * 256, off[u]);
        else if (j < NPC) buf_lds4(delta + q0, nl, st0 + OFF_G + (j - PQ - PD - PL) * 256, off[u]);
#endif
      }
    });
  }
};

// The buffer descriptors cover [row base, T rows) of each operand: every branch's
// columns must lie inside one row stride and the extents must fit the 32-bit
// record count.  Otherwise the DMA-by-address staging runs.
inline bool ring_layout_ok(const BwdParams& p, int es) {
  const int64_t qs = p.q.st, ds = p.dout.st;
  if (qs <= 0 || ds <= 0 || p.q.si < 0) return false;
  if ((int64_t)(p.N - 1) * p.q.si + p.HS > qs || p.DV > ds) return false;
  if ((int64_t)p.T * qs * es >= (1ll << 31) || (int64_t)p.T * ds * es >= (1ll << 31)) return false;
  if ((int64_t)p.N * p.B * p.H * p.T * 4 >= (1ll << 31)) return false;
  return true;
}

// --------------------------------------------------- backward: dK, dV ---

template <class E, int HS, int N, int DV, int NW, bool PR = false, bool GRX = false>
struct DkdvCfg {
  static constexpr int LIMB = PR ? 80 * 1024 : 160 * 1024;     // PR: paired 4-wave plan, two per CU
  static constexpr int BK = NW * 32;
  // LDS image widths (img_cols): Q rows at least 32 columns (dK's transposed reads take
  // 32-column blocks); K (row reads only) and dO at their power-of-two pitch
  static constexpr int HSP = img_cols(HS < 32 ? 32 : HS), KP = img_cols(HS), DVP = img_cols(DV);
  static constexpr int BQ = 32;                            // query rows per ring stage
  static constexpr int NP = (N * BQ + 63) / 64 * 64;      // fp32 row vectors, padded to DMA pieces
  static constexpr int nQ = N * BQ * HSP;
  static constexpr int nD = BQ * DVP;
  static constexpr int nK = N * BK * KP;                   // the workgroup's K_i rows (B of S_i)
  // GR (DkdvWaves sets it where no plan fits otherwise: N = 4 at head size >= 96, fp32
  // N = 4): the LSE / delta row vectors are read from global memory instead of the ring
  static constexpr int RB = 2 * NP * 4;                    // row-vector bytes per stage
  static constexpr bool GR = GRX;
  static constexpr int NS = ring_stages_lim(nK * (int)sizeof(E), (nQ + nD) * (int)sizeof(E) + (GR ? 0 : RB), LIMB);
  static constexpr int bytes = (nK + NS * nQ + NS * nD) * (int)sizeof(E) + (GR ? 0 : NS * RB);
};

// widest key block (waves x 32 keys) whose K rows plus a 2+-stage query ring fit LDS
// accumulator budget -> whether dK and dV share one launch
template <int HS, int N, int DV>
struct DkdvSplit {
  static constexpr int HSB = (HS < 32 ? 32 : HS + 31) / 32 * 32;     // dK accumulator columns
  static constexpr bool fused = (N * HSB / 2 + DV / 2) <= 160;
};

// widest key block (waves x 32 keys) whose K rows plus a 2+-stage query ring fit
// LDS; 8 waves (two per SIMD, 256 registers each) only while the rough register
// count of a launch (dK / dV accumulators, V fragments, scores) fits them
template <class E, int HS, int N, int DV, bool NP = false>
struct DkdvWaves {
  static constexpr int LIM = 160 * 1024;
  static constexpr int HSB = DkdvSplit<HS, N, DV>::HSB;
  static constexpr int regs8 = DkdvSplit<HS, N, DV>::fused ? N * HSB / 2 + DV / 2 + DV / 4 + 88
                             : (N * HSB / 2 + DV / 4 > DV / 2 ? N * HSB / 2 + DV / 4 : DV / 2) + 88;
  static constexpr int v8 = (sizeof(E) == 2 && DkdvCfg<E, HS, N, DV, 8>::bytes <= LIM && regs8 <= 256) ? 8
                          : DkdvCfg<E, HS, N, DV, 4>::bytes <= LIM ? 4 : 2;
  // paired plan: where the 8-wave plan applies, two 4-wave workgroups per CU instead
  // (bf16 only: the fp16 paired instantiation spills 16 VGPRs)
  static constexpr bool pair = !NP && std::is_same<E, __bf16>::value && v8 == 8 &&
                               DkdvCfg<E, HS, N, DV, 4, true>::bytes <= 80 * 1024;
  static constexpr int v0 = pair ? 4 : v8;
  // no plan with the row vectors in the ring fits: two waves (one where two do not fit:
  // fp32 at head size 96), row vectors from global memory
  static constexpr bool gr = DkdvCfg<E, HS, N, DV, v0, pair>::bytes > LIM;
  static constexpr int v = !gr ? v0 : (DkdvCfg<E, HS, N, DV, 2, false, true>::bytes <= LIM ? 2 : 1);
};

template <class E, int HS, int N, int DV, int NW, bool DK, bool DVV, bool SRD, bool DROP, bool PR, bool GRX,
          bool CFOLD = false>
__global__ __launch_bounds__(NW * 64, (NW >= 8 || PR ? 2 : 1))
void attn_dkdv_kernel(BwdParams p) {
  using O = Ops<E>;
  using frag = typename O::frag;
  using CF = DkdvCfg<E, HS, N, DV, NW, PR, GRX>;
  constexpr int HSP = CF::HSP, KP = CF::KP, DVP = CF::DVP, BQ = CF::BQ, BK = CF::BK, NP = CF::NP;
  constexpr int NTHR = NW * 64;
  using QI = Img<E, HSP>;
  using DI = Img<E, DVP>;
  constexpr int KS = O::KSTEP;
  constexpr int NSQ = HS / KS, NSV = DV / KS, SPB = 32 / KS;
  constexpr int NHB = (HS + 31) / 32, NVB = DV / 32;
  // the plans that spill (16-bit head size 128 at N >= 3, the dropout plans: 8-48 VGPRs at
  // head size 64 N = 2) take compiler-tracked transposed reads (see tr_load)
  constexpr bool SPILLS = sizeof(E) == 2 && (DROP || (HS >= 128 && N >= 3) || (HS >= 192 && N >= 2));

  using KI = Img<E, KP>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  E* Ks = reinterpret_cast<E*>(smem);     // [N][BK][KP]
  E* Qb = Ks + CF::nK;                    // [NS][N][BQ][HSP]
  constexpr int NS = CF::NS;
  E* Db = Qb + NS * CF::nQ;               // [NS][BQ][DVP]
  float* Lb = reinterpret_cast<float*>(Db + NS * CF::nD);  // [NS][NP] lse
  float* Gb = Lb + NS * NP;                                 // [NS][NP] delta
  // SRD: the ring is instead NS stages of TileRing's layout, filled by buffer_load ... lds
  constexpr bool GR = CF::GR;
  using RG = TileRing<E, HS, N, DV, NW, DK, BQ, !GR>;
  char* ringb = reinterpret_cast<char*>(Qb);
  static_assert(!SRD || (RG::ok && RG::SB * NS <= CF::bytes - CF::nK * (int)sizeof(E) && RG::HSP == HSP &&
                          RG::DVP == DVP), "ring layout");

  // wave index is wave-uniform: make it provably so (SGPR), or every branch on it
  // becomes an exec-masked divergent branch
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tid = threadIdx.x, lane = tid & 63;
  int hf = lane >> 5, c32 = lane & 31;
  int bx, by, bz, lin;
  lpt_order(bx, by, bz, lin);
  const int kblk = bx;                    // key block 0 has the most query tiles: rank 0
  const int hh = by, b = bz;
  const int T = p.T;
  const int kb0 = kblk * BK, kw0 = kb0 + wave * 32;
  int krow = kw0 + c32;

  const E* gq = reinterpret_cast<const E*>(p.q.p) + b * p.q.sb + hh * p.q.sh;
  const E* gk = reinterpret_cast<const E*>(p.k.p) + b * p.k.sb + hh * p.k.sh;
  const E* gv = reinterpret_cast<const E*>(p.v.p) + b * p.v.sb + hh * p.v.sh;
  const E* gdo = reinterpret_cast<const E*>(p.dout.p) + b * p.dout.sb + hh * p.dout.sh;
  const int64_t rowvec = ((int64_t)b * p.H + hh) * T;       // [i][b][h][t] offset of (b, h)
  const int64_t bstride = (int64_t)p.B * p.H * T;

  float coef[N];
  uint32_t dkey[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    coef[i] = p.coef[hh * p.cst + i];
    dkey[i] = DROP ? drop_key(p.drop_seed_lo, p.drop_seed_hi, b, hh, p.br0 + i, p.H, p.cst) : 0u;
  }
  // CFOLD (ABI 8 lse_c, 16-bit, no dropout): the S seeds are the stored LSE_i + log2|c_i| rows
  // attn_dq wrote, so exp gives P~_i = |c_i| P_i.  dV's operand sum_i c_i P_i = s_0 (P~_0 +
  // sum_{i>=1} s_0 s_i P~_i) with s_i = sign(c_i): branch 0 needs no multiply, the dV epilogue
  // takes s_0; dS_i is accumulated as P~_i (dP - delta_i), so dK_i's epilogue takes s_i, not c_i.
  static_assert(!CFOLD || (!DROP && sizeof(E) == 2 && !GRX), "CFOLD: 16-bit plans without dropout");
  auto sgn = [](float c) { return c < 0.f ? -1.f : 1.f; };
  float wv[N];                        // pc weights: c_i, or s_0 s_i (CFOLD)
#pragma unroll
  for (int i = 0; i < N; ++i) wv[i] = CFOLD ? sgn(coef[0]) * sgn(coef[i]) : coef[i];
  const float dvsc = CFOLD ? sgn(coef[0]) : 1.f;    // dV epilogue factor
  const float* lsep = CFOLD ? p.lsec : p.lse;
  // this wave's key rows of every K_i and of V as B fragments
  // this wave's V rows as B fragments of dP = dO V^T (registers); K_i rows live in LDS
  frag vf[DK ? NSV : 1];
  if constexpr (DK) {
#pragma unroll
    for (int s = 0; s < NSV; ++s)
      vf[s] = krow < T ? O::load_global(gv + (int64_t)krow * p.v.st + s * KS + hf * O::KH) : O::zero();
  }

  // per-lane DMA source offsets of this wave's pieces, computed once (VGPRs)
  uint32_t roff[SRD ? RG::MYP : 1];
  if constexpr (SRD) RG::offsets(p, bstride, wave, lane, roff);
  auto stage_q = [&](int q0, int buf) {
    if constexpr (SRD) {
      RG::issue_pre(p, gq, gdo, lsep + rowvec, p.delta + rowvec, bstride, q0, T, ringb + buf * RG::SB, wave, roff);
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i)
        stage<E, HSP, BQ, HS, NTHR>(Qb + (buf * N + i) * BQ * HSP, gq + i * p.q.si, p.q.st, q0, T - 1, tid);
      stage<E, DVP, BQ, DV, NTHR>(Db + buf * CF::nD, gdo, p.dout.st, q0, T - 1, tid);
      if constexpr (!GR) {
        stage_rows<N, BQ, NTHR>(Lb + buf * NP, lsep + rowvec, bstride, q0, T - 1, tid);
        if constexpr (DK) stage_rows<N, BQ, NTHR>(Gb + buf * NP, p.delta + rowvec, bstride, q0, T - 1, tid);
      }
    }
  };

  f32x16 dk[DK ? N : 1][NHB];
  f32x16 dv[DVV ? NVB : 1];
#pragma unroll
  for (int i = 0; i < (DK ? N : 1); ++i)
#pragma unroll
    for (int d = 0; d < NHB; ++d) dk[i][d] = f32x16{};
#pragma unroll
  for (int d = 0; d < (DVV ? NVB : 1); ++d) dv[d] = f32x16{};

  const int ntiles = kb0 < T ? (T - kb0 + BQ - 1) / BQ : 0;
#pragma unroll
  for (int i = 0; i < N; ++i) stage<E, KP, BK, HS, NTHR>(Ks + i * BK * KP, gk + i * p.k.si, p.k.st, kb0, T - 1, tid);
  const int tile_pieces = SRD ? RG::pieces(wave)
                              : N * stage_pieces<E, HSP, BQ, HS, NW>(wave) + stage_pieces<E, DVP, BQ, DV, NW>(wave) +
                                    rows_pieces<N, BQ, NW>(wave) * (DK ? 2 : 1);
  for (int j = 0; j < NS - 1; ++j)
    if (j < ntiles) stage_q(kb0 + j * BQ, j);
  wait_vm(tile_pieces * max(0, min(NS - 1, ntiles) - 1));
  lds_barrier();
  // K_i rows scaled once by scale*log2e in place, so S'_i = Q_i (sl2 K_i)^T; the S
  // accumulators start at the tile's -LSE rows and P = exp2(S'_i) needs no fma
  scale_lds<E, NTHR>(Ks, CF::nK, p.sl2, tid);
  lds_barrier();
  const bool wave_keys = kw0 < T;

  // masked diagonal tiles, unmasked interior, masked ragged tail tile; each loop
  // is one straight-line body (both variants behind a branch spill).  Lanes with
  // key >= T only pollute their own (never stored) dK/dV columns.
  // diagnostic builds only (DTA_STAMPS): dma_issue | dP, S, dS, dK, dV | wait_vm | barrier (four sums:
  // more SGPRs spill this plan's DMA offsets)
  Stamps<4> st;
  // per-lane LDS read bases, one register each across the loop: every read of a step
  // is then one v_xad (base ^ k-step) + stage
  int LrD = 0, LrQ = 0, LrK = 0, LtQ = 0, LtD = 0;
  // XA: the stage base is added to each family's lane base once per step and the
  // k-step / d-block XOR applied after it (valid: stage bases are multiples of XM, a
  // power of two above every XOR constant); region offsets ride in DS immediates.
  // (The dynamic LDS array starts at address 0: the kernel has no static LDS.)
  constexpr int XMAX = 64 * ((NVB > NHB ? NVB : NHB) - 1) + 32 + 32 * ((NSV > NSQ ? NSV : NSQ) - 1);
  constexpr int XM = XMAX < 256 ? 256 : (XMAX < 512 ? 512 : 1024);
  constexpr bool XA = SRD && sizeof(E) == 2 && (CF::nK * (int)sizeof(E)) % XM == 0 && RG::SB % XM == 0 &&
                      QI::ROWB == KI::ROWB;
  if constexpr (sizeof(E) == 2) {
    LrD = row_lane<DI::ROWB>(lane); LrQ = row_lane<QI::ROWB>(lane); LrK = row_lane<KI::ROWB>(lane);
    LtQ = tr_lane<QI::ROWB>(lane); LtD = tr_lane<DI::ROWB>(lane);
  }
  auto step = [&](int t, auto MASKED) {
    constexpr bool MASK = decltype(MASKED)::value;
    // keep lane-derived addresses loop-variant: recomputed per tile instead of
    // hoisted into (spilled) registers across the whole loop
    asm volatile("" : "+v"(lane));
    if constexpr (sizeof(E) == 2) {
      asm volatile("" : "+v"(LrD), "+v"(LrQ), "+v"(LtQ), "+v"(LtD));
      if constexpr (QI::ROWB == KI::ROWB) LrK = LrQ;     // same row pitch (HS >= 32)
      else asm volatile("" : "+v"(LrK));
    }
    tid = (wave << 6) + lane; hf = lane >> 5; c32 = lane & 31;
    krow = kw0 + c32;
    const int buf = t % NS;
    const int q0 = kb0 + t * BQ;
    if (t + NS - 1 < ntiles) stage_q(q0 + (NS - 1) * BQ, (t + NS - 1) % NS);
    st.lap<0>();
    if constexpr (DTA_DKDV_IGLP >= 0) __builtin_amdgcn_iglp_opt(DTA_DKDV_IGLP >= 0 ? DTA_DKDV_IGLP : 0);   // A/B: LLVM's MFMA / LDS interleave strategy
    if (wave_keys && q0 + 31 >= kw0) {
      const char* sg = ringb + buf * RG::SB;
      const E* Qc = SRD ? reinterpret_cast<const E*>(sg) : Qb + buf * N * BQ * HSP;
      const E* Dc = SRD ? reinterpret_cast<const E*>(sg + RG::OFF_D) : Db + buf * CF::nD;
      const float* Lc = SRD ? reinterpret_cast<const float*>(sg + RG::OFF_L) : Lb + buf * NP;
      const float* Gc = SRD ? reinterpret_cast<const float*>(sg + RG::OFF_G) : Gb + buf * NP;
      // rows 8g + 4hf .. + 3 of branch i's LSE / delta vector: from the ring, or (GR) from
      // global memory, rows past T clamped (they are masked)
      auto rows4 = [&](const float* ring, const float* glb, int i, int g) -> f32x4 {
        if constexpr (GR) {
          const float* v = glb + rowvec + i * bstride;
          const int r0 = q0 + 8 * g + 4 * hf;
          return f32x4{v[min(r0, T - 1)], v[min(r0 + 1, T - 1)], v[min(r0 + 2, T - 1)], v[min(r0 + 3, T - 1)]};
        } else {
          return *reinterpret_cast<const f32x4*>(ring + i * BQ + 8 * g + 4 * hf);
        }
      };
      unsigned bQ = 0, bD = 0, tQ = 0, tD = 0;
      if constexpr (XA) {
        const unsigned sb = lds_addr(sg);
        bQ = LrQ + sb; bD = LrD + sb; tQ = LtQ + sb; tD = LtD + sb;
      }
      {
      // Gc rows (attn_dq): without dropout -delta_0 | delta_0 - delta_i, and the dP
      // accumulator starts at -delta_0, so dS_0 / c_0 = P_0 dpa and dS_i / c_i =
      // P_i (dpa + delta_0 - delta_i); with dropout delta_i and an unseeded dP
      f32x16 dpa = f32x16{};
      if constexpr (DK && !DROP) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 g4 = rows4(Gc, p.delta, 0, g);
#pragma unroll
          for (int j = 0; j < 4; ++j) dpa[4 * g + j] = g4[j];
        }
      }
      if constexpr (DK) {
        if constexpr (sizeof(E) == 2) {
          const int Ld = LrD;
          const char* dbase = reinterpret_cast<const char*>(Dc);
#pragma unroll
          for (int s = 0; s < NSV; ++s) {
            if constexpr (XA) dpa = O::mma(lds_at<frag>(bD ^ (32 * s), RG::OFF_D), vf[s], dpa);
            else dpa = O::mma(*reinterpret_cast<const frag*>(dbase + (Ld ^ (32 * s))), vf[s], dpa);
          }
        } else {
#pragma unroll
          for (int s = 0; s < NSV; ++s) dpa = O::mma(DI::row(Dc, c32, s, hf), vf[s], dpa);
        }
      }
      f32x16 pc = f32x16{};
      // rows q0 + rowof(r) > lim are masked: query < key, or past the end
      const int lim_lo = krow - q0 - 4 * hf;          // masked if rowof_c < lim_lo (query < key)
      const int lim_hi = T - 1 - q0 - 4 * hf;         // masked if rowof_c > lim_hi (query >= T)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        // CFOLD: keep the branches in program order (with branch 0's dV operand free of a multiply
        // the scheduler otherwise hoists the next branch's score chain and spills)
        if constexpr (CFOLD) if (i > 0) __builtin_amdgcn_sched_barrier(0);
        // S'_i accumulator seeded with the -LSE rows (K_i is pre-scaled by sl2)
        f32x16 sa;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 l4 = rows4(Lc, lsep, i, g);
#pragma unroll
          for (int j = 0; j < 4; ++j) sa[4 * g + j] = l4[j];
        }
        const E* Qi = Qc + i * BQ * HSP;
        if constexpr (sizeof(E) == 2) {
          const int Lq = LrQ, Lk = LrK;
          const char* qbase = reinterpret_cast<const char*>(Qi);
          const char* kbase = reinterpret_cast<const char*>(Ks + i * BK * KP) + wave * 32 * KI::ROWB;
          // operand reads of this branch's S ahead of its MFMA chain (see attn_fwd_kernel)
          frag qfr[NSQ], kfr[NSQ];
#pragma unroll
          for (int s = 0; s < NSQ; ++s) {
            if constexpr (XA) qfr[s] = lds_at<frag>(bQ ^ (32 * s), i * RG::QB);
            else qfr[s] = *reinterpret_cast<const frag*>(qbase + (Lq ^ (32 * s)));
            kfr[s] = *reinterpret_cast<const frag*>(kbase + (Lk ^ (32 * s)));
          }
#pragma unroll
          for (int s = 0; s < NSQ; ++s) sa = O::mma(qfr[s], kfr[s], sa);
          __builtin_amdgcn_sched_group_barrier(0x100, 2 * NSQ, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NSQ, 0);
        } else {
#pragma unroll
          for (int s = 0; s < NSQ; ++s)
            sa = O::mma(QI::row(Qi, c32, s, hf), KI::row(Ks + i * BK * KP, wave * 32 + c32, s, hf), sa);
        }
        // DTA_DKDV_TR_EARLY: the transposed Q_i reads of dK_i issued here, ahead of the softmax
        // VALU below, so their LDS latency hides behind it (16 more VGPRs live across it)
        constexpr bool TRE = DTA_DKDV_TR_EARLY && DK && sizeof(E) == 2 && !SPILLS;
        lds64 rq[TRE ? NHB : 1][4];
        if constexpr (TRE) {
          const unsigned qb = lds_addr(Qi);
          const int Lq = LtQ;
          sfor<NHB>([&](auto D) {
            constexpr int d = decltype(D)::value;
            if constexpr (XA) tr_issue<QI::ROWB, 0>(rq[d], (tQ ^ (64 * d)) + i * RG::QB, (tQ ^ (64 * d + 32)) + i * RG::QB);
            else tr_issue<QI::ROWB, 0>(rq[d], qb + (Lq ^ (64 * d)), qb + (Lq ^ (64 * d + 32)));
          });
        }
        // sa[r] = S'_i[q0 + rowof(r)][krow] - LSE; rows 4g..4g+3 of a lane are consecutive
        constexpr bool PK = DTA_DKDV_PK && !DROP && DK && CFOLD;   // (the unfolded SRD plan spills 18 VGPRs with it)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 d4 = f32x4{};
          if constexpr (DK) if (DROP || i > 0) d4 = rows4(Gc, p.delta, i, g);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * g + j;
            float arg = sa[r];
            if constexpr (MASK) {
              const int rc = (r & 3) + 8 * (r >> 2);
              arg = (rc < lim_lo || rc > lim_hi) ? -INFINITY : arg;
            }
            const float pr = exp2_fast(arg);
            if constexpr (DROP) {
              // this map element's kept weight mask/(1-p)
              const float mk = drop_mul(dkey[i], q0 + (r & 3) + 8 * (r >> 2) + 4 * hf, krow, p.drop_thr, p.drop_scale);
              if constexpr (DVV) pc[r] = fmaf(coef[i] * mk, pr, pc[r]);
              if constexpr (DK) sa[r] = pr * fmaf(mk, dpa[r], -d4[j]);
            } else if constexpr (PK) {
              sa[r] = pr;                 // the pair math below, two rows per packed op
            } else {
              if constexpr (DVV) pc[r] = i == 0 ? (CFOLD ? pr : wv[0] * pr) : fmaf(wv[i], pr, pc[r]);
              if constexpr (DK) sa[r] = i == 0 ? pr * dpa[r] : pr * (dpa[r] + d4[j]);
            }
          }
          if constexpr (PK) {
            // v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32: two rows per VALU issue (the same
            // fp32 arithmetic per element, so results are bitwise those of the scalar form)
#pragma unroll
            for (int j = 0; j < 4; j += 2) {
              const int r = 4 * g + j;
              const f32x2 pr2 = f32x2{sa[r], sa[r + 1]};
              const f32x2 dp2 = f32x2{dpa[r], dpa[r + 1]};
              if constexpr (DVV) {
                f32x2 pc2 = f32x2{pc[r], pc[r + 1]};
                if (i == 0) pc2 = CFOLD ? pr2 : f32x2{wv[0], wv[0]} * pr2;
                else pc2 = __builtin_elementwise_fma(f32x2{wv[i], wv[i]}, pr2, pc2);
                pc[r] = pc2[0]; pc[r + 1] = pc2[1];
              }
              f32x2 s2;
              if (i == 0) s2 = pr2 * dp2;
              else s2 = pr2 * (dp2 + f32x2{d4[j], d4[j + 1]});
              sa[r] = s2[0]; sa[r + 1] = s2[1];
            }
          }
        }
        if constexpr (TRE) {
          lgkm_pin<NHB>(rq);
          const frag p0 = O::template pack<0>(sa), p1 = O::template pack<1>(sa);
#pragma unroll
          for (int d = 0; d < NHB; ++d) {
            dk[i][d] = O::mma(tr_frag<E>(rq[d], 0), p0, dk[i][d]);
            dk[i][d] = O::mma(tr_frag<E>(rq[d], 1), p1, dk[i][d]);
          }
        } else if constexpr (DK) {
          if constexpr (sizeof(E) == 2) {
            const unsigned qb = lds_addr(Qi);
            const int Lq = LtQ;
            lds64 r[NHB][4];
            sfor<NHB>([&](auto D) {
              constexpr int d = decltype(D)::value;
              if constexpr (SPILLS) {
                if constexpr (XA) tr_load<QI::ROWB, 0>(r[d], (tQ ^ (64 * d)) + i * RG::QB, (tQ ^ (64 * d + 32)) + i * RG::QB);
                else tr_load<QI::ROWB, 0>(r[d], qb + (Lq ^ (64 * d)), qb + (Lq ^ (64 * d + 32)));
              } else {
                if constexpr (XA) tr_issue<QI::ROWB, 0>(r[d], (tQ ^ (64 * d)) + i * RG::QB, (tQ ^ (64 * d + 32)) + i * RG::QB);
                else tr_issue<QI::ROWB, 0>(r[d], qb + (Lq ^ (64 * d)), qb + (Lq ^ (64 * d + 32)));
              }
            });
            if constexpr (!SPILLS) lgkm_pin<NHB>(r);
            const frag p0 = O::template pack<0>(sa), p1 = O::template pack<1>(sa);
#pragma unroll
            for (int d = 0; d < NHB; ++d) {
              dk[i][d] = O::mma(tr_frag<E>(r[d], 0), p0, dk[i][d]);
              dk[i][d] = O::mma(tr_frag<E>(r[d], 1), p1, dk[i][d]);
            }
          } else {
#pragma unroll
            for (int d = 0; d < NHB; ++d)
#pragma unroll
              for (int s = 0; s < SPB; ++s) dk[i][d] = O::mma(QI::tr_perm(Qi, 0, s, hf, d * 32, lane), sa[s], dk[i][d]);
          }
        }
      }
      if constexpr (DVV) {
        if constexpr (sizeof(E) == 2) {
          const unsigned db = lds_addr(Dc);
          const int Ld = LtD;
          const frag p0 = O::template pack<0>(pc), p1 = O::template pack<1>(pc);
          constexpr int NP2 = NVB >= 2 ? 2 : 1;       // d-blocks per LDS read batch
          auto dv_blocks = [&](auto D0, auto NB) {
            constexpr int d0 = decltype(D0)::value, nb = decltype(NB)::value;
            lds64 r[nb][4];
            sfor<nb>([&](auto E2) {
              constexpr int d = d0 + decltype(E2)::value;
              if constexpr (SPILLS) {
                if constexpr (XA) tr_load<DI::ROWB, 0, RG::OFF_D>(r[decltype(E2)::value], tD ^ (64 * d), tD ^ (64 * d + 32));
                else tr_load<DI::ROWB, 0>(r[decltype(E2)::value], db + (Ld ^ (64 * d)), db + (Ld ^ (64 * d + 32)));
              } else {
                if constexpr (XA) tr_issue<DI::ROWB, 0, RG::OFF_D>(r[decltype(E2)::value], tD ^ (64 * d), tD ^ (64 * d + 32));
                else tr_issue<DI::ROWB, 0>(r[decltype(E2)::value], db + (Ld ^ (64 * d)), db + (Ld ^ (64 * d + 32)));
              }
            });
            if constexpr (!SPILLS) lgkm_pin<nb>(r);
#pragma unroll
            for (int e = 0; e < nb; ++e) {
              dv[d0 + e] = O::mma(tr_frag<E>(r[e], 0), p0, dv[d0 + e]);
              dv[d0 + e] = O::mma(tr_frag<E>(r[e], 1), p1, dv[d0 + e]);
            }
          };
          sfor<NVB / NP2>([&](auto D2) {
            dv_blocks(std::integral_constant<int, NP2 * decltype(D2)::value>{}, std::integral_constant<int, NP2>{});
          });
          // an odd block count (dv = 96): the last 32 columns on their own
          if constexpr (NVB % NP2) dv_blocks(std::integral_constant<int, NVB - 1>{}, std::integral_constant<int, 1>{});
        } else {
#pragma unroll
          for (int d = 0; d < NVB; ++d)
#pragma unroll
            for (int s = 0; s < SPB; ++s) dv[d] = O::mma(DI::tr_perm(Dc, 0, s, hf, d * 32, lane), pc[s], dv[d]);
        }
      }
      }
    }
    st.lap<1>();
    wait_vm(tile_pieces * max(0, min(NS - 2, ntiles - 2 - t)));
    st.lap<2>();
    lds_barrier();
    st.lap<3>();
  };
  st.start();
  const int thead = min(ntiles, (BK - 2) / BQ + 1);                  // q0 < kb0 + BK - 1
  const int ttail = max(thead, ntiles - ((T - kb0) % BQ != 0 ? 1 : 0));  // q0 + BQ > T
  for (int t = 0; t < thead; ++t) step(t, std::true_type{});
  for (int t = thead; t < ttail; ++t) step(t, std::false_type{});
  for (int t = ttail; t < ntiles; ++t) step(t, std::true_type{});
  st.flush(p.stamps, lin * NW + wave, lane);

  if (!wave_keys) return;
  if (DTA_EPI_SKIP == 1 && p.T != -7) return;
  // bounced epilogue (see bounce_store; the ring and the K_i rows are idle): dK, and dV
  // unless it adds to an earlier branch group's partial
  constexpr bool BNC = DTA_BWD_BOUNCE && sizeof(E) == 2 && (!DK || NHB % 2 == 0) && (!DVV || NVB % 2 == 0) &&
                       CF::bytes >= NW * 8192;
  if constexpr (BNC) {
    float* g32 = p.dv32 ? p.dv32 + (((int64_t)b * p.T + kw0) * p.H + hh) * p.DV : nullptr;
    const bool to32 = g32 != nullptr && !p.dv_last;
    if ((!DK || t5_aligned16(p.dk, sizeof(E))) && (!DVV || p.dv_acc || to32 || t5_aligned16(p.dv, sizeof(E)))) {
      float* reg = reinterpret_cast<float*>(smem) + wave * 2048;
      const int nrows = min(32, T - kw0);
      const int rrow = min(krow, T - 1);       // RoPE table row (rows past T are not stored)
      if constexpr (DK) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
          const float sc = p.scale * (CFOLD ? sgn(coef[i]) : coef[i]);   // dS_i was accumulated without c_i (CFOLD: |c_i| in)
          bounce_store<E, NHB>(reg, lane, [&](int d, int g) {
            float a0 = dk[i][d][4 * g] * sc, a1 = dk[i][d][4 * g + 1] * sc;
            float a2 = dk[i][d][4 * g + 2] * sc, a3 = dk[i][d][4 * g + 3] * sc;
            if (p.rope) rope_inv4(p.rope, rrow, HS, d * 32 + 8 * g + 4 * hf, a0, a1, a2, a3);
            return f32x4{a0, a1, a2, a3};
          }, reinterpret_cast<E*>(p.dk.p) + b * p.dk.sb + (int64_t)kw0 * p.dk.st + hh * p.dk.sh + i * p.dk.si,
             p.dk.st, nrows);
        }
      }
      if constexpr (DVV) {
        if (!p.dv_acc) {
          auto val = [&](int d, int g) {
            return f32x4{dv[d][4 * g] * dvsc, dv[d][4 * g + 1] * dvsc, dv[d][4 * g + 2] * dvsc, dv[d][4 * g + 3] * dvsc};
          };
          if (to32) bounce_store<float, NVB>(reg, lane, val, g32, (int64_t)p.H * p.DV, nrows);
          else bounce_store<E, NVB>(reg, lane, val, reinterpret_cast<E*>(p.dv.p) + b * p.dv.sb + (int64_t)kw0 * p.dv.st +
                                                       hh * p.dv.sh, p.dv.st, nrows);
          return;
        }
      } else {
        return;
      }
      // dV of a later branch group: the per-lane read-add-store below, after the bounced dK
      if (krow >= T) return;
      float* g32r = p.dv32 ? p.dv32 + (((int64_t)b * p.T + krow) * p.H + hh) * p.DV : nullptr;
      E* gdv = reinterpret_cast<E*>(p.dv.p) + b * p.dv.sb + (int64_t)krow * p.dv.st + hh * p.dv.sh;
#pragma unroll
      for (int d = 0; d < (DVV ? NVB : 1); ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int e = d * 32 + 8 * g + 4 * hf;
          float a0 = dv[d][4 * g] * dvsc, a1 = dv[d][4 * g + 1] * dvsc, a2 = dv[d][4 * g + 2] * dvsc,
                a3 = dv[d][4 * g + 3] * dvsc;
          if (g32r) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(g32r + e);
            a0 += v[0]; a1 += v[1]; a2 += v[2]; a3 += v[3];
          } else {
            a0 += (float)gdv[e]; a1 += (float)gdv[e + 1]; a2 += (float)gdv[e + 2]; a3 += (float)gdv[e + 3];
          }
          if (to32) store4<float>(g32r + e, a0, a1, a2, a3);
          else store4<E>(gdv + e, a0, a1, a2, a3);
        }
      return;
    }
  }
  if (krow >= T) return;
  if constexpr (DK) {
    E* gdk = reinterpret_cast<E*>(p.dk.p) + b * p.dk.sb + (int64_t)krow * p.dk.st + hh * p.dk.sh;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const float sc = p.scale * (CFOLD ? sgn(coef[i]) : coef[i]);   // dS_i was accumulated without c_i (CFOLD: |c_i| in)
#pragma unroll
      for (int d = 0; d < NHB; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int e = d * 32 + 8 * g + 4 * hf;
          if (e < HS) {
            float a0 = dk[i][d][4 * g] * sc, a1 = dk[i][d][4 * g + 1] * sc;
            float a2 = dk[i][d][4 * g + 2] * sc, a3 = dk[i][d][4 * g + 3] * sc;
            if (p.rope) rope_inv4(p.rope, krow, HS, e, a0, a1, a2, a3);
            store4<E>(gdk + i * p.dk.si + e, a0, a1, a2, a3);
          }
        }
    }
  }
  if constexpr (DVV) {
    E* gdv = reinterpret_cast<E*>(p.dv.p) + b * p.dv.sb + (int64_t)krow * p.dv.st + hh * p.dv.sh;
    // branch groups with an fp32 dV workspace (dv32): every group but the last keeps the
    // running sum there, the last adds it and does the only rounding to E
    float* g32 = p.dv32 ? p.dv32 + (((int64_t)b * p.T + krow) * p.H + hh) * p.DV : nullptr;
    const bool to32 = g32 != nullptr && !p.dv_last;
#pragma unroll
    for (int d = 0; d < NVB; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int e = d * 32 + 8 * g + 4 * hf;
        float a0 = dv[d][4 * g] * dvsc, a1 = dv[d][4 * g + 1] * dvsc, a2 = dv[d][4 * g + 2] * dvsc,
              a3 = dv[d][4 * g + 3] * dvsc;
        if (p.dv_acc) {        // a later branch group: dV = sum over every group's branches
          if (g32) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(g32 + e);
            a0 += v[0]; a1 += v[1]; a2 += v[2]; a3 += v[3];
          } else {
            a0 += (float)gdv[e]; a1 += (float)gdv[e + 1]; a2 += (float)gdv[e + 2]; a3 += (float)gdv[e + 3];
          }
        }
        if (to32) store4<float>(g32 + e, a0, a1, a2, a3);
        else store4<E>(gdv + e, a0, a1, a2, a3);
      }
  }
}

// ------------------------------------------------------------ launchers ---
template <class K>
static inline int set_smem(K kernel, int bytes) {
  if (bytes > 65536)
    return (int)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  return 0;
}

// O = sum_i c_i O_i after a branch-split forward (HBM-bound: N + 1 passes of
// B*T*H*dv elements).  One thread per 16 bytes of an output row, fp32 sums.
// NC > 0: the branch count at compile time; 0: p.N at run time (branch counts without
// an N-branch plan, which always run branch-split).
// index split by launch-constant fast division (the int64 div / mod it replaced cost more
// VALU than the kernel's HBM time); the output is written once by whole 16-byte vectors
struct CombineDiv {
  FastDiv vpr, H, T;
};
inline CombineDiv combine_div(const FwdParams& p, int esize) {
  return CombineDiv{FastDiv((uint32_t)(p.DV / (16 / esize))), FastDiv((uint32_t)p.H), FastDiv((uint32_t)p.T)};
}
template <class E, int NC>
__global__ __launch_bounds__(256) void branch_combine_kernel(FwdParams p, CombineDiv dv) {
  const int N = NC > 0 ? NC : p.N;
  constexpr int V = 16 / (int)sizeof(E);
  typedef float f32xv __attribute__((ext_vector_type(V)));
  typedef E ev __attribute__((ext_vector_type(V)));
  const uint32_t idx = blockIdx.x * 256 + threadIdx.x;
  const uint32_t total = (uint32_t)p.B * p.T * p.H * dv.vpr.d;
  if (idx >= total) return;
  const uint32_t row = dv.vpr.div(idx);
  const int e = (int)(idx - row * dv.vpr.d) * V;
  const uint32_t bt = dv.H.div(row);
  const int hh = (int)(row - bt * p.H);
  const uint32_t b = dv.T.div(bt);
  const int t = (int)(bt - b * p.T);
  const int64_t src = b * p.obr.sb + (int64_t)t * p.obr.st + hh * p.obr.sh + e;
  f32xv acc = f32xv{};
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float c = p.coef[hh * p.cst + i];
    if constexpr (V == 8) {
      if (p.ob16) {                                                          // fp16 O_i
        float x[8];
        load_ob8(p.obr.p, src + i * p.obr.si, true, x);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = fmaf(c, x[j], acc[j]);
        continue;
      }
    }
    const f32xv x = *reinterpret_cast<const f32xv*>(reinterpret_cast<const float*>(p.obr.p) + src + i * p.obr.si);
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = fmaf(c, x[j], acc[j]);
  }
  ev y;
#pragma unroll
  for (int j = 0; j < V; ++j) y[j] = (E)acc[j];
  __builtin_nontemporal_store(y, reinterpret_cast<ev*>(reinterpret_cast<E*>(p.o.p) + b * p.o.sb + (int64_t)t * p.o.st +
                                                       hh * p.o.sh + e));
}

// Branch-split forward policy: workgroups that hold ONE branch over the whole dv instead
// of all N branches over a dv chunk.  Auto (DTA_FWD_BSPLIT unset / -1): wherever the
// N-branch plan splits dv into chunks (each chunk redoes every branch's QK^T and
// softmax: head size 128 at N = 2, cfg5; N = 4 at head size 64, cfg3) or runs one wave
// per SIMD (N = 3 at head size 64, cfg3).  One-process A/B (profiles/r03_bsplit_ab.json):
// cfg5 fwd 20.54 -> 12.66 ms, cfg3 N=4 0.744 -> 0.485, N=3 0.409 -> 0.361; cfg2's
// paired N = 2 plan stays (split: 0.999 -> 1.126).  A/B builds: the macro DTA_FWD_BSPLIT = 0
// builds no split at all, 1 also splits the non-auto plans (the product build is -1).
#ifndef DTA_FWD_BSPLIT
#define DTA_FWD_BSPLIT -1
#endif
// Sequential-branch forward (SEQ kernels): where the N-branch forward runs branch-split and
// the single-branch plan is the paired one with the whole dv in one workgroup, the N
// branches of a query block run one after another in one workgroup, which forms O itself
// instead of a combine pass re-reading every fp32 O_i (DTA_FWD_SEQ = 0 in A/B builds: the
// branch-split workgroups plus branch_combine_kernel).
#ifndef DTA_FWD_SEQ
#define DTA_FWD_SEQ 1
#endif
template <class E, int HS, int DV, bool DROP>
constexpr bool fwd_seq_ok() {
  return DTA_FWD_SEQ && !DROP && sizeof(E) == 2 && DV == 2 * HS && FwdPick<E, HS, 1, DV, DROP>::pair &&
         FwdPick<E, HS, 1, DV, DROP>::DVC == DV;
}

template <class E, int HS, int N, int DV_ = 2 * HS>
struct Plan {
  static constexpr int DV = DV_;
  using FP = FwdPick<E, HS, N, DV>;
  using DP = DqPick<E, HS, N, DV>;
  static constexpr int KVW = DkdvWaves<E, HS, N, DV>::v;
  static constexpr bool KPR = DkdvWaves<E, HS, N, DV>::pair && !DkdvWaves<E, HS, N, DV>::gr;
  static constexpr bool ok = FP::ok && DP::ok &&
                             DkdvCfg<E, HS, N, DV, KVW, KPR, DkdvWaves<E, HS, N, DV>::gr>::bytes <= 160 * 1024;
};

template <class E, int HS, int N, int DV_, bool DROP>
int launch_fwd_t(const FwdParams& p, hipStream_t st) {
  using PL = Plan<E, HS, N, DV_>;
  using FP = FwdPick<E, HS, N, PL::DV, DROP>;
  constexpr int DVC = FP::DVC, NW = FP::NW;
  constexpr int QH = FP::QH;
  constexpr int bytes = FwdCfg<E, HS, N, DVC, NW, FP::QREG, QH>::bytes;
  // auto: the N-branch plan splits dv, or (16-bit, head size >= 64) it is not the paired
  // two-workgroups-per-CU plan (N >= 3, head size 96 / 128: one wave per SIMD).  Auto
  // plans always split (their N-branch kernel is not built); an A/B build with
  // DTA_FWD_BSPLIT = 1 also splits the others.
  constexpr bool CAN = N >= 2 && Plan<E, HS, 1, PL::DV>::ok;
  constexpr bool AUTO = CAN && DTA_FWD_BSPLIT != 0 &&
                        (DVC < PL::DV || (sizeof(E) == 2 && HS >= 64 && !FwdPick<E, HS, N, PL::DV>::pair));
  if constexpr (CAN) {
    if (AUTO || DTA_FWD_BSPLIT > 0) {
      FwdParams q = p;
      if constexpr (fwd_seq_ok<E, HS, PL::DV, DROP>()) {
        q.bseq = N;
        return launch_fwd_t<E, HS, 1, DV_, DROP>(q, st);
      }
      q.bsplit = N;
      if (int e = launch_fwd_t<E, HS, 1, DV_, DROP>(q, st)) return e;
      const int64_t n = (int64_t)p.B * p.T * p.H * (PL::DV / (16 / (int)sizeof(E)));
      if (n >= (1ll << 31)) return -2;
      hipLaunchKernelGGL((branch_combine_kernel<E, N>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p,
                         combine_div(p, (int)sizeof(E)));
      return (int)hipGetLastError();
    }
  }
  if constexpr (AUTO) {
    return -2;       // unreachable
  } else {
  const int nsp = (N == 1 && p.bsplit > 1) ? p.bsplit : 1;
  dim3 grid((p.T + NW * 32 - 1) / (NW * 32), p.H * nsp * (PL::DV / DVC), p.B);
  auto run = [&](auto SRDV) -> int {
    auto go = [&](auto K) -> int {
      if (int e = set_smem(K, bytes)) return e;
      hipLaunchKernelGGL(K, grid, dim3(NW * 64), bytes, st, p);
      return 0;
    };
    if constexpr (N == 1 && fwd_seq_ok<E, HS, PL::DV, DROP>())
      if (p.bseq > 1) return go(attn_fwd_kernel<E, HS, N, DVC, NW, FP::QREG, decltype(SRDV)::value, DROP, QH, true>);
    return go(attn_fwd_kernel<E, HS, N, DVC, NW, FP::QREG, decltype(SRDV)::value, DROP, QH>);
  };
  int e = 0;
  if constexpr (KvRing<E, HS, N, DVC, FwdCfg<E, HS, N, DVC, NW, FP::QREG, QH>::BN, NW>::ok)
    e = kv_layout_ok(p, (int)sizeof(E)) ? run(std::true_type{}) : run(std::false_type{});
  else
    e = run(std::false_type{});
  if (e) return e;
  return (int)hipGetLastError();
  }
}

template <class E, int HS, int N, int DV_, bool DROP>
int launch_dq_t(const BwdParams& p, hipStream_t st) {
  using PL = Plan<E, HS, N, DV_>;
  using DP = DqPick<E, HS, N, PL::DV, DROP>;
  constexpr int NW = DP::NW, DV = PL::DV;
  constexpr bool QR = DP::QREG;
  constexpr int QH = DP::QH;
  constexpr bool B32 = DP::B32;
  using CF = DqCfg<E, HS, N, DV, NW, QR, QH, B32>;
  constexpr int bytes = CF::bytes;
  dim3 grid((p.T + NW * 32 - 1) / (NW * 32), p.H, p.B);
  auto run = [&](auto F32, auto SRDV) -> int {
    auto kern = attn_dq_kernel<E, HS, N, DV, NW, QR, decltype(F32)::value, decltype(SRDV)::value, DROP, QH, B32>;
    if (int e = set_smem(kern, bytes)) return e;
    hipLaunchKernelGGL(kern, grid, dim3(NW * 64), bytes, st, p);
    return 0;
  };
  auto go = [&](auto SRDV) -> int { return p.dq32 ? run(std::true_type{}, SRDV) : run(std::false_type{}, SRDV); };
  int e = 0;
  if constexpr (KvRing<E, HS, N, DV, CF::BN, NW>::ok && CF::HSP == img_cols(HS))
    e = kv_layout_ok(p, (int)sizeof(E)) ? go(std::true_type{}) : go(std::false_type{});
  else
    e = go(std::false_type{});
  if (e) return e;
  return (int)hipGetLastError();
}

template <class E, int HS, int N, int DV_, bool DROP>
int launch_dkdv_t(const BwdParams& p, hipStream_t st) {
  using PL = Plan<E, HS, N, DV_>;
  using KW = DkdvWaves<E, HS, N, PL::DV, DROP>;
  constexpr int NW = KW::v, DV = PL::DV;
  constexpr bool GR = KW::gr;
  constexpr bool PR = KW::pair && !GR;
  using CF = DkdvCfg<E, HS, N, DV, NW, PR, GR>;
  constexpr int bytes = CF::bytes;
  dim3 grid((p.T + NW * 32 - 1) / (NW * 32), p.H, p.B);
  dim3 block(NW * 64);
  // one-wave-per-SIMD 16-bit plans (4 waves, not paired) have 512 registers: dK and dV
  // accumulators up to 288 of them share one launch (head size 128 at N = 2, cfg5)
  constexpr int HSB = DkdvSplit<HS, N, DV>::HSB;
  constexpr bool FUSED = DkdvSplit<HS, N, DV>::fused ||
                         (DTA_DKDV_FUSE1 && sizeof(E) == 2 && NW == 4 && !PR && N * HSB / 2 + DV / 2 <= 288);
  // ABI 8 lse_c (p.lsec): the |c_i|-folded instantiation, built for the 16-bit plans without
  // dropout whose row vectors ride in the ring
  constexpr bool CAN_FOLD = sizeof(E) == 2 && !DROP && !GR && DTA_DKDV_CFOLD;
  auto run = [&](auto DKV, auto DVVV, auto SRDV) -> int {
    auto launch = [&](auto CFV) -> int {
      auto kern = attn_dkdv_kernel<E, HS, N, DV, NW, decltype(DKV)::value, decltype(DVVV)::value,
                                   decltype(SRDV)::value, DROP, PR, GR, decltype(CFV)::value>;
      if (int e = set_smem(kern, bytes)) return e;
      hipLaunchKernelGGL(kern, grid, block, bytes, st, p);
      return 0;
    };
    if constexpr (CAN_FOLD)
      if (p.lsec) return launch(std::true_type{});
    return launch(std::false_type{});
  };
  auto go = [&](auto SRDV) -> int {
    if constexpr (FUSED) {
      return run(std::true_type{}, std::true_type{}, SRDV);
    } else {
      if (int e = run(std::true_type{}, std::false_type{}, SRDV)) return e;
      return run(std::false_type{}, std::true_type{}, SRDV);
    }
  };
  int e = 0;
  if constexpr (TileRing<E, HS, N, DV, NW, true, CF::BQ, !GR>::ok) {
    e = ring_layout_ok(p, (int)sizeof(E)) ? go(std::true_type{}) : go(std::false_type{});
  } else {
    e = go(std::false_type{});
  }
  if (e) return e;
  return (int)hipGetLastError();
}

// Head size 256 (16-bit diff plans; fp32 only the control's dv = hs one fits): head sizes 129-256
// run there zero-padded (ops.padded_head), the reference accepting any n_embd // (2 n_head)
// (diff_transformer.py:111).  Its N = 2 backward plans spill, so the backward runs it as
// single-branch groups (capi.hip bwd_group_cap) and those plans read LDS through
// compiler-tracked loads (SPILLS).
// (head size, branches, value width): the differential models' dv = 2 hs, plus the
// control model's standard attention (N = 1, dv = hs; control.py:38-63).  Head size 96
// is the reference's own TrainingConfig (n_embd 768, n_head 4: train.py:60-61 with
// diff_transformer.py:111 gives 768 // 8; the control model's 2 * n_head heads also 96).
// (A/B variant builds may predefine DTA_FOR_CONFIGS to a subset: faster experiment builds)
#ifndef DTA_FOR_CONFIGS
#define DTA_FOR_CONFIGS(X) \
  X(16, 1, 32) X(16, 2, 32) X(16, 3, 32) X(16, 4, 32) X(32, 1, 64) X(32, 2, 64) X(32, 3, 64) X(32, 4, 64) \
  X(64, 1, 128) X(64, 2, 128) X(64, 3, 128) X(64, 4, 128) X(128, 1, 256) X(128, 2, 256) X(128, 3, 256) \
  X(128, 4, 256) X(64, 1, 64) X(128, 1, 128) X(32, 1, 32) \
  X(96, 1, 192) X(96, 2, 192) X(96, 3, 192) X(96, 4, 192) X(96, 1, 96) \
  X(256, 1, 512) X(256, 2, 512) X(256, 1, 256)
#endif

// whether the N-branch plan of (HS, N, DV) is built for E
template <class E>
bool native_t(int hs, int n, int dv) {
#define DTA_S(HS_, N_, DV_) if (hs == HS_ && n == N_ && dv == DV_) return Plan<E, HS_, N_, DV_>::ok;
  DTA_FOR_CONFIGS(DTA_S)
#undef DTA_S
  return false;
}

// Any branch count N >= 2 whose N-branch plan is not built (N >= 5, fp32 N = 3 / 4 at head
// sizes 96 / 128): N single-branch workgroups per (query block, head) -- the N = 1 kernel
// with bsplit = N, each writing its O_i and LSE_i -- then the combine O = sum_i c_i O_i
// with the branch count at run time.  The backward runs such calls as branch groups
// (capi.hip).
template <class E, bool DROP>
int fwd_branch_split_any(const FwdParams& p, hipStream_t st) {
  FwdParams q = p;
  q.bsplit = p.N;
  int e = -2;
  bool seq = false;
#define DTA_F1(HS_, N_, DV_) \
  if (N_ == 1 && p.HS == HS_ && p.DV == DV_) { \
    if constexpr (N_ == 1 && Plan<E, HS_, 1, DV_>::ok) { \
      if constexpr (fwd_seq_ok<E, HS_, DV_, DROP>()) { q.bsplit = 0; q.bseq = p.N; seq = true; } \
      e = launch_fwd_t<E, HS_, 1, DV_, DROP>(q, st); } }
  DTA_FOR_CONFIGS(DTA_F1)
#undef DTA_F1
  if (e || seq) return e;
  const int64_t n = (int64_t)p.B * p.T * p.H * (p.DV / (16 / (int)sizeof(E)));
  if (n >= (1ll << 31)) return -2;
  hipLaunchKernelGGL((branch_combine_kernel<E, 0>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p,
                     combine_div(p, (int)sizeof(E)));
  return (int)hipGetLastError();
}

template <class E, bool DROP>
int dispatch_fwd(const FwdParams& p, hipStream_t st) {
#define DTA_F(HS_, N_, DV_) \
  if (p.HS == HS_ && p.N == N_ && p.DV == DV_) { \
    if constexpr (Plan<E, HS_, N_, DV_>::ok) return launch_fwd_t<E, HS_, N_, DV_, DROP>(p, st); }
  DTA_FOR_CONFIGS(DTA_F)
#undef DTA_F
  if (p.N >= 2) return fwd_branch_split_any<E, DROP>(p, st);
  return -2;
}

// the backward kernels take native branch counts only (capi.hip splits the others into groups)
template <class E, bool DROP>
int dispatch_dq(const BwdParams& p, hipStream_t st) {
#define DTA_Q(HS_, N_, DV_) \
  if (p.HS == HS_ && p.N == N_ && p.DV == DV_) { \
    if constexpr (Plan<E, HS_, N_, DV_>::ok) return launch_dq_t<E, HS_, N_, DV_, DROP>(p, st); else return -2; }
  DTA_FOR_CONFIGS(DTA_Q)
#undef DTA_Q
  return -2;
}

template <class E, bool DROP>
int dispatch_dkdv(const BwdParams& p, hipStream_t st) {
#define DTA_K(HS_, N_, DV_) \
  if (p.HS == HS_ && p.N == N_ && p.DV == DV_) { \
    if constexpr (Plan<E, HS_, N_, DV_>::ok) return launch_dkdv_t<E, HS_, N_, DV_, DROP>(p, st); else return -2; }
  DTA_FOR_CONFIGS(DTA_K)
#undef DTA_K
  return -2;
}

}  // namespace dta
