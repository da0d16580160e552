// attn_kernels.h -- fused N-branch causal differential attention, gfx950.
//
// Forward (replaces diff_transformer.py:57-72 for every head at once, and the
// branch loop of Ndiff_transformer.py:102-125):
//   O = sum_i c[h][i] * softmax_causal(Q_i K_i^T * scale) V
// One workgroup = 4 waves = 128 query rows of one (b, h, dv-chunk); each wave
// owns 32 rows.  Key tiles of BN rows of every K_i and of V are staged in LDS
// once per workgroup and feed all N branches.  Scores are computed transposed
// (S^T = K Q^T, key in registers, query on the lane), so the online softmax of
// a query row lives in one lane pair (l, l^32) and P^T is already the B
// operand of O^T += V^T P^T (V^T read from the row-major V tile with
// ds_read_b64_tr_b16).  Outputs: the combined O, the per-branch normalised
// O_i (for the backward's delta_i) and the per-branch log2-sum-exp.
//
// Backward: one workgroup = NW waves = NW*32 keys of one (b, h); each wave
// keeps dK_i^T and dV^T of its 32 keys in registers while the workgroup sweeps
// 32-row query tiles at and below the diagonal.  S is computed with the key on
// the lane, so P, dS are directly the B operands of dV^T += dO^T P_c and
// dK_i^T += Q_i^T dS_i; dS crosses LDS once for dQ_i = dS_i K_i, which is
// summed across key blocks with fp32 atomics.  dS_i = c_i P_i (dP - delta_i),
// dP = dO V^T shared by all branches, P_c = sum_i c_i P_i.
#pragma once
#include "dta_common.h"
#include "dta_internal.h"

namespace dta {

constexpr int FWD_WAVES = 4;
constexpr int FWD_BM = FWD_WAVES * 32;

template <class E> struct FwdTile { static constexpr int BN = 64; };
template <> struct FwdTile<float> { static constexpr int BN = 32; };

// dv chunk per forward workgroup: keep N * DVC/2 accumulator VGPRs <= 128
template <int N, int DV>
struct FwdChunk {
  static constexpr int cap = (256 / N) / 32 * 32;
  static constexpr int DVC = DV <= cap ? DV : (cap >= 128 && DV % 128 == 0 ? 128 : (cap >= 64 ? 64 : 32));
};

template <class E, int HS, int N, int DVC>
struct FwdSmem {
  static constexpr int BN = FwdTile<E>::BN;
  static constexpr int KSTR = HS + Pad<E>::v;
  static constexpr int VSTR = DVC + (sizeof(E) == 2 ? 32 : 0);
  static constexpr int bytes = (N * BN * KSTR + BN * VSTR) * (int)sizeof(E);
};

template <class E, int HS, int N, int DVC>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(FwdParams p) {
  using O = Ops<E>;
  using frag = typename O::frag;
  constexpr int BN = FwdTile<E>::BN;
  constexpr int KS = O::KSTEP;
  constexpr int KSTR = FwdSmem<E, HS, N, DVC>::KSTR;
  constexpr int VSTR = FwdSmem<E, HS, N, DVC>::VSTR;
  constexpr int NSQ = HS / KS;          // k-steps of QK^T
  constexpr int NKB = BN / 32;          // 32-key blocks per tile
  constexpr int SPB = 32 / KS;          // PV k-steps per 32-key block
  constexpr int NDB = DVC / 32;
  constexpr int VEC = O::VEC;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  E* Ks = reinterpret_cast<E*>(smem);
  E* Vs = Ks + N * BN * KSTR;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int nch = p.DV / DVC;
  const int qt = gridDim.x - 1 - blockIdx.x;           // longest (causal) tiles first
  const int hh = blockIdx.y / nch, dc0 = (blockIdx.y % nch) * DVC;
  const int b = blockIdx.z;
  const int T = p.T;
  const int q0 = qt * FWD_BM, qw0 = q0 + wave * 32;
  const int qrow = qw0 + c32;

  const E* gq = reinterpret_cast<const E*>(p.q.p) + b * p.q.sb + hh * p.q.sh;
  const E* gk = reinterpret_cast<const E*>(p.k.p) + b * p.k.sb + hh * p.k.sh;
  const E* gv = reinterpret_cast<const E*>(p.v.p) + b * p.v.sb + hh * p.v.sh + dc0;

  float coef[N];
#pragma unroll
  for (int i = 0; i < N; ++i) coef[i] = p.coef[hh * N + i];

  // Q fragments (B operand of S^T = K Q^T) live in registers for the whole sweep
  frag qf[N][NSQ];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int s = 0; s < NSQ; ++s)
      qf[i][s] = qrow < T ? O::load_global(gq + (int64_t)qrow * p.q.st + i * p.q.si + s * KS + hf * O::KH)
                          : O::zero();

  f32x16 acc[N][NDB];
  float m[N], l[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    m[i] = -INFINITY;
    l[i] = 0.f;
#pragma unroll
    for (int d = 0; d < NDB; ++d) acc[i][d] = f32x16{};
  }

  const int kend = min(T, q0 + FWD_BM);
  const int ntiles = (kend + BN - 1) / BN;
  const bool wave_live = qw0 < T;

  for (int kt = 0; kt < ntiles; ++kt) {
    const int k0 = kt * BN;
    __syncthreads();
    // ---- stage K_i tiles and the V chunk into LDS
    {
      constexpr int KCH = HS / VEC;
      constexpr int NKC = N * BN * KCH;
      for (int c = tid; c < NKC; c += 256) {
        const int i = c / (BN * KCH), rem = c % (BN * KCH);
        const int r = rem / KCH, cc = rem % KCH;
        const int key = k0 + r;
        stage_vec<E>(Ks + (i * BN + r) * KSTR + cc * VEC,
                     gk + (int64_t)key * p.k.st + i * p.k.si + cc * VEC, key < T);
      }
      constexpr int VCH = DVC / VEC;
      for (int c = tid; c < BN * VCH; c += 256) {
        const int r = c / VCH, cc = c % VCH;
        const int key = k0 + r;
        stage_vec<E>(Vs + r * VSTR + cc * VEC, gv + (int64_t)key * p.v.st + cc * VEC, key < T);
      }
    }
    __syncthreads();
    if (!wave_live || k0 > qw0 + 31) continue;      // tile entirely above this wave's diagonal

    const bool needmask = (k0 + BN - 1 > qw0) || (k0 + BN > T);
    frag pf[N][NKB * SPB];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      f32x16 sa[NKB];
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        sa[kb] = f32x16{};
        const E* krow = Ks + (i * BN + kb * 32 + c32) * KSTR;
#pragma unroll
        for (int s = 0; s < NSQ; ++s) sa[kb] = O::mma(O::row(krow, s, hf), qf[i][s], sa[kb]);
      }
      if (needmask) {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + kb * 32 + rowof(r, hf);
            if (key > qrow || key >= T) sa[kb][r] = -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sa[kb][r]);
      mx = wave_max_halves(mx);
      const float mnew = fmaxf(m[i], mx * p.sl2);
      const float alpha = exp2_fast(m[i] - mnew);
      m[i] = mnew;
      float ls = 0.f;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = exp2_fast(fmaf(sa[kb][r], p.sl2, -mnew));
          sa[kb][r] = e;
          ls += e;
        }
      l[i] = fmaf(l[i], alpha, ls);
#pragma unroll
      for (int d = 0; d < NDB; ++d) acc[i][d] *= alpha;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        if constexpr (SPB == 2) {
          pf[i][kb * 2 + 0] = O::template pack<0>(sa[kb]);
          pf[i][kb * 2 + 1] = O::template pack<1>(sa[kb]);
        } else {
#pragma unroll
          for (int s = 0; s < 16; ++s) pf[i][kb * SPB + s] = sa[kb][s];
        }
      }
    }
    // ---- O_i^T += V^T P_i^T, the V fragment shared by all branches
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int s = 0; s < SPB; ++s) {
          const frag va = O::tr_perm(Vs + (kb * 32) * VSTR + d * 32, VSTR, s, hf, lane);
#pragma unroll
          for (int i = 0; i < N; ++i) acc[i][d] = O::mma(va, pf[i][kb * SPB + s], acc[i][d]);
        }
  }

  if (!wave_live || qrow >= T) return;
  // ---- epilogue: normalise, combine, store O, O_i and LSE
  float inv[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float lt = l[i] + __shfl_xor(l[i], 32, 64);
    inv[i] = 1.f / lt;
    if (dc0 == 0 && hf == 0)
      p.lse[(((int64_t)i * p.B + b) * p.H + hh) * T + qrow] = m[i] + __builtin_log2f(lt);
  }
  E* go = reinterpret_cast<E*>(p.o.p) + b * p.o.sb + (int64_t)qrow * p.o.st + hh * p.o.sh + dc0;
  E* gob = reinterpret_cast<E*>(p.obr.p) + b * p.obr.sb + (int64_t)qrow * p.obr.st + hh * p.obr.sh + dc0;
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
        store4<E>(gob + i * p.obr.si + e, a0, a1, a2, a3);
        o0 = fmaf(coef[i], a0, o0); o1 = fmaf(coef[i], a1, o1);
        o2 = fmaf(coef[i], a2, o2); o3 = fmaf(coef[i], a3, o3);
      }
      store4<E>(go + e, o0, o1, o2, o3);
    }
}

// ------------------------------------------------------------- backward ---
template <class E> struct BwdWaves { static constexpr int v = 4; };
template <> struct BwdWaves<float> { static constexpr int v = 2; };

template <class E, int HS, int N, int DV>
struct BwdSmem {
  static constexpr int NW = BwdWaves<E>::v;
  static constexpr int BK = NW * 32;
  static constexpr int HSP = HS < 32 ? 32 : HS;
  static constexpr int KSTR = HSP + Pad<E>::v;
  static constexpr int QSTR = HSP + Pad<E>::v;
  static constexpr int DOSTR = DV + Pad<E>::v;
  static constexpr int DSSTR = 32 + Pad<E>::v;
  static constexpr int nK = N * BK * KSTR, nQ = N * 32 * QSTR, nDO = 32 * DOSTR, nDS = N * BK * DSSTR;
  static constexpr int bytes = (nK + nQ + nDO + nDS) * (int)sizeof(E) + 2 * N * 32 * 4;
};

// accumulator budget -> whether dK/dQ and dV are computed by one launch
template <class E, int HS, int N, int DV>
struct BwdSplit {
  static constexpr int HSP = HS < 32 ? 32 : HS;
  static constexpr bool fused = (N * HSP / 2 + DV / 2) <= 160;
};

template <class E, int HS, int N, int DV, bool DKQ, bool DVV>
__global__ __launch_bounds__(BwdWaves<E>::v * 64, 1) void attn_bwd_kernel(BwdParams p) {
  using O = Ops<E>;
  using frag = typename O::frag;
  using SM = BwdSmem<E, HS, N, DV>;
  constexpr int NW = SM::NW, BK = SM::BK, HSP = SM::HSP;
  constexpr int KSTR = SM::KSTR, QSTR = SM::QSTR, DOSTR = SM::DOSTR, DSSTR = SM::DSSTR;
  constexpr int KS = O::KSTEP;
  constexpr int VEC = O::VEC;
  constexpr int NTHR = NW * 64;
  constexpr int NSQ = HS / KS;         // k-steps over head dim
  constexpr int NSV = DV / KS;         // k-steps over dv
  constexpr int SPB = 32 / KS;         // k-steps over a 32-row query tile
  constexpr int NHB = HSP / 32;
  constexpr int NVB = DV / 32;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  E* Ks = reinterpret_cast<E*>(smem);
  E* Qs = Ks + SM::nK;
  E* dOs = Qs + SM::nQ;
  E* dSs = dOs + SM::nDO;
  float* lse_s = reinterpret_cast<float*>(dSs + SM::nDS);
  float* del_s = lse_s + N * 32;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hf = lane >> 5, c32 = lane & 31;
  const int kblk = blockIdx.x;                // block 0 has the most query tiles: launched first
  const int hh = blockIdx.y, b = blockIdx.z;
  const int T = p.T;
  const int kb0 = kblk * BK, kw0 = kb0 + wave * 32;
  const int krow = kw0 + c32;

  const E* gq = reinterpret_cast<const E*>(p.q.p) + b * p.q.sb + hh * p.q.sh;
  const E* gk = reinterpret_cast<const E*>(p.k.p) + b * p.k.sb + hh * p.k.sh;
  const E* gv = reinterpret_cast<const E*>(p.v.p) + b * p.v.sb + hh * p.v.sh;
  const E* gdo = reinterpret_cast<const E*>(p.dout.p) + b * p.dout.sb + hh * p.dout.sh;

  float coef[N];
#pragma unroll
  for (int i = 0; i < N; ++i) coef[i] = p.coef[hh * N + i];

  // ---- the workgroup's key block of every K_i, head dim zero-padded to HSP
  {
    constexpr int KCH = HSP / VEC;
    for (int c = tid; c < N * BK * KCH; c += NTHR) {
      const int i = c / (BK * KCH), rem = c % (BK * KCH);
      const int r = rem / KCH, cc = rem % KCH;
      const int key = kb0 + r;
      stage_vec<E>(Ks + (i * BK + r) * KSTR + cc * VEC,
                   gk + (int64_t)key * p.k.st + i * p.k.si + cc * VEC, key < T && cc * VEC < HS);
    }
  }
  // ---- this wave's V rows as B fragments of dP = dO V^T
  frag vf[NSV];
#pragma unroll
  for (int s = 0; s < NSV; ++s)
    vf[s] = (DKQ && krow < T) ? O::load_global(gv + (int64_t)krow * p.v.st + s * KS + hf * O::KH) : O::zero();

  f32x16 dk[DKQ ? N : 1][NHB];
  f32x16 dvacc[DVV ? NVB : 1];
#pragma unroll
  for (int i = 0; i < (DKQ ? N : 1); ++i)
#pragma unroll
    for (int d = 0; d < NHB; ++d) dk[i][d] = f32x16{};
#pragma unroll
  for (int d = 0; d < (DVV ? NVB : 1); ++d) dvacc[d] = f32x16{};

  const bool wave_keys = kw0 < T;
  for (int q0 = kb0; q0 < T; q0 += 32) {
    __syncthreads();
    {
      constexpr int QCH = HSP / VEC;
      for (int c = tid; c < N * 32 * QCH; c += NTHR) {
        const int i = c / (32 * QCH), rem = c % (32 * QCH);
        const int r = rem / QCH, cc = rem % QCH;
        const int q = q0 + r;
        stage_vec<E>(Qs + (i * 32 + r) * QSTR + cc * VEC,
                     gq + (int64_t)q * p.q.st + i * p.q.si + cc * VEC, q < T && cc * VEC < HS);
      }
      constexpr int OCH = DV / VEC;
      for (int c = tid; c < 32 * OCH; c += NTHR) {
        const int r = c / OCH, cc = c % OCH;
        const int q = q0 + r;
        stage_vec<E>(dOs + r * DOSTR + cc * VEC, gdo + (int64_t)q * p.dout.st + cc * VEC, q < T);
      }
      for (int c = tid; c < N * 32; c += NTHR) {
        const int i = c / 32, r = c % 32, q = q0 + r;
        const int64_t off = (((int64_t)i * p.B + b) * p.H + hh) * T + q;
        lse_s[c] = q < T ? p.lse[off] : 0.f;
        del_s[c] = q < T ? p.delta[off] : 0.f;
      }
    }
    __syncthreads();
    const bool live = wave_keys && (q0 + 31 >= kw0);
    if (live) {
      const bool needmask = (kw0 + 31 > q0) || (q0 + 32 > T) || (kw0 + 32 > T);
      f32x16 dp = f32x16{};
      if constexpr (DKQ) {
#pragma unroll
        for (int s = 0; s < NSV; ++s) dp = O::mma(O::row(dOs + c32 * DOSTR, s, hf), vf[s], dp);
      }
      f32x16 pc = f32x16{};
#pragma unroll
      for (int i = 0; i < N; ++i) {
        f32x16 sa = f32x16{};
        const E* qrowp = Qs + (i * 32 + c32) * QSTR;
        const E* krowp = Ks + (i * BK + wave * 32 + c32) * KSTR;
#pragma unroll
        for (int s = 0; s < NSQ; ++s) sa = O::mma(O::row(qrowp, s, hf), O::row(krowp, s, hf), sa);
        // sa[r] = S[q0 + rowof(r)][krow]  ->  P, dS
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qq = rowof(r, hf);
          float pr = exp2_fast(fmaf(sa[r], p.sl2, -lse_s[i * 32 + qq]));
          if (needmask && (krow > q0 + qq || q0 + qq >= T || krow >= T)) pr = 0.f;
          if constexpr (DVV) pc[r] = fmaf(coef[i], pr, pc[r]);
          if constexpr (DKQ) sa[r] = coef[i] * pr * (dp[r] - del_s[i * 32 + qq]);
        }
        if constexpr (DKQ) {
          // dK_i^T += Q_i^T dS_i
#pragma unroll
          for (int d = 0; d < NHB; ++d) {
            const E* qb = Qs + i * 32 * QSTR + d * 32;
            if constexpr (SPB == 2) {
              dk[i][d] = O::mma(O::tr_perm(qb, QSTR, 0, hf, lane), O::template pack<0>(sa), dk[i][d]);
              dk[i][d] = O::mma(O::tr_perm(qb, QSTR, 1, hf, lane), O::template pack<1>(sa), dk[i][d]);
            } else {
#pragma unroll
              for (int s = 0; s < SPB; ++s) dk[i][d] = O::mma(O::tr_perm(qb, QSTR, s, hf, lane), sa[s], dk[i][d]);
            }
          }
          // dS_i -> LDS image [key][query] for dQ
          E* dsrow = dSs + (i * BK + wave * 32 + c32) * DSSTR;
#pragma unroll
          for (int g = 0; g < 4; ++g)
            store4_lds<E>(dsrow + 8 * g + 4 * hf, sa[4 * g], sa[4 * g + 1], sa[4 * g + 2], sa[4 * g + 3]);
        }
      }
      if constexpr (DVV) {
#pragma unroll
        for (int d = 0; d < NVB; ++d) {
          const E* ob = dOs + d * 32;
          if constexpr (SPB == 2) {
            dvacc[d] = O::mma(O::tr_perm(ob, DOSTR, 0, hf, lane), O::template pack<0>(pc), dvacc[d]);
            dvacc[d] = O::mma(O::tr_perm(ob, DOSTR, 1, hf, lane), O::template pack<1>(pc), dvacc[d]);
          } else {
#pragma unroll
            for (int s = 0; s < SPB; ++s) dvacc[d] = O::mma(O::tr_perm(ob, DOSTR, s, hf, lane), pc[s], dvacc[d]);
          }
        }
      }
    } else if constexpr (DKQ) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        E* dsrow = dSs + (i * BK + wave * 32 + c32) * DSSTR;
#pragma unroll
        for (int g = 0; g < 4; ++g) store4_lds<E>(dsrow + 8 * g + 4 * hf, 0.f, 0.f, 0.f, 0.f);
      }
    }
    if constexpr (DKQ) {
      __syncthreads();
      // dQ_i[q][d] = sum_k dS_i[q][k] K_i[k][d] over this block's keys; fp32 atomics across blocks
      constexpr int NB = N * NHB;
      for (int bi = wave; bi < NB; bi += NW) {
        const int i = bi / NHB, d = bi % NHB;
        f32x16 a = f32x16{};
        const E* dsb = dSs + i * BK * DSSTR;
        const E* kbp = Ks + i * BK * KSTR + d * 32;
#pragma unroll 4
        for (int s = 0; s < BK / KS; ++s)
          a = O::mma(O::tr_nat(dsb, DSSTR, s, hf, lane), O::tr_nat(kbp, KSTR, s, hf, lane), a);
        const int dcol = d * 32 + c32;
        if (dcol < HS) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int q = q0 + rowof(r, hf);
            if (q < T)
              atomicAdd(p.dq + ((((int64_t)b * T + q) * p.H + hh) * N + i) * HS + dcol, a[r] * p.scale);
          }
        }
      }
    }
  }

  if (!wave_keys || krow >= T) return;
  if constexpr (DKQ) {
    E* gdk = reinterpret_cast<E*>(p.dk.p) + b * p.dk.sb + (int64_t)krow * p.dk.st + hh * p.dk.sh;
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int d = 0; d < NHB; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int e = d * 32 + 8 * g + 4 * hf;
          if (e < HS)
            store4<E>(gdk + i * p.dk.si + e, dk[i][d][4 * g] * p.scale, dk[i][d][4 * g + 1] * p.scale,
                      dk[i][d][4 * g + 2] * p.scale, dk[i][d][4 * g + 3] * p.scale);
        }
  }
  if constexpr (DVV) {
    E* gdv = reinterpret_cast<E*>(p.dv.p) + b * p.dv.sb + (int64_t)krow * p.dv.st + hh * p.dv.sh;
#pragma unroll
    for (int d = 0; d < NVB; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int e = d * 32 + 8 * g + 4 * hf;
        store4<E>(gdv + e, dvacc[d][4 * g], dvacc[d][4 * g + 1], dvacc[d][4 * g + 2], dvacc[d][4 * g + 3]);
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

template <class E, int HS, int N>
int launch_fwd_t(const FwdParams& p, hipStream_t st) {
  constexpr int DV = 2 * HS;
  constexpr int DVC = FwdChunk<N, DV>::DVC;
  constexpr int bytes = FwdSmem<E, HS, N, DVC>::bytes;
  auto kern = attn_fwd_kernel<E, HS, N, DVC>;
  if (int e = set_smem(kern, bytes)) return e;
  dim3 grid((p.T + FWD_BM - 1) / FWD_BM, p.H * (DV / DVC), p.B);
  hipLaunchKernelGGL(kern, grid, dim3(256), bytes, st, p);
  return (int)hipGetLastError();
}

template <class E, int HS, int N>
int launch_bwd_t(const BwdParams& p, hipStream_t st) {
  constexpr int DV = 2 * HS;
  using SM = BwdSmem<E, HS, N, DV>;
  constexpr int bytes = SM::bytes;
  dim3 grid((p.T + SM::BK - 1) / SM::BK, p.H, p.B);
  dim3 block(SM::NW * 64);
  if constexpr (BwdSplit<E, HS, N, DV>::fused) {
    auto kern = attn_bwd_kernel<E, HS, N, DV, true, true>;
    if (int e = set_smem(kern, bytes)) return e;
    hipLaunchKernelGGL(kern, grid, block, bytes, st, p);
  } else {
    auto k1 = attn_bwd_kernel<E, HS, N, DV, true, false>;
    auto k2 = attn_bwd_kernel<E, HS, N, DV, false, true>;
    if (int e = set_smem(k1, bytes)) return e;
    if (int e = set_smem(k2, bytes)) return e;
    hipLaunchKernelGGL(k1, grid, block, bytes, st, p);
    hipLaunchKernelGGL(k2, grid, block, bytes, st, p);
  }
  return (int)hipGetLastError();
}

template <class E, int HS, int N>
constexpr bool fits() {
  return BwdSmem<E, HS, N, 2 * HS>::bytes <= 160 * 1024 &&
         FwdSmem<E, HS, N, FwdChunk<N, 2 * HS>::DVC>::bytes <= 160 * 1024;
}

template <class E>
int dispatch_fwd(const FwdParams& p, hipStream_t st) {
#define DTA_F(HS_, N_) \
  if (p.HS == HS_ && p.N == N_) { if constexpr (fits<E, HS_, N_>()) return launch_fwd_t<E, HS_, N_>(p, st); else return -2; }
#define DTA_FN(HS_) DTA_F(HS_, 1) DTA_F(HS_, 2) DTA_F(HS_, 3) DTA_F(HS_, 4)
  DTA_FN(16) DTA_FN(32) DTA_FN(64) DTA_FN(128)
#undef DTA_FN
#undef DTA_F
  return -2;
}

template <class E>
int dispatch_bwd(const BwdParams& p, hipStream_t st) {
#define DTA_B(HS_, N_) \
  if (p.HS == HS_ && p.N == N_) { if constexpr (fits<E, HS_, N_>()) return launch_bwd_t<E, HS_, N_>(p, st); else return -2; }
#define DTA_BN(HS_) DTA_B(HS_, 1) DTA_B(HS_, 2) DTA_B(HS_, 3) DTA_B(HS_, 4)
  DTA_BN(16) DTA_BN(32) DTA_BN(64) DTA_BN(128)
#undef DTA_BN
#undef DTA_B
  return -2;
}

template <class E>
bool supported_t(int hs, int n) {
#define DTA_S(HS_, N_) if (hs == HS_ && n == N_) return fits<E, HS_, N_>();
#define DTA_SN(HS_) DTA_S(HS_, 1) DTA_S(HS_, 2) DTA_S(HS_, 3) DTA_S(HS_, 4)
  DTA_SN(16) DTA_SN(32) DTA_SN(64) DTA_SN(128)
#undef DTA_SN
#undef DTA_S
  return false;
}

}  // namespace dta
