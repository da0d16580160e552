/*
 * diffattn.h -- C ABI of libdiffattn.so, the MI355X (gfx950) differential
 * attention library.
 *
 * The reference (JoshFCooper415/differential_transformer_replication) has no
 * native code, plugin or FFI: its hot path is eager ATen called from
 * nn.Module.forward.  Each entry point below replaces a group of those eager
 * ops; the comment on each cites the reference lines it replaces.  The Python
 * package binds these through ctypes (differential_transformer_replication_amd/
 * _lib.py); INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *  - Plain C types only: device pointers, element strides (int64, in
 *    ELEMENTS not bytes), sizes, a hipStream_t passed as void*.
 *  - The caller (PyTorch's caching allocator) owns every buffer.  The library
 *    never allocates or frees device memory and keeps no state.
 *  - Every launch is asynchronous on the given stream; no host sync.
 *  - Functions return DTA_OK (0) or a negative error code and never throw
 *    across the ABI; dta_error_string() describes a code.
 *  - dtype applies to Q/K/V/O/dO/dQ/dK/dV activations; Obr, LSE, delta, the
 *    coefficients, the LayerNorm statistics/parameters and every *_f32 buffer
 *    are always fp32.
 *
 * Layouts (element strides are given per tensor so strided views of one
 * packed projection output can be passed without copies):
 *   Q, K   [b][t][h][i][d]   i < n_terms (the N softmax branches), d < head_size
 *   V, O   [b][t][h][e]      e < dv (dv = 2*head_size for diff attention; dv = head_size with n_terms = 1
 *                             for standard attention, head_size 64 or 128)
 *   Obr    [i][b][t][h][e]   per-branch normalised outputs A_i V, fp32 (default) or fp16
 *                             (obr_dtype, 16-bit activations only); saved for bwd:
 *                             delta_i = <dO, O_i> and d(coef) come from them
 *   LSE    [i][b][h][t]      fp32, NEGATED log2-sum-exp of the scaled scores (-log2 sum 2^(s*scale*log2e))
 *   coef   [h][i]            fp32, signed branch weights (diff: [1, -lambda];
 *                            N-diff: [+l0, -l1, +l2, ...])
 */
#ifndef DIFFATTN_H_
#define DIFFATTN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DTA_ABI_VERSION 8   /* 8: lse_c workspace (the key-major kernel folds |c_i| into its probabilities);
                               7: per-stage backward branch-group caps (group_max_dq, group_max_dkdv);
                               6: obr_dtype (fp16 O_i for 16-bit activations);
                               5: RoPE of Q_i at the forward's load (rope_freqs, q_rot);
                               4: Obr is fp32 for every dtype; any n_terms >= 1 */

enum dta_dtype { DTA_BF16 = 0, DTA_F16 = 1, DTA_F32 = 2 };

enum dta_status {
  DTA_OK = 0,
  DTA_ERR_INVALID = -1,      /* bad shape / stride / pointer / argument   */
  DTA_ERR_UNSUPPORTED = -2,  /* head_size / n_terms / dtype not built     */
  DTA_ERR_LAUNCH = -3,       /* hipLaunch / hipMemsetAsync failed         */
  DTA_ERR_DROPOUT = -4       /* attention dropout p outside [0, 1)         */
};

typedef struct dta_tensor {
  void* ptr;
  int64_t sb, st, sh, si;    /* strides for [b][t][h][i]; si unused for V/O */
} dta_tensor;

/* Forward of the fused N-branch causal differential attention core.
 * Replaces, for all heads at once, DiffHead.forward's scores/mask/softmax/
 * dropout/combine/@V (diff_transformer.py:57-72), the per-head loop
 * (diff_transformer.py:89) and AlternatingDiffHead's branch loop
 * (Ndiff_transformer.py:102-125; RoPE: K_i beforehand by dta_rope, Q_i at load, rope_freqs).
 * O = sum_i coef[h][i] * softmax(mask(Q_i K_i^T / sqrt(hs))) V. */
typedef struct dta_attn_fwd_args {
  int32_t dtype;             /* enum dta_dtype */
  int32_t B, T, H, n_terms, head_size, dv;
  float scale;               /* 1/sqrt(head_size) (diff_transformer.py:57) */
  float dropout_p;           /* attention-map dropout in [0, 1) (diff_transformer.py:66-67):
                                element (q, k) of map i of head h, batch b is kept iff
                                fmix32((key + q*0x9e3779b1) ^ (k*0x7feb352d)) >= p*2^32,
                                key = fmix32(seed_lo ^ fmix32(((b*H + h)*N + i) + seed_hi))
                                (fmix32: murmur3's finaliser), kept elements x 1/(1-p);
                                the row sums normalising the map see every element */
  dta_tensor q, k, v;        /* inputs */
  dta_tensor o;              /* output, combined */
  dta_tensor obr;            /* output [i][b][t][h][e]: sb,st,sh,si = strides of b,t,h,i; fp32 or fp16 (obr_dtype) */
  float* lse;                /* output fp32 [i][b][h][t], contiguous */
  const float* coef;         /* fp32 [h][i], contiguous */
  uint64_t dropout_seed;     /* with dropout_p > 0: the mask's seed (pass the same to dta_attn_bwd) */
  /* ABI 5, optional: RoPE of Q_i fused into the load (Ndiff_transformer.py:104-109).
   * With rope_freqs (fp32 [T][head_size/2][2] (cos, sin), 16-byte aligned) q holds the
   * UN-rotated Q_i; the kernel rotates each row as it loads it and writes the rotated row
   * to q_rot (same shape as q, dtype) for dta_attn_bwd.  k must already be rotated
   * (dta_rope over the K_i only).  NULL: q is used as given. */
  const float* rope_freqs;
  dta_tensor q_rot;
  int32_t obr_dtype;         /* ABI 6: 0 / DTA_F32 = obr is fp32; DTA_F16 = fp16 (16-bit dtype only:
                                2^-11 resolution, eight times bf16's, half the bytes of fp32) */
} dta_attn_fwd_args;

int dta_attn_fwd(const dta_attn_fwd_args* a, void* stream);

/* Backward of dta_attn_fwd (the autograd of diff_transformer.py:57-72 and
 * Ndiff_transformer.py:102-125): dQ_i, dK_i, dV and d(coef).  Maps are
 * recomputed from LSE; nothing T x T is stored and no atomics touch dQ.
 * Two fused kernels: a query-major one (delta_i = <dO, O_i>, dQ_i, d(coef))
 * and a key-major one (dK_i, dV).  dcoef[h][i] = sum_{b,t} <dO, A_i V>
 * (SURVEY semantic 5), from which autograd reaches the lambda_q and lambda_k
 * params through get_lambda (diff_transformer.py:41-48).
 * Workspaces (caller-allocated, see dta_attn_bwd_workspace_bytes):
 *   delta   fp32 [i][b][h][t]: PRIVATE to the backward.  The DQ stage writes it in an
 *           encoding only the DKDV stage of the same call reads (row constants relative
 *           to each branch group's first branch, re-based in place where the two stages
 *           group branches differently).  Run DTA_BWD_DQ exactly once per backward and
 *           DTA_BWD_DKDV after it on the same delta; never read or reuse it otherwise.
 *           When the stages run as separate calls, both calls must pass the SAME
 *           group_max_dq and group_max_dkdv (the DQ stage encodes delta for the DKDV
 *           grouping those caps give; different caps in the DKDV call decode it wrongly).
 *   dq_f32  optional fp32 [b][t][h][i][d] contiguous: when dq.ptr is NULL the
 *           dQ kernel writes fp32 here instead (callers that post-process dQ,
 *           e.g. the inverse RoPE, keep full precision). */
typedef struct dta_attn_bwd_args {
  int32_t dtype;
  int32_t B, T, H, n_terms, head_size, dv;
  float scale;
  float dropout_p;           /* as dta_attn_fwd_args; obr must be the forward's (dropped) O_i */
  dta_tensor q, k, v, obr;
  const float* lse;          /* fp32 [i][b][h][t] from the forward */
  const float* coef;         /* fp32 [h][i] */
  dta_tensor dout;           /* dO [b][t][h][e] */
  dta_tensor dq, dk, dv_out; /* outputs (dtype) */
  float* dcoef;              /* output fp32 [h][i] (overwritten) */
  float* delta;              /* workspace fp32 [i][b][h][t] */
  float* dq_f32;             /* see above */
  int32_t stages;            /* 0 = all; else bitmask of DTA_BWD_PRE (zero dcoef; a no-op when
                                dcoef_partial is given, whose ordered reduce writes dcoef whole),
                                DTA_BWD_DQ (query-major kernel), DTA_BWD_DKDV
                                (key-major kernel) -- lets a caller bracket one
                                kernel with events on the same stream; DQ must
                                run before DKDV (it produces delta) */
  const float* rope_freqs;   /* optional fp32 [T][head_size/2][2] (cos, sin) table,
                                16-byte aligned: q and k are the RoPE'd Q_i / K_i
                                (Ndiff_transformer.py:104-109), and dQ / dK are
                                returned w.r.t. the UN-rotated projections -- the
                                inverse rotation (apply_rotary_emb's backward) runs
                                in the kernels' epilogues, no extra pass or buffer */
  float* dcoef_partial;      /* optional fp32 workspace, dta_attn_bwd_dcoef_partial_bytes:
                                with it dcoef is summed from per-wave partials in a fixed
                                order (bitwise reproducible run to run); without it the
                                query-major kernel adds into dcoef by float atomics */
  uint64_t dropout_seed;     /* the forward's dropout seed */
  int32_t obr_dtype;         /* ABI 6: as dta_attn_fwd_args (the forward's obr) */
  int32_t group_max_dq;      /* ABI 7, optional (0 = the library's default per stage): the largest
                                branch group the DQ stage runs as one launch (n_terms above it run
                                as groups of the largest built branch count <= this cap, one launch
                                each).  Defaults: 4 for fp32; 16-bit: 2 at head_size 128 and at 64
                                with n_terms >= 4, else 4.  Setting it to 4 forces every built
                                native plan (the GPU tests check each one). */
  int32_t group_max_dkdv;    /* ABI 7, as group_max_dq for the DKDV stage.  Defaults: 4 for fp32;
                                16-bit: 2 at head_size >= 64, else 4.  Groups after the first
                                add their dV into the first group's. */
  float* dv_f32;             /* ABI 7, optional fp32 workspace [b][t][h][e] contiguous (B*T*H*dv
                                floats, 16-byte aligned): where the DKDV stage runs more than one
                                group (dta_attn_bwd_dkdv_groups > 1), the running dV sum stays here
                                in fp32 and only the last group rounds it to dtype.  NULL: each later
                                group adds into dv_out (one extra 16-bit rounding per group). */
  float* lse_c;              /* ABI 8, optional fp32 workspace [i][b][h][t] (n_terms*B*H*T floats, 16-byte
                                aligned), PRIVATE to the backward like delta: with 16-bit activations and
                                no dropout the DQ stage writes each row's stored LSE_i + log2|c_i| here and
                                the DKDV stage seeds its scores with it, so its probabilities come out
                                already scaled by |c_i| (one VALU op per element less in dV's operand).
                                Requires |c_i| < 2^64.  NULL (or fp32 / dropout): the unfolded kernels. */
} dta_attn_bwd_args;

enum { DTA_BWD_PRE = 1, DTA_BWD_DQ = 2, DTA_BWD_DKDV = 4 };

int dta_attn_bwd(const dta_attn_bwd_args* a, void* stream);
size_t dta_attn_bwd_workspace_bytes(int32_t B, int32_t T, int32_t H, int32_t n_terms,
                                    int32_t head_size);
size_t dta_attn_bwd_dcoef_partial_bytes(int32_t B, int32_t T, int32_t H, int32_t n_terms);
/* The number of dK/dV launches (branch groups) dta_attn_bwd runs for this shape with the given
 * group_max_dkdv (0 = default); 0 if the shape is unsupported or the cap is negative (which
 * dta_attn_bwd rejects).  > 1: pass dv_f32. */
int dta_attn_bwd_dkdv_groups(int32_t dtype, int32_t head_size, int32_t n_terms, int32_t dv, int32_t group_max_dkdv);

/* Cross-head LayerNorm x out_scale (GroupLayerNorm.forward,
 * diff_transformer.py:15-20, then `out * (1 - self.lambda_init)`,
 * diff_transformer.py:90-91; same at Ndiff_transformer.py:33-38,145-146).
 * Rows of width C; y = ((x - mean) * rstd * w + b) * out_scale.
 * mean/rstd (fp32 [rows]) are saved for dta_ln_bwd. */
typedef struct dta_ln_args {
  int32_t dtype;
  int64_t rows, C;
  float eps, out_scale;
  const void* x; int64_t x_stride;   /* row stride, elements */
  void* y; int64_t y_stride;
  const float* w; const float* b;    /* fp32 [C] */
  float* mean; float* rstd;          /* fp32 [rows] */
  /* backward only */
  const void* dy; int64_t dy_stride;
  void* dx; int64_t dx_stride;
  float* dw; float* db;              /* fp32 [C], accumulated (caller zeroes) */
  float* partial;                    /* optional fp32 workspace (dta_ln_bwd_workspace_bytes):
                                        per-block column partials summed in a fixed order, so
                                        dw/db are bitwise reproducible; 16-byte aligned;
                                        NULL: float atomics */
  int32_t io_dtype;                  /* 0: y / dy have `dtype`; else 1 + the y / dy dtype code,
                                        with dtype = DTA_F32 and y / dy DTA_BF16 or DTA_F16 (an fp32
                                        residual stream normalised straight into the autocast
                                        dtype, and its backward from that dtype's gradient) */
  /* residual fusion, io_dtype != 0 only (NULL = off): the pre-LN residual add of a
   * Block (diff_transformer.py:121-125, x + attn(ln1(x)) feeding ln2) in the same pass */
  const void* res; int64_t res_stride;   /* fwd: normalises x + res (res in the y dtype) ... */
  float* xo; int64_t xo_stride;          /* ... and writes x + res here (fp32, required with res) */
  const float* dres; int64_t dres_stride;  /* bwd: dx += dres (fp32 gradient of the residual branch) */
  void* dx16; int64_t dx16_stride;       /* bwd: dx also written in the y dtype */
} dta_ln_args;

int dta_ln_fwd(const dta_ln_args* a, void* stream);
int dta_ln_bwd(const dta_ln_args* a, void* stream);
size_t dta_ln_bwd_workspace_bytes(int64_t rows, int64_t C);

/* Interleaved-pair RoPE of every Q_i and K_i (apply_rotary_emb,
 * Ndiff_transformer.py:11-22 / control.py:11-22, rotation in fp32 then cast).
 * inverse != 0 applies the conjugate rotation (its backward).
 * src may be fp32 (src_f32 != 0) or dtype; dst is dtype.
 * freqs: fp32 [T][head_size/2][2] = view_as_real(freqs_cis[:T]). */
typedef struct dta_rope_args {
  int32_t dtype;
  int32_t B, T, H, n_terms, head_size;
  int32_t inverse, src_f32;
  dta_tensor src, dst;               /* [b][t][h][i][d] */
  const float* freqs;
} dta_rope_args;

int dta_rope(const dta_rope_args* a, void* stream);

/* One-token decode over a KV cache (incremental generate).
 * Replaces, for the newest position only, the full-prefix recompute that
 * generate() does per token (diff_transformer.py:177-185; the same loop in
 * Ndiff_transformer.py and control.py:163-171): for every (b, h)
 *   o = sum_i coef[h][i] * softmax(q_i . K_i[0:length]^T * scale) V[0:length]
 * which is the last row of dta_attn_fwd's output at T = length (the newest key
 * is the query's own position, so the causal mask keeps every cached key).
 * q: [b][.][h][i][d] (st ignored), k_cache [b][t][h][i][d], v_cache [b][t][h][e],
 * o [b][.][h][e] (st ignored).  head_size % 8 == 0, head_size <= 128,
 * n_terms <= 4, dv <= 256; every tensor 16-byte aligned with strides that are
 * multiples of 16 bytes.  workspace: fp32, dta_attn_decode_workspace_bytes
 * (covers both plans).  Plans: a split-key plan -- key chunks scored by separate
 * workgroups, then one combine launch -- for (head_size, dv) in {(32,64),
 * (64,128), (128,256)} and, with n_terms = 1, dv = head_size in {64, 128}; a
 * single-pass workgroup per (b, h) otherwise.  The split plan uses 256-key
 * chunks, or 512-key chunks when ceil(t_cap/256) * H * B >= 8192 workgroups;
 * the choice depends on t_cap only, so calls with the same t_cap reduce in the
 * same order whatever their length.  It is used while ceil(t_cap/chunk) *
 * n_terms <= 2048 (the combine's LDS weights). */
typedef struct dta_attn_decode_args {
  int32_t dtype;
  int32_t B, H, n_terms, head_size, dv;
  int32_t length;            /* valid cached keys, including the new token's */
  int32_t t_cap;             /* workspace row length (>= length) */
  float scale;
  dta_tensor q, k_cache, v_cache, o;
  const float* coef;         /* fp32 [h][i] */
  float* workspace;
  const int32_t* length_dev; /* optional device int32: the valid length, read by the
                                kernels (graph replay with a moving position); then
                                `length` is only its upper bound and sizes the grid.
                                Precondition 1 <= *length_dev <= length <= t_cap; the
                                kernels clamp it to [0, length] */
} dta_attn_decode_args;
int dta_attn_decode(const dta_attn_decode_args* a, void* stream);
size_t dta_attn_decode_workspace_bytes(int32_t B, int32_t H, int32_t n_terms, int32_t head_size, int32_t dv,
                                       int32_t t_cap);
/* SwiGLU of the Block feed-forward (diff_transformer.py SwiGLU.forward,
 * Ndiff_transformer.py:86-93 equivalent, control.py:80-90): out = silu(a) * b over
 * rows x n elements (n % 8 == 0; every row stride a multiple of 8 elements, every
 * pointer 16-byte aligned), and its backward da = dout * b * silu'(a),
 * db = dout * silu(a).  Unused pointers of the other direction may be NULL. */
typedef struct {
  int32_t dtype;
  int64_t rows, n;
  const void* a; int64_t a_stride;
  const void* b; int64_t b_stride;
  void* out; int64_t out_stride;
  const void* dout; int64_t dout_stride;
  void* da; int64_t da_stride;
  void* db; int64_t db_stride;
  /* backward, optional (ABI 3): with dbias, also the column sums of dA | dB as stored
   * (fp32 [2n]: the gate / xform Linears' bias gradient), through dbias_work
   * (dta_swiglu_bwd_workspace_bytes), summed in a fixed order */
  float* dbias; float* dbias_work;
} dta_swiglu_args;
int dta_swiglu_fwd(const dta_swiglu_args* a, void* stream);
int dta_swiglu_bwd(const dta_swiglu_args* a, void* stream);
size_t dta_swiglu_bwd_workspace_bytes(int64_t rows, int64_t n);

/* dst[i] += (float)src[i], i < n: gradient accumulation of a bf16/fp16/fp32 weight
 * gradient into fp32 master-gradient storage (the training step's packed projection
 * weights, SURVEY 8e/8f: torch.autograd's AccumulateGrad of the reference's
 * nn.Linear parameters, train.py:251-279).  src and dst 16-byte aligned. */
int dta_accumulate_f32(int32_t dtype, int64_t n, const void* src, float* dst, void* stream);

/* Cast/copy a [b][t][h][i][d] tensor from fp32 to dtype (dQ finalisation). */
int dta_cast_f32(int32_t dtype, int32_t B, int32_t T, int32_t H, int32_t n_terms,
                 int32_t head_size, const float* src, dta_tensor dst, void* stream);

const char* dta_error_string(int code);
int dta_abi_version(void);
/* 1 if (dtype, head_size, n_terms, dv) runs: an n_terms-branch kernel plan is built for
 * it, or (n_terms >= 2, dv = 2*head_size) the single-branch plan is -- then the forward
 * runs n_terms single-branch workgroups per query block and head plus a combine pass.
 * The backward runs each stage as branch groups of the largest built branch count not
 * above that stage's cap (group_max_dq / group_max_dkdv and their defaults), one launch
 * per group (dV summed over the groups, d(coef) reduced over all n_terms); where the two
 * stages group differently the DQ stage re-bases the delta rows for the DKDV stage.  Head sizes
 * 16, 32, 64, 96, 128 (dv = 2*head_size), and dv = head_size at n_terms = 1 for 32, 64,
 * 96, 128; the Python layer runs other head sizes up to 128 zero-padded to the next one. */
int dta_supported(int32_t dtype, int32_t head_size, int32_t n_terms, int32_t dv);

#ifdef __cplusplus
}
#endif
#endif /* DIFFATTN_H_ */
