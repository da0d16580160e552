// attn_bf16_dq2.hip -- attn_fwd3_kernel, attn_dq2_kernel and attn_dkdv2_kernel (one wave per
// SIMD, compile-time MFMA streams; attn_kernels.h) for bf16, in a unit of its own: the Makefile
// builds it with -mllvm -amdgpu-mfma-vgpr-form=1, so the builtin MFMAs keep their accumulators
// (S', dP: read by the VALU) in VGPRs, while O / dQ / dK / dV stay in AGPRs through mfma_agpr.
#include "attn_kernels.h"

namespace dta {
int launch_attn_dq2_bf16(const BwdParams& p, hipStream_t st) {
#define DTA_D2(HS_, N_, DV_)                                                    \
  if (p.HS == HS_ && p.N == N_ && p.DV == DV_) {                                \
    if constexpr (Dq2Cfg<__bf16, HS_, N_, DV_>::ok) return launch_dq2_t<__bf16, HS_, N_, DV_>(p, st); \
  }
  DTA_FOR_CONFIGS(DTA_D2)
#undef DTA_D2
  return -2;
}
int launch_attn_fwd3_bf16(const FwdParams& p, hipStream_t st) {
#define DTA_F3(HS_, N_, DV_)                                                    \
  if (p.HS == HS_ && p.N == N_ && p.DV == DV_) {                                \
    if constexpr (Fw3Cfg<__bf16, HS_, N_, DV_>::ok) return launch_fwd3_t<__bf16, HS_, N_, DV_>(p, st); \
  }
  DTA_FOR_CONFIGS(DTA_F3)
#undef DTA_F3
  return -2;
}
int launch_attn_dkdv2_bf16(const BwdParams& p, hipStream_t st) {
#define DTA_K2(HS_, N_, DV_)                                                    \
  if (p.HS == HS_ && p.N == N_ && p.DV == DV_) {                                \
    if constexpr (Kv2Cfg<__bf16, HS_, N_, DV_>::ok) return launch_dkdv2_t<__bf16, HS_, N_, DV_>(p, st); \
  }
  DTA_FOR_CONFIGS(DTA_K2)
#undef DTA_K2
  return -2;
}
}  // namespace dta
