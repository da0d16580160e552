// attn_f16_drop.hip -- _Float16 instantiations of the attention kernels with attention
// dropout compiled in (p > 0 in training; diff_transformer.py:66-67,
// Ndiff_transformer.py:114).  A separate unit so the p = 0 kernels build in parallel.
#include "attn_kernels.h"

namespace dta {
int launch_attn_fwd_f16_drop(const FwdParams& p, hipStream_t st) { return dispatch_fwd<_Float16, true>(p, st); }
int launch_attn_dq_f16_drop(const BwdParams& p, hipStream_t st) { return dispatch_dq<_Float16, true>(p, st); }
int launch_attn_dkdv_f16_drop(const BwdParams& p, hipStream_t st) { return dispatch_dkdv<_Float16, true>(p, st); }
}  // namespace dta
