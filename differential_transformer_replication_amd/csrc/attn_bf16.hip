// attn_bf16.hip -- __bf16 instantiations of the attention kernels (attn_kernels.h).
#include "attn_kernels.h"

namespace dta {
int launch_attn_fwd_bf16(const FwdParams& p, hipStream_t st) { return dispatch_fwd<__bf16, false>(p, st); }
int launch_attn_dq_bf16(const BwdParams& p, hipStream_t st) { return dispatch_dq<__bf16, false>(p, st); }
int launch_attn_dkdv_bf16(const BwdParams& p, hipStream_t st) { return dispatch_dkdv<__bf16, false>(p, st); }
bool attn_native_bf16(int hs, int n, int dv) { return native_t<__bf16>(hs, n, dv); }
}  // namespace dta
