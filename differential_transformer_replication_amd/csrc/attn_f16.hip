// attn_f16.hip -- _Float16 instantiations of the attention kernels (attn_kernels.h).
#include "attn_kernels.h"

namespace dta {
int launch_attn_fwd_f16(const FwdParams& p, hipStream_t st) { return dispatch_fwd<_Float16, false>(p, st); }
int launch_attn_dq_f16(const BwdParams& p, hipStream_t st) { return dispatch_dq<_Float16, false>(p, st); }
int launch_attn_dkdv_f16(const BwdParams& p, hipStream_t st) { return dispatch_dkdv<_Float16, false>(p, st); }
bool attn_native_f16(int hs, int n, int dv) { return native_t<_Float16>(hs, n, dv); }
}  // namespace dta
