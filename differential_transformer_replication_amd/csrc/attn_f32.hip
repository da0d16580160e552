// attn_f32.hip -- float instantiations of the attention kernels (attn_kernels.h).
#include "attn_kernels.h"

namespace dta {
int launch_attn_fwd_f32(const FwdParams& p, hipStream_t st) { return dispatch_fwd<float, false>(p, st); }
int launch_attn_dq_f32(const BwdParams& p, hipStream_t st) { return dispatch_dq<float, false>(p, st); }
int launch_attn_dkdv_f32(const BwdParams& p, hipStream_t st) { return dispatch_dkdv<float, false>(p, st); }
bool attn_native_f32(int hs, int n, int dv) { return native_t<float>(hs, n, dv); }
}  // namespace dta
