// FP256BN (AMCL) instances of the idemix identity kernels (idemix_identity.hip):
// the same source compiled as a second translation unit with the host side left
// out, so the two curves' pairing kernels compile in parallel.
#define IDV_FBN_TU 1
#include "idemix_identity.hip"

namespace idv {
template void launch_tvals<FbnCurve>(const Chain&);
template void launch_batch<FbnCurve>(const Chain&);
template void launch_pairing<FbnCurve>(const Chain&, unsigned, bool);
template void launch_lines<FbnCurve>(const uint8_t*, uint32_t*, int32_t*, hipStream_t);
}  // namespace idv
