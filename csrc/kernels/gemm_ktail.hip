// Ragged-K (K % 64 != 0) instantiations of the plain-operand bf16 GEMM kernels
// (gemm_core.h): the last K-tile masks its out-of-range k through the buffer
// descriptor's range check.  Split from gemm.hip so the two compile in parallel.
#include "gemm_core.h"

namespace hetu {
namespace gemm {
template int launch_buf<false>(const bf16*, const bf16*, int, int, int64_t, int64_t, int64_t, int64_t, const Epi&,
                               int64_t, int64_t, int64_t, int, int, hipStream_t, int);
}  // namespace gemm
}  // namespace hetu
