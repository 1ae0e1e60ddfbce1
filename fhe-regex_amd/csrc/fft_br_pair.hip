// The pair shape's blind-rotation kernel (k_blind_rotate_fft<2048, 1, 4, true, 2>, fft_br.hip)
// in a translation unit of its own, so the Makefile can compile it under the max-ILP machine
// scheduler (PAIR_SCHED) while every other kernel keeps the default.  Device code and the
// kernel template come from fft_br.hip; its host side is left out (FR_BR_PAIR_TU).
#define FR_BR_PAIR_TU 1
#include "fft_br.hip"

namespace fr {
template __global__ void k_blind_rotate_fft<2048, 1, 4, true, 2>(const uint64_t*, int, int, const DevGate*, int,
                                                                  const double2*, const double2*, const double2*,
                                                                  const uint16_t*, uint64_t*, int);
}  // namespace fr
