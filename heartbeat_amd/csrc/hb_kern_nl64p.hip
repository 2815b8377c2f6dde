// Instantiations of the hb_kernels.hpp templates for 64-limb (<= 2048-bit)
// primes: PRF batches, Montgomery conversion, weighted sums and prove (the
// encode kernels: hb_kern_nl64.hip).
#include "hb_kernels.hpp"

HB_INST_PRF(64)
