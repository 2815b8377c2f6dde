// Instantiations of the hb_kernels.hpp templates for 32-limb (<= 1024-bit)
// primes: PRF batches, Montgomery conversion, weighted sums and prove (the
// encode kernels: hb_kern_nl32.hip).
#include "hb_kernels.hpp"

HB_INST_PRF(32)
