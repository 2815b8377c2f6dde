// Instantiations of the hb_kernels.hpp templates for 32-limb (<= 1024-bit)
// primes: the encode kernels (the PRF / prove ones: hb_kern_nl32p.hip).
#include "hb_kernels.hpp"

HB_INST_ENC(32)
