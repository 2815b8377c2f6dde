// Instantiations of the hb_kernels.hpp templates for 64-limb (<= 2048-bit)
// primes: the encode kernels (the PRF / prove ones: hb_kern_nl64p.hip).
#include "hb_kernels.hpp"

HB_INST_ENC(64)
