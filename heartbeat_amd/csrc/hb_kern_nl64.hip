// Instantiations of the hb_kernels.hpp templates for 64-limb (<= 2048-bit) primes.
#include "hb_kernels.hpp"

HB_INST(64)
