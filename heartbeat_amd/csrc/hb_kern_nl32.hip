// Instantiations of the hb_kernels.hpp templates for 32-limb (<= 1024-bit) primes.
#include "hb_kernels.hpp"

HB_INST(32)
