// Instantiations of the hb_kernels.hpp templates for 16-limb (<= 512-bit) primes.
#include "hb_kernels.hpp"

HB_INST(16)
