// Instantiations of the hb_kernels.hpp templates for 8-limb (<= 256-bit) primes.
#include "hb_kernels.hpp"

HB_INST(8)
