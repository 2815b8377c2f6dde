// Instantiations of the split wide-prime MAC kernels (hb_wide.hpp) for 16-,
// 32- and 64-limb primes.
#include "hb_wide.hpp"

HB_INST_WIDE(16)
HB_INST_WIDE(32)
#if !defined(HB_NO_NL64)
HB_INST_WIDE(64)
#endif
