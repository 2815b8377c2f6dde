// The fused verify (hb_verify_fused_kernel) for 8-, 16- and 32-limb primes, in a
// translation unit of its own (parallel build).
#include "hb_kernels.hpp"

HB_INST_VERIFY_FUSED(8)
HB_INST_VERIFY_FUSED(16)
HB_INST_VERIFY_FUSED(32)
