// Instantiations of the hb_kernels.hpp templates for 32-limb (<= 1024-bit)
// primes: the encode dispatcher; its passes' kernels are in
// hb_kern_nl32e{0,1,2,3}.hip, the PRF / prove ones in hb_kern_nl32p.hip.
#include "hb_kernels.hpp"

HB_EXTERN_ENC_PASSES(32)
HB_INST_ENC(32)
