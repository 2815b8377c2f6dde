// Instantiations of the hb_kernels.hpp templates for 64-limb (<= 2048-bit)
// primes: the encode dispatcher; its passes' kernels are in
// hb_kern_nl64e{0,1,2,3}.hip, the PRF / prove ones in hb_kern_nl64p.hip.
#include "hb_kernels.hpp"

HB_EXTERN_ENC_PASSES(64)
HB_INST_ENC(64)
