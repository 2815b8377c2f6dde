// 32-limb encode kernels of pass 0 (hb_launch_encode_pass; see hb_kern_nl32.hip).
#include "hb_kernels.hpp"

HB_INST_ENC_PASS(32, 0)
