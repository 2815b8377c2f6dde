// 64-limb encode kernels of pass 3 (hb_launch_encode_pass; see hb_kern_nl64.hip).
#include "hb_kernels.hpp"

HB_INST_ENC_PASS(64, 3)
