// hb_build_id.cpp -- provenance of libhbswizzle.so (include/hbswizzle.h).
// HB_BUILD_ID and HB_BUILD_FLAGS_STR come from csrc/Makefile: the SHA-256 of
// every source file of the library plus the compiler flags
// (heartbeat_amd/build_id.py), and those flags.
#include "../../include/hbswizzle.h"

#ifndef HB_BUILD_ID
#error "HB_BUILD_ID is set by csrc/Makefile"
#endif
#ifndef HB_BUILD_FLAGS_STR
#error "HB_BUILD_FLAGS_STR is set by csrc/Makefile"
#endif

extern "C" {

const char *hb_build_id(void) { return HB_BUILD_ID; }

const char *hb_build_flags_string(void) { return HB_BUILD_FLAGS_STR; }

}  // extern "C"
