// gs_build_id: the digest of the sources this library was built from
// (Makefile SRC_SHA over csrc/ and include/gpusched.h).  tests/test_abi.py
// and smoke() compare it with the tree they run from.
#ifndef GS_SOURCE_SHA
#define GS_SOURCE_SHA "unknown"
#endif
extern "C" const char* gs_build_id(void) { return GS_SOURCE_SHA; }
