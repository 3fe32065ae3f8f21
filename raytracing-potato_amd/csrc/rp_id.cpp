// rp_build_id (include/rp.h): the hash build_id.sh makes of the render kernel's, the tree builders' and the scheduling
// code's machine code (Makefile), compiled into this object alone so that rp_api.o itself can enter the hash.
#include "rp.h"

#ifndef RP_BUILD_ID
#error "build with the Makefile: it passes -include build_id.h"
#endif

extern "C" const char* rp_build_id(void) { return RP_BUILD_ID; }
