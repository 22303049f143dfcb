// cvlite C ABI — library-level entry points (version).
#include "cvl_common.h"

extern "C" int cvl_version(void) { return 100; }  // 0.1.0
