// cvlite C ABI — library-level entry points (version).
#include "cvl_common.h"
#include <string.h>

extern "C" int cvl_version(void) { return 100; }  // 0.1.0

// CVL_DISPATCH test hooks (cvl_common.h): "key" (= 1) or "key=value", comma-separated
int cvl_dispatch_int(const char* key, int dflt) {
  const char* v = getenv("CVL_DISPATCH");
  if (!v || !v[0]) return dflt;
  const size_t kl = strlen(key);
  for (const char* p = v; *p;) {
    const char* e = strchr(p, ',');
    const size_t n = e ? (size_t)(e - p) : strlen(p);
    if (n >= kl && strncmp(p, key, kl) == 0 && (n == kl || p[kl] == '=')) return n == kl ? 1 : atoi(p + kl + 1);
    if (!e) break;
    p = e + 1;
  }
  return dflt;
}
