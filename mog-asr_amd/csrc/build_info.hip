// Build provenance: the hash of the sources this library was compiled from
// (Makefile: sha256 of csrc/*.hip, csrc/*.h and include/*.h, in that sorted
// order, first 16 hex digits), so the host can refuse a library that is older
// than the sources next to it (mog_air._lib.load).
#include <string.h>

#include "build_id.h"
#include "mog_common.h"

extern "C" int mog_build_id(char* out, int cap) {
  MOG_CHECK_ARG(out && cap > (int)strlen(MOG_BUILD_ID));
  memcpy(out, MOG_BUILD_ID, strlen(MOG_BUILD_ID) + 1);
  return 0;
}
