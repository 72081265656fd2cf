// Library-level entry points: version and status strings.
#include "common.h"

extern "C" int kge_version(void) { return 100; }  // 1.0.0

extern "C" const char* kge_error_string(int status) {
  switch (status) {
    case 0: return "ok";
    case KGE_ERR_ARG: return "kgescore: invalid argument (shape, enum or null pointer)";
    case KGE_ERR_ALIGN: return "kgescore: misaligned pointer or leading dimension";
    case KGE_ERR_NOGPU: return "kgescore: no gfx950 device";
    case KGE_ERR_SCRATCH:
      return "kgescore: the problem needs more scratch than the library's static buffer holds "
             "(use the entry point that takes a caller workspace)";
    default: return hipGetErrorString((hipError_t)status);
  }
}
