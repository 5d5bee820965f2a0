// ABI metadata for libpcops.so (include/pcops.h).
#include "common.h"

extern "C" const char *pcops_status_string(int status) {
  switch (status) {
    case PCOPS_OK: return "ok";
    case PCOPS_ERR_INVALID: return "invalid argument (sizes or null pointers)";
    case PCOPS_ERR_LAUNCH: return "HIP kernel launch failed";
    case PCOPS_ERR_WORKSPACE: return "workspace missing or too small";
    case PCOPS_ERR_UNSUPPORTED: return "unsupported configuration";
    default: return "unknown status";
  }
}

extern "C" int pcops_abi_version(void) { return 2; }
