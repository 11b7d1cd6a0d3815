// Thread-local error reporting for the pcs C ABI (no exceptions cross the boundary).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../include/pcs.h"

static thread_local char g_err[512] = "";

int pcs_set_error(hipError_t e, const char *where) {
  snprintf(g_err, sizeof g_err, "%s: %s (%d)", where, hipGetErrorString(e), (int)e);
  return -(int)e;
}

int pcs_set_einval(const char *where, const char *msg) {
  snprintf(g_err, sizeof g_err, "%s: %s", where, msg);
  return PCS_EINVAL;
}

extern "C" const char *pcs_last_error(void) { return g_err; }
// PCS_ABI_VERSION (include/pcs.h): bumped whenever an argument struct's layout or an entry
// point's signature changes; _lib.load() refuses a library whose number differs
extern "C" int pcs_abi_version(void) { return PCS_ABI_VERSION; }
