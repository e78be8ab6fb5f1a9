// abi.hip — version and status strings of the C ABI (include/hygrid.h).
#include "common.h"

extern "C" {

int hg_abi_version(void) { return HG_ABI_VERSION; }

const char* hg_strerror(int status) {
    switch (status) {
    case HG_OK: return "success";
    case HG_EINVAL: return "invalid argument";
    case HG_EDTYPE: return "unsupported dtype";
    case HG_ESHAPE: return "input too small for the operator, or size overflow";
    case HG_EUNSUP: return "parameter combination not implemented";
    default:
        if (status > 0) return hipGetErrorString(static_cast<hipError_t>(status));
        return "unknown status";
    }
}

}  // extern "C"
