// stubs.cpp — entry points not yet implemented in this build.
#include "../../include/crdtm.h"
extern "C" {
int crdtm_forest_apply(crdtm_ctx*, int64_t, const crdtm_ops*, const uint32_t*, uint64_t, int, int32_t*, int64_t*,
                       uint32_t*, uint64_t*) { return CRDTM_E_ARG; }
}
