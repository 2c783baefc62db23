/* crdtm_test.h — test-only entry points of libcrdtm.so. Not part of the
 * drop-in ABI (include/crdtm.h) and not a reference surface: they act only
 * when the process sets CRDTM_TEST_HOOKS=1 (else CRDTM_E_ARG). */
#ifndef CRDTM_TEST_H
#define CRDTM_TEST_H

#include "crdtm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Overwrite one word of the device state (field: 0 s_next, 1 s_child,
 * 2 s_dict, 3 d_sent) so the tests can check that the host readers
 * (crdtm_tree_canonical, crdtm_tree_walk) refuse an unsound state with
 * CRDTM_E_STATE instead of following a bad index. The tree's merge indexes
 * (incremental key index, level-replay index, clean-flat mark) are dropped:
 * no later merge trusts them. */
int crdtm_debug_poke(crdtm_tree *tree, int field, uint64_t index, uint32_t value);

#ifdef __cplusplus
}
#endif

#endif
