// Entry points of include/orbx.h whose device implementation is not built
// yet.  They fail loudly (ORBX_ERR_UNSUPPORTED); there is no CPU fallback.
#include "orbx_internal.h"

extern "C" {
int orbx_lba_solve(orbx_ctx*, orbx_ba_problem*, int, int, const volatile uint8_t*, uint8_t*, uint8_t*, orbx_ba_stats*) { return ORBX_ERR_UNSUPPORTED; }
int orbx_lba_solve_batch(orbx_ctx*, int, orbx_ba_problem*, int, int, uint8_t* const*, uint8_t* const*, orbx_ba_stats*) { return ORBX_ERR_UNSUPPORTED; }
}
