// Entry points of include/orbx.h whose device implementation is not built
// yet.  They fail loudly (ORBX_ERR_UNSUPPORTED); there is no CPU fallback.
#include "orbx_internal.h"

extern "C" {
int orbx_hamming_bf(orbx_ctx*, const uint8_t*, int, const uint8_t*, int, int32_t*, int32_t*, int32_t*) { return ORBX_ERR_UNSUPPORTED; }
int orbx_match_bf(orbx_ctx*, const uint8_t*, int, const uint8_t*, int, int, float, int32_t*, int*) { return ORBX_ERR_UNSUPPORTED; }
int orbx_search_for_initialization(orbx_ctx*, const orbx_frame_view*, const orbx_frame_view*, float*, int32_t*, int, float, int, int*) { return ORBX_ERR_UNSUPPORTED; }
int orbx_window_search(orbx_ctx*, const orbx_frame_view*, const orbx_frame_view*, const uint8_t*, int, int, int, float, int, int32_t*, int*) { return ORBX_ERR_UNSUPPORTED; }
int orbx_search_by_projection_pair(orbx_ctx*, const orbx_frame_view*, const orbx_frame_view*, const float*, const uint8_t*, const uint8_t*, const float*, const float*, int, float, int32_t*, int*) { return ORBX_ERR_UNSUPPORTED; }
int orbx_search_by_projection_motion(orbx_ctx*, const orbx_frame_view*, const orbx_frame_view*, const float*, const uint8_t*, const uint8_t*, const float*, const float*, float, int, int32_t*, int*) { return ORBX_ERR_UNSUPPORTED; }
int orbx_search_by_projection_local(orbx_ctx*, const orbx_frame_view*, int, const uint8_t*, const float*, const int32_t*, const float*, const uint8_t*, const uint8_t*, float, float, int32_t*, int*) { return ORBX_ERR_UNSUPPORTED; }
int orbx_lba_solve(orbx_ctx*, orbx_ba_problem*, int, int, const volatile uint8_t*, uint8_t*, uint8_t*, orbx_ba_stats*) { return ORBX_ERR_UNSUPPORTED; }
int orbx_lba_solve_batch(orbx_ctx*, int, orbx_ba_problem*, int, int, uint8_t* const*, uint8_t* const*, orbx_ba_stats*) { return ORBX_ERR_UNSUPPORTED; }
}
