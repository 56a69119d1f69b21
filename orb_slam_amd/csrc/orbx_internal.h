// Internal definitions shared by the orbx host code and HIP kernels.
//
// Data layout in HBM (one orbx_ctx, `slots` frames):
//   frames      slots x (w*h)                  input mono8, dense rows
//   pyr_raw     slots x frame_pyr_bytes        padded levels (w_l+32)x(h_l+32),
//                                              rows padded to 64 B; level l at
//                                              LevelGeom::off.  Unblurred.
//   pyr_blur    slots x frame_pyr_bytes        same layout; interior blurred,
//                                              border = unblurred border
//   cell_lists  slots x list_entries  u32      FAST corners per cell, raster
//                                              order, packed score<<24|y<<12|x
//                                              (level coordinates)
//   retain_scratch slots x (list_entries + 4 n_cells) i32  nth_element
//                                              scratch for lists too long for LDS
//   cell_count  slots x n_cells_total i32
//   level_keys  slots x level_entries u32      retained keypoints per level
//   level_count slots x nlevels       i32
//   out_kps     slots x nfeatures     orbx_keypoint (reference output order)
//   out_desc    slots x nfeatures x 32 B
//   out_n       slots                 i32
//   match12     slots x nfeatures     i32      SearchForInitialization result
//   match_n     slots                 i32
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/orbx.h"

namespace orbx {

constexpr int kEdge = 16;        // EDGE_THRESHOLD (src/ORBextractor.cc:77)
constexpr int kHalfPatch = 15;   // HALF_PATCH_SIZE (:76)
constexpr int kPatch = 31;       // PATCH_SIZE (:75)
constexpr int kMaxLevels = 16;
// Largest nfeatures of a context.  The reference's constructor has no bound
// (src/ORBextractor.cc:457-487); its callers use Settings.yaml's nFeatures
// (1000, Data/Settings.yaml) and twice that for the initialisation extractor
// (src/Tracking.cc:128), so 4096 covers nFeatures up to 2048.  Kernels that
// pack a keypoint index into a key field depend on it: the brute-force keys
// (16 bits, orbx_match.hip), the matcher frame views (orbx_search.hip,
// orbx_kfproj.hip); each checks it where it packs.
constexpr int kMaxFeatures = 4096;
constexpr int kGridCols = 64;    // FRAME_GRID_COLS (include/Frame.h:35)
constexpr int kGridRows = 48;    // FRAME_GRID_ROWS (include/Frame.h:36)
#ifndef ORBX_BLUR_STRIP
#define ORBX_BLUR_STRIP 28
#endif
constexpr int kBlurStrip = ORBX_BLUR_STRIP;   // output rows per blur thread (rolling window; chunks of 7)
constexpr int kBlurItems = 256;  // blur threads per block (4 waves, one (strip, column chunk) each)
constexpr int kBlurChunkCols = 62;   // output dword columns per blur wave (+ one halo lane each side)

#ifndef ORBX_RES_ROWS
#define ORBX_RES_ROWS 16
#endif
constexpr int kResRows = ORBX_RES_ROWS;   // output rows per staged resize strip (k_pyr_resize_lds)

struct LevelGeom {
    int w, h;             // level size
    int pw, ph;           // padded size
    int stride;           // row pitch of the padded buffer
    int nvec_resize;      // columns on the SSE2 VResize path (rest: scalar)
    int nvec_blur;        // columns on the SSE2 SymmColumn path
    long long off;        // byte offset inside one frame's pyramid
    int n_desired;        // mnFeaturesPerLevel
    int cell_base;        // first cell of this level in the cell table
    int n_cells;          // levelRows * levelCols
    int level_cols, level_rows;
    int nfeatures_cell;
    int level_off;        // offset (entries) of this level in level_keys
    int level_cap;        // capacity of that slot
    float scale;          // mvScaleFactor[level]
    float patch_size;     // (int)(PATCH_SIZE * scale)
    int res_col_off;      // offset into the resize column table (level >= 1)
    int res_row_off;      // offset into the resize row table
    int res_span;         // max source rows feeding one strip of kResRows output rows
    int res_strip_off;    // res_rows index of this level's per-strip entries (sy0 = first source row)
};

struct CellGeom {
    int level, i, j;
    int ini_x, ini_y;     // ROI origin in level coordinates
    int hx, hy;           // ROI size (FAST runs on rows/cols [3, h-4])
    int valid;            // 0 when the reference skips the cell (h <= 0)
    int list_off;         // offset (entries) in the per-frame corner arena
    int list_cap;         // ceil(iw/2)*ceil(ih/2): bound on NMS survivors
};

struct ResizeCol { int16_t sx0, sx1, a0, a1; };
struct ResizeRow { int16_t sy0, sy1, b0, b1; };

// Extractor configuration and per-image-size geometry (host computed, the
// way OpenCV computes its tables per call).
struct Geometry {
    int nfeatures = 0, nlevels = 0, fast_th = 20;
    float scale_factor = 1.2f;
    std::vector<float> scale, inv_scale;
    std::vector<int> features_per_level;
    std::vector<int> umax;
    int w = 0, h = 0;
    std::vector<LevelGeom> levels;
    std::vector<CellGeom> cells;
    std::vector<ResizeCol> res_cols;
    std::vector<ResizeRow> res_rows;
    long long frame_pyr_bytes = 0;
    int list_entries = 0;     // corner arena entries per frame
    int level_entries = 0;    // level_keys entries per frame
    int max_tile_bytes = 0;   // max hx*hy over cells
    int max_list_cap = 0;     // max list_cap over cells
    int max_level_cap = 0;
    int max_cells_per_level = 0;
    // band cascade of the raw pyramid (k_pyr_cascade): per (band, level) the
    // owned padded rows [x, y) and the computed ROI rows [z, w]; 0 bands when
    // the geometry does not take it (the staged launches run instead)
    std::vector<int4> cascade;
    int cascade_bands = 0, cascade_buf_x = 0, cascade_lds = 0;
    // the single-frame cascade (1024 threads) stages every level's resize
    // column table and its band's row-table slices in LDS after the buffers:
    // cascade_tab_cols entries, then cascade_tab_rows (the most any band needs)
    int cascade_tab_cols = 0, cascade_tab_rows = 0;
};

// ORBextractor constructor tables (src/ORBextractor.cc:457-511).
void init_extractor_tables(Geometry& g, int nfeatures, float scale_factor, int nlevels, int fast_th);
// Per image size: level sizes, cell grid, resize coefficient tables.
// Returns ORBX_OK or ORBX_ERR_UNSUPPORTED for sizes the reference cannot
// handle (empty cell grid, 2x INTER_AREA decimation).
int compute_geometry(Geometry& g, int w, int h);
// The band plan of k_pyr_cascade for the current geometry (fills
// g.cascade*; leaves 0 bands when the frame width is not a multiple of 16 or
// no band count fits lds_target bytes of LDS).
void plan_cascade(Geometry& g, int lds_target);
#ifndef ORBX_CASCADE_LDS
#define ORBX_CASCADE_LDS (40 * 1024)   // 4 workgroups per CU
#endif
constexpr int kCascadeLds = ORBX_CASCADE_LDS;

// Device copies of the geometry tables.
struct DeviceGeometry {
    LevelGeom* levels = nullptr;
    CellGeom* cells = nullptr;
    ResizeCol* res_cols = nullptr;
    ResizeRow* res_rows = nullptr;
    int* umax = nullptr;
};

struct KernelTimer {
    std::string name;
    std::vector<hipEvent_t> start, stop;   // pairs recorded since reset
    int used = 0;
};

struct LbaResident;   // orbx_lba.hip
}  // namespace orbx

namespace orbx {
// Per-slot BoW of device-resident frames (orbx_dev_compute_bow), each array
// slots x nf entries (fv_ptr: slots x (nf + 1); counts: slots x 2 =
// n_words, n_fv_nodes).
constexpr int kBowSortMax = 4096;   // features per frame the block sort holds
struct SlotBowDev {
    int32_t* word;
    double* weight;
    int32_t* node;
    uint32_t* fv_nodes;
    int32_t* fv_ptr;
    int32_t* fv_feat;
    uint32_t* bow_words;
    double* bow_values;
    int32_t* counts;
};
}  // namespace orbx

struct orbx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;      // second half of large extraction batches
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // pipelined extraction in split_ways parts (2..kMaxWays): part i on
    // streams[i] (streams[0] = stream, streams[1] = stream2), released by
    // part i - 1's FAST (ev_part_fast), joined by the match (ev_part_done)
    static constexpr int kMaxWays = 4;
    static constexpr int kDefaultWays = 3;
    int split_ways = kDefaultWays;
    hipStream_t xstreams[kMaxWays - 2] = {};
    hipEvent_t ev_part_fast[kMaxWays] = {}, ev_part_done[kMaxWays] = {};
    bool split = true;                  // run large batches as concurrent parts (split_ways, or halves)
    // Asynchronous matching (orbx_dev_set_async_match): the matching of an
    // extract_match call runs on mstream while later calls extract other
    // slots.  pend[] lists the matches queued on mstream, oldest first: the
    // slots each reads and the event recorded after it.
    // pend[] also lists the asynchronous read-backs of orbx_dev_download_async
    // (queued on mstream too): an extraction rewriting those slots waits.
    static constexpr int kMaxPending = 8;
    struct PendingMatch {
        int lo, hi;
        hipEvent_t done;
    };
    hipStream_t mstream = nullptr;
    hipEvent_t ev_extracted = nullptr;
    hipEvent_t ev_match[kMaxPending] = {};
    PendingMatch pend[kMaxPending] = {};
    int n_pend = 0, next_ev = 0;
    bool async_match = false;
    // Host-fed pipeline (orbx_dev_upload_async): frame uploads queued on
    // ustream (created on first use), each ordered after every extraction
    // queued before it; an extraction of slots an upload writes waits for it.
    static constexpr int kMaxUploads = 4;
    hipStream_t ustream = nullptr;
    hipEvent_t ev_now[kMaxWays] = {};          // "extraction streams so far" marks
    hipEvent_t ev_upload[kMaxUploads] = {};
    PendingMatch uploads[kMaxUploads] = {};
    int n_uploads = 0, next_upload = 0;
    // Single-frame host path (orbx_extract): page-locked staging for the
    // image and the outputs, and the whole call (upload, extraction launches,
    // read-back) captured once per configuration as a hipGraph
    // (orbx_set_launch_mode).
    int launch_mode = 1;                       // 0: stream launches, 1: one captured graph per call
    bool single_frame = false;                // launch_extract: one frame, latency-first launches (graph capture)
    uint8_t* single_out = nullptr;            // its page-locked read-back block (k_describe writes it)
    void* one_in = nullptr;
    size_t one_in_bytes = 0;
    void* one_out = nullptr;
    size_t one_out_bytes = 0;
    hipGraph_t one_graph = nullptr;
    hipGraphExec_t one_exec = nullptr;
    struct GraphKey {                          // configuration the graph was captured for
        unsigned geom_gen = 0;
        int fp_contract = 0, nth_pivot = 0;
        bool valid = false;
        bool operator==(const GraphKey& o) const
        {
            return valid && o.valid && geom_gen == o.geom_gen && fp_contract == o.fp_contract &&
                   nth_pivot == o.nth_pivot;
        }
    };
    GraphKey one_key;
    unsigned geom_gen = 0;                     // bumped whenever set_geometry changes the buffers
    bool stream_dirty = true;   // the context stream got work outside the async pipeline
    orbx::Geometry geom;
    orbx::DeviceGeometry dgeom;
    int max_w = 0, max_h = 0, slots = 0;
    int geom_w = -1, geom_h = -1;   // size the device tables describe
    // device buffers
    uint8_t* frames = nullptr;
    uint8_t* pyr_raw = nullptr;
    uint8_t* pyr_blur = nullptr;
    uint32_t* cell_lists = nullptr;
    int32_t* retain_scratch = nullptr;   // slots x (list_entries + 4 cells)
    int32_t* cell_count = nullptr;
    uint32_t* level_keys = nullptr;
    // HARRIS_SCORE (score_type 0) only: u64 entries, Harris key << 32 | y << 12 | x
    uint64_t* cell_keys64 = nullptr;    // slots x list_entries
    uint64_t* level_keys64 = nullptr;   // slots x level_entries
    int harris = 0;
    int fp_contract = 0;               // orbx_set_fp_contract
    int nth_pivot = ORBX_NTH_PIVOT_GCC48;   // orbx_set_nth_pivot (the reference's documented platforms)
    int32_t* level_count = nullptr;
    orbx_keypoint* out_kps = nullptr;
    uint8_t* out_desc = nullptr;
    int32_t* out_n = nullptr;
    int32_t* match12 = nullptr;
    int32_t* match_n = nullptr;
    int32_t* error_flags = nullptr;   // kernel-side overflow / invariant flags
    // capacities the buffers were allocated for
    long long cap_frame_px = 0;
    long long cap_pyr_bytes = 0;
    long long cap_list_entries = 0;
    long long cap_level_entries = 0;
    int cap_cells = 0;
    int cap_res_cols = 0, cap_res_rows = 0, cap_blur_tiles = 0;
    int4* blur_tiles = nullptr;        // (level, first item, dwords/row, strips) blur blocks
    int4* cascade = nullptr;           // k_pyr_cascade band plan (Geometry::cascade)
    int cap_cascade = 0;
    int blur_tiles_n = 0;
    int last_first = 0, last_count = 0;   // batch of the most recent extract
    // Frame::ComputeImageBounds of the slots' keypoints (orbx_dev_set_image_bounds;
    // has_bounds 0: 0..w x 0..h, the undistorted case) for the device matchers
    int has_bounds = 0;
    float bounds[4] = {0.f, 0.f, 0.f, 0.f};
    // generic scratch for the one-shot matcher / BA entry points
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    void* host_pinned = nullptr;
    size_t host_pinned_bytes = 0;
    // staged pose-optimisation batch (orbx_pose_stage / run / fetch)
    orbx::LbaResident* lba_res = nullptr;   // orbx_lba_stage's batch (orbx_lba.hip)
    // single-problem local BA over several workgroups (k_lba_split): the
    // setting (orbx_lba_set_workgroups; 0 automatic), its device buffers, and
    // the failed flag of the last solve
    int lba_workgroups = 0;
    void* lba_split = nullptr;
    size_t lba_split_bytes = 0;
    // k_lba_split's grid barrier needs all G workgroups resident at once:
    // G is clamped to the device's capacity for the kernel (occupancy query
    // x CUs, cached per record type and LDS size), and a solve whose barrier
    // timed out (bar[1]) is run again on one workgroup (lba_split_fallback).
    // Plain launches by default: a cooperative launch gave the same bits but
    // delayed the other threads' contexts (LoopClosing's calls 0.22 -> 0.51
    // ms beside a local BA, tests/test_threads_gpu.py)
    int lba_split_cap[2] = {0, 0};
    size_t lba_split_cap_lds[2] = {0, 0};
    int lba_last_workgroups = 0;        // G of the last launch (after clamping and fallback)
    bool lba_force_single = false;      // the fallback re-run in progress
    bool lba_split_timed_out = false;   // set by lba_readback
    bool lba_split_fallback = true;     // orbx_debug_lba_split: off = return ORBX_ERR_HIP instead
    int lba_split_coop = 0;             // 1: cooperative launch (-1: where the device offers it)
    int lba_dbg_fail = 0;               // test hook: split launches whose barrier is made to time out
    int lba_dbg_cap = 0;                // test hook: > 0 caps the residency capacity
    int lba_res_iters[2] = {0, 0};      // the resident batch's last run (the fallback re-runs it)
    void* pose_dev = nullptr;
    size_t pose_dev_bytes = 0;
    void* pose_host = nullptr;
    size_t pose_host_bytes = 0;
    bool pose_exact = true;    // orbx_pose_set_exact: sequential sums in g2o's edge order (default)
    int pose_wide_max = 1;     // batches up to this size run a workgroup per frame (k_pose_opt kW > 1)
    int pose_P = 0;
    long long pose_E = 0;
    size_t pose_o_flags = 0, pose_o_out = 0, pose_out_bytes = 0;
    std::vector<int32_t> pose_edge_kp;     // edge -> keypoint index (frame-local)
    std::vector<long long> pose_e0;        // first edge of each frame
    bool pose_ran = false;
    // per-slot BoW (orbx_vocab.hip): one allocation carved into bow; a
    // slot's entry of bow_ready is cleared when the slot is extracted again
    void* bow_dev = nullptr;
    int bow_nf = 0;
    orbx::SlotBowDev bow = {};
    std::vector<uint8_t> bow_ready;
    // timing
    bool timing = false;
    std::string timing_only;   // non-empty: only this timer records (orbx_dev_kernel_time_select)
    std::vector<orbx::KernelTimer> timers;
};

namespace orbx {
// orbx_extract.hip (declared below with the match spec)
// orbx_match.hip
int launch_match_prev(orbx_ctx* ctx, int first, int count, int seq_len, int window,
                      float nnratio, int check_ori, hipStream_t st = nullptr);
int launch_match_bf_prev(orbx_ctx* ctx, int first, int count, int seq_len, int th_low, float nnratio,
                         hipStream_t st = nullptr);
// Extraction of slots [first, first+count) followed by matching each slot
// against its predecessor; with two streams, each half's internal pairs are
// matched right after that half is extracted (overlapping the other half).
struct MatchSpec {
    int kind;           // 0 none, 1 SearchForInitialization, 2 brute force
    int seq_len, window, th_low, check_ori;
    float nnratio;
};
int launch_extract(orbx_ctx* ctx, int first, int count, const MatchSpec* m = nullptr);
// timing helpers (orbx_api.cpp)
void timer_begin(orbx_ctx* ctx, const char* name, hipStream_t st = nullptr);
void timer_end(orbx_ctx* ctx, const char* name, hipStream_t st = nullptr);
int ensure_scratch(orbx_ctx* ctx, size_t bytes);
int ensure_aux_streams(orbx_ctx* ctx);   // stream2, the part streams and mstream (first batch use)
int ensure_geometry(orbx_ctx* ctx, int w, int h);   // device tables and buffers for frames of w x h
void lba_resident_free(orbx_ctx* ctx);
int ensure_pinned(orbx_ctx* ctx, size_t bytes);
}  // namespace orbx

#define ORBX_HIP_CHECK(expr)                              \
    do {                                                  \
        hipError_t _e = (expr);                           \
        if (_e != hipSuccess) return ORBX_ERR_HIP;        \
    } while (0)

// Entry of every API call that touches the context's device state: select
// the device and order ctx->stream after a pending asynchronous match.
inline void ctx_enter(orbx_ctx* ctx)
{
    (void)hipSetDevice(ctx->device);
    ctx->stream_dirty = true;
    if (ctx->n_pend > 0) {   // mstream is in order: its newest event covers all
        (void)hipStreamWaitEvent(ctx->stream, ctx->pend[ctx->n_pend - 1].done, 0);
        ctx->n_pend = 0;
    }
    if (ctx->n_uploads > 0) {   // ustream is in order too
        (void)hipStreamWaitEvent(ctx->stream, ctx->uploads[ctx->n_uploads - 1].done, 0);
        ctx->n_uploads = 0;
    }
}

// Record the end of the work just queued on mstream as a pending entry that
// reads slots [lo, hi) (a match or an asynchronous read-back).
inline hipError_t push_pending(orbx_ctx* ctx, int lo, int hi)
{
    if (ctx->n_pend == orbx_ctx::kMaxPending) {   // table full: retire the oldest
        hipError_t e = hipStreamWaitEvent(ctx->stream, ctx->pend[0].done, 0);
        if (e != hipSuccess) return e;
        for (int i = 1; i < ctx->n_pend; i++) ctx->pend[i - 1] = ctx->pend[i];
        ctx->n_pend--;
    }
    // an event not referenced by any pending entry
    hipEvent_t ev = nullptr;
    for (int t = 0; t < orbx_ctx::kMaxPending && !ev; t++) {
        hipEvent_t c = ctx->ev_match[(ctx->next_ev + t) % orbx_ctx::kMaxPending];
        bool used = false;
        for (int i = 0; i < ctx->n_pend; i++) used = used || ctx->pend[i].done == c;
        if (!used) {
            ev = c;
            ctx->next_ev = (ctx->next_ev + t + 1) % orbx_ctx::kMaxPending;
        }
    }
    hipError_t e = hipEventRecord(ev, ctx->mstream);
    if (e != hipSuccess) return e;
    ctx->pend[ctx->n_pend++] = orbx_ctx::PendingMatch{lo, hi, ev};
    return hipSuccess;
}

// Order stream st after the queued uploads that write a slot of
// [first, first + count) (orbx_dev_upload_async), and forget them.
inline void wait_uploads_overlap(orbx_ctx* ctx, int first, int count, hipStream_t st)
{
    int last = -1;
    for (int i = 0; i < ctx->n_uploads; i++)
        if (first < ctx->uploads[i].hi && first + count > ctx->uploads[i].lo) last = i;
    if (last < 0) return;
    (void)hipStreamWaitEvent(st, ctx->uploads[last].done, 0);
    for (int i = last + 1; i < ctx->n_uploads; i++) ctx->uploads[i - last - 1] = ctx->uploads[i];
    ctx->n_uploads -= last + 1;
}

// Order ctx->stream after every pending match that reads a slot of
// [first, first + count) (and, mstream being in order, after the older ones).
inline void wait_pending_overlap(orbx_ctx* ctx, int first, int count, hipStream_t st)
{
    int last = -1;
    for (int i = 0; i < ctx->n_pend; i++)
        if (first < ctx->pend[i].hi && first + count > ctx->pend[i].lo) last = i;
    if (last < 0) return;
    (void)hipStreamWaitEvent(st, ctx->pend[last].done, 0);
    for (int i = last + 1; i < ctx->n_pend; i++) ctx->pend[i - last - 1] = ctx->pend[i];
    ctx->n_pend -= last + 1;
}
