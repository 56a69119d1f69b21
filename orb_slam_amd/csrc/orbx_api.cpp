// C ABI of liborbx (include/orbx.h): context lifetime, device buffers,
// host <-> HBM transfers, kernel timing, and the drop-in entry points that
// replace ORBextractor::operator() / ORBmatcher / Optimizer calls.
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <new>

#include "orbx_internal.h"

using namespace orbx;

namespace orbx {

static KernelTimer* find_timer(orbx_ctx* ctx, const char* name)
{
    for (auto& t : ctx->timers)
        if (t.name == name) return &t;
    ctx->timers.push_back(KernelTimer{name, {}, {}, 0});
    return &ctx->timers.back();
}

void timer_begin(orbx_ctx* ctx, const char* name, hipStream_t st)
{
    if (!ctx->timing || (!ctx->timing_only.empty() && ctx->timing_only != name)) return;
    KernelTimer* t = find_timer(ctx, name);
    if (t->used == (int)t->start.size()) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
        t->start.push_back(a);
        t->stop.push_back(b);
    }
    (void)hipEventRecord(t->start[t->used], st ? st : ctx->stream);
}

void timer_end(orbx_ctx* ctx, const char* name, hipStream_t st)
{
    if (!ctx->timing || (!ctx->timing_only.empty() && ctx->timing_only != name)) return;
    KernelTimer* t = find_timer(ctx, name);
    if (t->used >= (int)t->stop.size()) return;
    (void)hipEventRecord(t->stop[t->used], st ? st : ctx->stream);
    t->used++;
}

int ensure_scratch(orbx_ctx* ctx, size_t bytes)
{
    if (bytes <= ctx->scratch_bytes) return ORBX_OK;
    if (ctx->scratch) hipFree(ctx->scratch);
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
    if (hipMalloc(&ctx->scratch, bytes) != hipSuccess) return ORBX_ERR_NOMEM;
    ctx->scratch_bytes = bytes;
    return ORBX_OK;
}

int ensure_pinned(orbx_ctx* ctx, size_t bytes)
{
    if (bytes <= ctx->host_pinned_bytes) return ORBX_OK;
    if (ctx->host_pinned) hipHostFree(ctx->host_pinned);
    ctx->host_pinned = nullptr;
    ctx->host_pinned_bytes = 0;
    if (hipHostMalloc(&ctx->host_pinned, bytes, hipHostMallocDefault) != hipSuccess) return ORBX_ERR_NOMEM;
    ctx->host_pinned_bytes = bytes;
    return ORBX_OK;
}

template <typename T>
static int realloc_dev(T*& p, size_t count)
{
    if (p) (void)hipFree(p);
    p = nullptr;
    if (count == 0) count = 1;
    if (hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)) != hipSuccess) return ORBX_ERR_NOMEM;
    return ORBX_OK;
}

static void free_buffers(orbx_ctx* ctx)
{
    void* ptrs[] = {ctx->frames, ctx->pyr_raw, ctx->pyr_blur, ctx->cell_lists, ctx->retain_scratch, ctx->cell_count,
                    ctx->level_keys, ctx->cell_keys64, ctx->level_keys64, ctx->level_count, ctx->out_kps, ctx->out_desc, ctx->out_n,
                    ctx->match12, ctx->match_n, ctx->error_flags, ctx->dgeom.levels, ctx->dgeom.cells,
                    ctx->dgeom.res_cols, ctx->dgeom.res_rows, ctx->dgeom.umax, ctx->blur_tiles, ctx->cascade,
                    ctx->scratch, ctx->pose_dev, ctx->bow_dev};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (ctx->host_pinned) (void)hipHostFree(ctx->host_pinned);
    if (ctx->pose_host) (void)hipHostFree(ctx->pose_host);
}

// Make the device tables and buffers describe frames of w x h.
static int set_geometry(orbx_ctx* ctx, int w, int h)
{
    if (ctx->geom_w == w && ctx->geom_h == h) return ORBX_OK;
    if (w > ctx->max_w || h > ctx->max_h) return ORBX_ERR_CAPACITY;
    hipStreamSynchronize(ctx->stream);
    Geometry& g = ctx->geom;
    int r = compute_geometry(g, w, h);
    if (r != ORBX_OK) return r;
    plan_cascade(g, kCascadeLds);
    const int S = ctx->slots;
    // per-slot buffers depend on the frame size / config only
    if ((long long)w * h > (long long)ctx->cap_frame_px) {
        if ((r = realloc_dev(ctx->frames, (size_t)S * w * h)) != ORBX_OK) return r;
        ctx->cap_frame_px = (long long)w * h;
    }
    if (g.frame_pyr_bytes > ctx->cap_pyr_bytes) {
        if ((r = realloc_dev(ctx->pyr_raw, (size_t)S * g.frame_pyr_bytes)) != ORBX_OK) return r;
        if ((r = realloc_dev(ctx->pyr_blur, (size_t)S * g.frame_pyr_bytes)) != ORBX_OK) return r;
        ctx->cap_pyr_bytes = g.frame_pyr_bytes;
    }
    if (g.list_entries + 4LL * (long long)g.cells.size() > ctx->cap_list_entries) {
        const long long e = g.list_entries + 4LL * (long long)g.cells.size();
        if ((r = realloc_dev(ctx->cell_lists, (size_t)S * e)) != ORBX_OK) return r;
        if ((r = realloc_dev(ctx->retain_scratch, (size_t)S * e)) != ORBX_OK) return r;
        if (ctx->harris && (r = realloc_dev(ctx->cell_keys64, (size_t)S * e)) != ORBX_OK) return r;
        ctx->cap_list_entries = e;
    }
    if ((int)g.cells.size() > ctx->cap_cells) {
        if ((r = realloc_dev(ctx->cell_count, (size_t)S * g.cells.size())) != ORBX_OK) return r;
        if ((r = realloc_dev(ctx->dgeom.cells, g.cells.size())) != ORBX_OK) return r;
        ctx->cap_cells = (int)g.cells.size();
    }
    if (g.level_entries > ctx->cap_level_entries) {
        if ((r = realloc_dev(ctx->level_keys, (size_t)S * g.level_entries)) != ORBX_OK) return r;
        if (ctx->harris && (r = realloc_dev(ctx->level_keys64, (size_t)S * g.level_entries)) != ORBX_OK) return r;
        ctx->cap_level_entries = g.level_entries;
    }
    if ((int)g.res_cols.size() > ctx->cap_res_cols) {
        if ((r = realloc_dev(ctx->dgeom.res_cols, g.res_cols.size())) != ORBX_OK) return r;
        ctx->cap_res_cols = (int)g.res_cols.size();
    }
    if ((int)g.res_rows.size() > ctx->cap_res_rows) {
        if ((r = realloc_dev(ctx->dgeom.res_rows, g.res_rows.size())) != ORBX_OK) return r;
        ctx->cap_res_rows = (int)g.res_rows.size();
    }
    // blur work blocks: per level, wave items = (row strip, chunk of
    // kBlurChunkCols dword columns) in strip-major order; one block = 4
    // consecutive wave items of a level.
    std::vector<int4> tiles;
    for (int l = 0; l < g.nlevels; l++) {
        const LevelGeom& L = g.levels[l];
        const int ndw = L.stride / 4, nstrips = (L.ph + kBlurStrip - 1) / kBlurStrip;
        const int nchunks = (ndw + kBlurChunkCols - 1) / kBlurChunkCols;
        for (int b = 0; b < nchunks * nstrips; b += kBlurItems / 64) tiles.push_back(make_int4(l, b, nchunks, nstrips));
    }
    if ((int)tiles.size() > ctx->cap_blur_tiles) {
        if ((r = realloc_dev(ctx->blur_tiles, tiles.size())) != ORBX_OK) return r;
        ctx->cap_blur_tiles = (int)tiles.size();
    }
    ctx->blur_tiles_n = (int)tiles.size();
    ORBX_HIP_CHECK(hipMemcpy(ctx->dgeom.levels, g.levels.data(), g.levels.size() * sizeof(LevelGeom), hipMemcpyHostToDevice));
    ORBX_HIP_CHECK(hipMemcpy(ctx->dgeom.cells, g.cells.data(), g.cells.size() * sizeof(CellGeom), hipMemcpyHostToDevice));
    if (!g.res_cols.empty())
        ORBX_HIP_CHECK(hipMemcpy(ctx->dgeom.res_cols, g.res_cols.data(), g.res_cols.size() * sizeof(ResizeCol), hipMemcpyHostToDevice));
    if (!g.res_rows.empty())
        ORBX_HIP_CHECK(hipMemcpy(ctx->dgeom.res_rows, g.res_rows.data(), g.res_rows.size() * sizeof(ResizeRow), hipMemcpyHostToDevice));
    ORBX_HIP_CHECK(hipMemcpy(ctx->blur_tiles, tiles.data(), tiles.size() * sizeof(int4), hipMemcpyHostToDevice));
    if ((int)g.cascade.size() > ctx->cap_cascade) {
        if ((r = realloc_dev(ctx->cascade, g.cascade.size())) != ORBX_OK) return r;
        ctx->cap_cascade = (int)g.cascade.size();
    }
    if (!g.cascade.empty())
        ORBX_HIP_CHECK(hipMemcpy(ctx->cascade, g.cascade.data(), g.cascade.size() * sizeof(int4), hipMemcpyHostToDevice));
    // The retain kernel keeps per-cell state for up to 256 cells per level.
    if (g.max_cells_per_level > 256) return ORBX_ERR_UNSUPPORTED;
    ctx->geom_w = w;
    ctx->geom_h = h;
    ctx->geom_gen++;   // a captured single-frame graph holds the old tables and buffers
    return ORBX_OK;
}

// The streams of the batch pipeline (stream2, the part streams, the match
// stream), created on first use.  HIP maps each new stream of a process onto
// its hardware queues in turn (GPU_MAX_HW_QUEUES, 4 by default): a context
// that only ever serves single calls -- the Tracking, LocalMapping and
// LoopClosing threads of the reference each hold one -- then keeps one
// stream, and three such contexts get a hardware queue each instead of
// sharing them with idle pipeline streams (a call queued behind another
// context's 3 ms local BA on a shared queue waits for it).
int ensure_aux_streams(orbx_ctx* ctx)
{
    if (ctx->mstream) return ORBX_OK;
    hipStream_t s2 = nullptr, ms = nullptr, xs[orbx_ctx::kMaxWays - 2] = {};
    bool ok = hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&ms, hipStreamNonBlocking) == hipSuccess;
    for (int i = 0; ok && i < orbx_ctx::kMaxWays - 2; i++)
        ok = hipStreamCreateWithFlags(&xs[i], hipStreamNonBlocking) == hipSuccess;
    if (!ok) {
        for (hipStream_t s : {s2, ms, xs[0], xs[1]})
            if (s) (void)hipStreamDestroy(s);
        return ORBX_ERR_HIP;
    }
    ctx->stream2 = s2;
    for (int i = 0; i < orbx_ctx::kMaxWays - 2; i++) ctx->xstreams[i] = xs[i];
    ctx->mstream = ms;   // last: its presence marks the set complete
    return ORBX_OK;
}

int ensure_geometry(orbx_ctx* ctx, int w, int h) { return set_geometry(ctx, w, h); }

// Make stream dst wait for everything queued so far on the extraction streams
// (the context stream, stream2 and the pipeline part streams).
static int order_after_extraction(orbx_ctx* ctx, hipStream_t dst)
{
    const hipStream_t S[orbx_ctx::kMaxWays] = {ctx->stream, ctx->stream2, ctx->xstreams[0], ctx->xstreams[1]};
    for (int i = 0; i < orbx_ctx::kMaxWays; i++) {
        if (!S[i] || S[i] == dst) continue;
        ORBX_HIP_CHECK(hipEventRecord(ctx->ev_now[i], S[i]));
        ORBX_HIP_CHECK(hipStreamWaitEvent(dst, ctx->ev_now[i], 0));
    }
    return ORBX_OK;
}

static void drop_single_graph(orbx_ctx* ctx)
{
    if (ctx->one_exec) (void)hipGraphExecDestroy(ctx->one_exec);
    if (ctx->one_graph) (void)hipGraphDestroy(ctx->one_graph);
    ctx->one_exec = nullptr;
    ctx->one_graph = nullptr;
    ctx->one_key = orbx_ctx::GraphKey{};
}

static int check_errors(orbx_ctx* ctx)
{
    int32_t flags = 0;
    ORBX_HIP_CHECK(hipMemcpy(&flags, ctx->error_flags, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (flags) {
        hipMemset(ctx->error_flags, 0, sizeof(int32_t));
        return ORBX_ERR_CAPACITY;
    }
    return ORBX_OK;
}

}  // namespace orbx

extern "C" {

const char* orbx_version(void) { return "orbx 0.1 (gfx950)"; }

int orbx_abi_version(void) { return ORBX_ABI_VERSION; }

/* Diagnostics (not in include/orbx.h): the device error flags of the last
 * batch without clearing them (1: a cell list overflowed its capacity,
 * 2: a level list overflowed). */
int orbx_debug_error_flags(orbx_ctx* ctx)
{
    if (!ctx) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    int32_t flags = 0;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(&flags, ctx->error_flags, sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return ORBX_ERR_HIP;
    return flags;
}

/* Diagnostics: per cell of slot `slot`'s last extraction, 8 ints: level, i,
 * j, ini_x, ini_y, hx, hy, FAST corner count (list capacity in the 9th).
 * Returns the number of cells. */
int orbx_debug_cells(orbx_ctx* ctx, int slot, int32_t* out, int cap)
{
    if (!ctx || slot < 0 || slot >= ctx->slots) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    const Geometry& g = ctx->geom;
    const int n = (int)g.cells.size();
    if (cap < 9 * n) return ORBX_ERR_CAPACITY;
    std::vector<int32_t> cnt(n);
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(cnt.data(), ctx->cell_count + (size_t)slot * n, 4 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
        return ORBX_ERR_HIP;
    for (int c = 0; c < n; c++) {
        const CellGeom& C = g.cells[c];
        const int32_t v[9] = {C.level, C.i, C.j, C.ini_x, C.ini_y, C.hx, C.hy, cnt[c], C.list_cap};
        for (int k = 0; k < 9; k++) out[9 * c + k] = v[k];
    }
    return n;
}

int orbx_create(orbx_ctx** out, int device, int nfeatures, float scale_factor, int nlevels,
                int score_type, int fast_th, int max_w, int max_h, int max_batch)
{
    if (!out) return ORBX_ERR_ARG;
    *out = nullptr;
    if (nfeatures <= 0 || nfeatures > kMaxFeatures || nlevels <= 0 || nlevels > kMaxLevels ||
        !(scale_factor > 1.0f) || max_w <= 0 || max_h <= 0 || max_w > 4095 || max_h > 4095 ||
        max_batch <= 0 || fast_th < 1 || fast_th > 255)
        return ORBX_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ORBX_ERR_HIP;
    if (device < 0 || device >= ndev) return ORBX_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ERR_HIP;
    orbx_ctx* ctx = new (std::nothrow) orbx_ctx();
    if (!ctx) return ORBX_ERR_NOMEM;
    ctx->device = device;
    ctx->max_w = max_w;
    ctx->max_h = max_h;
    ctx->slots = max_batch;
    // ORB::HARRIS_SCORE == 0 selects Harris responses; any other value is
    // FAST_SCORE, as in the reference (src/ORBextractor.cc:616)
    ctx->harris = score_type == 0;
    init_extractor_tables(ctx->geom, nfeatures, scale_factor, nlevels, fast_th);
    int r = ORBX_OK;
    const int S = max_batch;
    // the context stream; a batch context (several slots) also creates the
    // pipeline's part and match streams now, right after it -- HIP maps the
    // streams of a process onto its hardware queues in creation order, and
    // created together they take neighbouring queues (created later, between
    // other contexts' streams, they were measured to share queues: c2
    // 249 k -> 226-230 k frames/s on one box).  A one-slot context (the
    // reference's per-thread extractor / matcher / optimizer) keeps one
    // stream and creates the others only if a batch call needs them
    // (ensure_aux_streams), so several such contexts get a queue each.
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) r = ORBX_ERR_HIP;
    if (r == ORBX_OK && max_batch > 1) r = ensure_aux_streams(ctx);
    if (r == ORBX_OK && (hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming) != hipSuccess ||
                         hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming) != hipSuccess ||
                         hipEventCreateWithFlags(&ctx->ev_extracted, hipEventDisableTiming) != hipSuccess))
        r = ORBX_ERR_HIP;
    for (int i = 0; r == ORBX_OK && i < orbx_ctx::kMaxPending; i++)
        if (hipEventCreateWithFlags(&ctx->ev_match[i], hipEventDisableTiming) != hipSuccess) r = ORBX_ERR_HIP;
    for (int i = 0; r == ORBX_OK && i < orbx_ctx::kMaxWays; i++)
        if (hipEventCreateWithFlags(&ctx->ev_part_fast[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ctx->ev_part_done[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ctx->ev_now[i], hipEventDisableTiming) != hipSuccess)
            r = ORBX_ERR_HIP;
    for (int i = 0; r == ORBX_OK && i < orbx_ctx::kMaxUploads; i++)
        if (hipEventCreateWithFlags(&ctx->ev_upload[i], hipEventDisableTiming) != hipSuccess) r = ORBX_ERR_HIP;
    if (r == ORBX_OK) r = realloc_dev(ctx->dgeom.levels, kMaxLevels);
    if (r == ORBX_OK) r = realloc_dev(ctx->dgeom.umax, kHalfPatch + 1);
    if (r == ORBX_OK) r = realloc_dev(ctx->level_count, (size_t)S * nlevels);
    if (r == ORBX_OK) r = realloc_dev(ctx->out_kps, (size_t)S * nfeatures);
    if (r == ORBX_OK) r = realloc_dev(ctx->out_desc, (size_t)S * nfeatures * 32);
    if (r == ORBX_OK) r = realloc_dev(ctx->out_n, (size_t)S);
    if (r == ORBX_OK) r = realloc_dev(ctx->match12, (size_t)S * nfeatures);
    if (r == ORBX_OK) r = realloc_dev(ctx->match_n, (size_t)S);
    if (r == ORBX_OK) r = realloc_dev(ctx->error_flags, 4);
    if (r == ORBX_OK && hipMemset(ctx->error_flags, 0, 4 * sizeof(int32_t)) != hipSuccess) r = ORBX_ERR_HIP;
    if (r == ORBX_OK && hipMemset(ctx->out_n, 0, S * sizeof(int32_t)) != hipSuccess) r = ORBX_ERR_HIP;
    if (r == ORBX_OK &&
        hipMemcpy(ctx->dgeom.umax, ctx->geom.umax.data(), ctx->geom.umax.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
        r = ORBX_ERR_HIP;
    // size the per-frame buffers for the largest frame up front
    if (r == ORBX_OK) r = set_geometry(ctx, max_w, max_h);
    if (r != ORBX_OK) {
        orbx_destroy(ctx);
        return r;
    }
    *out = ctx;
    return ORBX_OK;
}

void orbx_destroy(orbx_ctx* ctx)
{
    if (!ctx) return;
    ctx_enter(ctx);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
    for (hipStream_t x : ctx->xstreams)
        if (x) (void)hipStreamSynchronize(x);
    if (ctx->mstream) (void)hipStreamSynchronize(ctx->mstream);
    if (ctx->ustream) (void)hipStreamSynchronize(ctx->ustream);
    drop_single_graph(ctx);
    if (ctx->one_in) (void)hipHostFree(ctx->one_in);
    if (ctx->one_out) (void)hipHostFree(ctx->one_out);
    for (auto e : ctx->ev_now)
        if (e) (void)hipEventDestroy(e);
    for (auto e : ctx->ev_upload)
        if (e) (void)hipEventDestroy(e);
    if (ctx->ustream) (void)hipStreamDestroy(ctx->ustream);
    for (auto& t : ctx->timers) {
        for (auto e : t.start) hipEventDestroy(e);
        for (auto e : t.stop) hipEventDestroy(e);
    }
    free_buffers(ctx);
    lba_resident_free(ctx);
    if (ctx->lba_split) (void)hipFree(ctx->lba_split);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->ev_extracted) (void)hipEventDestroy(ctx->ev_extracted);
    for (auto e : ctx->ev_match)
        if (e) (void)hipEventDestroy(e);
    if (ctx->mstream) (void)hipStreamDestroy(ctx->mstream);
    if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
    for (hipStream_t x : ctx->xstreams)
        if (x) (void)hipStreamDestroy(x);
    for (int i = 0; i < orbx_ctx::kMaxWays; i++) {
        if (ctx->ev_part_fast[i]) (void)hipEventDestroy(ctx->ev_part_fast[i]);
        if (ctx->ev_part_done[i]) (void)hipEventDestroy(ctx->ev_part_done[i]);
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int orbx_get_levels(const orbx_ctx* ctx) { return ctx ? ctx->geom.nlevels : 0; }
float orbx_get_scale_factor(const orbx_ctx* ctx) { return ctx ? ctx->geom.scale_factor : 0.f; }

int orbx_get_features_per_level(const orbx_ctx* ctx, int32_t* out, int cap)
{
    if (!ctx || !out) return ORBX_ERR_ARG;
    const auto& v = ctx->geom.features_per_level;
    for (int i = 0; i < (int)v.size() && i < cap; i++) out[i] = v[i];
    return (int)v.size();
}

int orbx_get_scale_factors(const orbx_ctx* ctx, float* out, int cap)
{
    if (!ctx || !out) return ORBX_ERR_ARG;
    const auto& v = ctx->geom.scale;
    for (int i = 0; i < (int)v.size() && i < cap; i++) out[i] = v[i];
    return (int)v.size();
}

int orbx_dev_upload(orbx_ctx* ctx, int first, int count, const uint8_t* imgs, int w, int h, size_t stride)
{
    if (!ctx || !imgs || count <= 0 || first < 0 || first + count > ctx->slots || stride < (size_t)w)
        return ORBX_ERR_ARG;
    ctx_enter(ctx);
    int r = set_geometry(ctx, w, h);
    if (r != ORBX_OK) return r;
    ORBX_HIP_CHECK(hipMemcpy2DAsync(ctx->frames + (size_t)first * w * h, (size_t)w, imgs, stride, (size_t)w,
                                    (size_t)h * count, hipMemcpyHostToDevice, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return ORBX_OK;
}

int orbx_dev_extract(orbx_ctx* ctx, int first, int count)
{
    if (!ctx || count <= 0 || first < 0 || first + count > ctx->slots || ctx->geom_w <= 0) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ctx->last_first = first;
    ctx->last_count = count;
    return launch_extract(ctx, first, count);
}

int orbx_dev_match_prev(orbx_ctx* ctx, int first, int count, int seq_len, int window, float nnratio,
                        int check_ori)
{
    if (!ctx || count <= 0 || first < 0 || first + count > ctx->slots || seq_len <= 0 || window < 0)
        return ORBX_ERR_ARG;
    if (first % seq_len != 0 && first + count > ((first / seq_len) + 1) * seq_len) return ORBX_ERR_ARG;
    if (((first + count - 1) / seq_len + 1) * seq_len > ctx->slots) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    return launch_match_prev(ctx, first, count, seq_len, window, nnratio, check_ori);
}

int orbx_dev_extract_match(orbx_ctx* ctx, int first, int count, int seq_len, int mode, int window, int th_low,
                           float nnratio, int check_ori)
{
    if (!ctx || count <= 0 || first < 0 || first + count > ctx->slots || seq_len <= 0 || window < 0 ||
        (mode != 1 && mode != 2))
        return ORBX_ERR_ARG;
    if (first % seq_len != 0 && first + count > ((first / seq_len) + 1) * seq_len) return ORBX_ERR_ARG;
    if (((first + count - 1) / seq_len + 1) * seq_len > ctx->slots) return ORBX_ERR_ARG;
    if (ctx->geom_w <= 0) return ORBX_ERR_ARG;
    (void)hipSetDevice(ctx->device);   // launch_extract orders against a pending match
    ctx->last_first = first;
    ctx->last_count = count;
    MatchSpec m{mode, seq_len, window, th_low, check_ori, nnratio};
    return launch_extract(ctx, first, count, &m);
}

int orbx_dev_set_split(orbx_ctx* ctx, int enable)
{
    if (!ctx || enable < 0 || enable > orbx_ctx::kMaxWays) return ORBX_ERR_ARG;
    ctx->split = enable != 0;
    // 1 restores the documented default of three parts
    if (enable != 0) ctx->split_ways = enable >= 2 ? enable : orbx_ctx::kDefaultWays;
    return ORBX_OK;
}

int orbx_set_fp_contract(orbx_ctx* ctx, int enable)
{
    if (!ctx || enable < 0 || enable > 1) return ORBX_ERR_ARG;
    ctx_enter(ctx);   // extractions already queued keep the mode they were launched with
    ctx->fp_contract = enable;
    return ORBX_OK;
}

int orbx_get_fp_contract(const orbx_ctx* ctx) { return ctx ? ctx->fp_contract : ORBX_ERR_ARG; }

int orbx_set_nth_pivot(orbx_ctx* ctx, int mode)
{
    if (!ctx || (mode != ORBX_NTH_PIVOT_GCC49 && mode != ORBX_NTH_PIVOT_GCC48)) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ctx->nth_pivot = mode;
    return ORBX_OK;
}

int orbx_get_nth_pivot(const orbx_ctx* ctx) { return ctx ? ctx->nth_pivot : ORBX_ERR_ARG; }

int orbx_dev_set_async_match(orbx_ctx* ctx, int enable)
{
    if (!ctx) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ctx->async_match = enable != 0;
    return ORBX_OK;
}

int orbx_dev_match_bf_prev(orbx_ctx* ctx, int first, int count, int seq_len, int th_low, float nnratio)
{
    if (!ctx || count <= 0 || first < 0 || first + count > ctx->slots || seq_len <= 0) return ORBX_ERR_ARG;
    if (first % seq_len != 0 && first + count > ((first / seq_len) + 1) * seq_len) return ORBX_ERR_ARG;
    if (((first + count - 1) / seq_len + 1) * seq_len > ctx->slots) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    return launch_match_bf_prev(ctx, first, count, seq_len, th_low, nnratio);
}

int orbx_dev_sync(orbx_ctx* ctx)
{
    if (!ctx) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return check_errors(ctx);
}

int orbx_dev_read_features(orbx_ctx* ctx, int slot, orbx_keypoint* kps, uint8_t* desc, int cap, int* n_out)
{
    if (!ctx || slot < 0 || slot >= ctx->slots || !n_out) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    int32_t n = 0;
    ORBX_HIP_CHECK(hipMemcpy(&n, ctx->out_n + slot, sizeof(int32_t), hipMemcpyDeviceToHost));
    *n_out = n;
    if (n > cap) return ORBX_ERR_CAPACITY;
    const size_t nf = ctx->geom.nfeatures;
    if (n > 0 && kps)
        ORBX_HIP_CHECK(hipMemcpy(kps, ctx->out_kps + slot * nf, n * sizeof(orbx_keypoint), hipMemcpyDeviceToHost));
    if (n > 0 && desc)
        ORBX_HIP_CHECK(hipMemcpy(desc, ctx->out_desc + slot * nf * 32, (size_t)n * 32, hipMemcpyDeviceToHost));
    return ORBX_OK;
}

int orbx_dev_read_matches(orbx_ctx* ctx, int slot, int32_t* matches12, int cap, int* n_matches, int* n1)
{
    if (!ctx || slot < 0 || slot >= ctx->slots) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const int seq_prev_unknown = 0;
    (void)seq_prev_unknown;
    int32_t nm = 0;
    ORBX_HIP_CHECK(hipMemcpy(&nm, ctx->match_n + slot, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (n_matches) *n_matches = nm;
    const int nf = ctx->geom.nfeatures;
    if (n1) *n1 = nf;
    if (matches12) {
        if (cap < nf) return ORBX_ERR_CAPACITY;
        ORBX_HIP_CHECK(hipMemcpy(matches12, ctx->match12 + (size_t)slot * nf, nf * sizeof(int32_t), hipMemcpyDeviceToHost));
    }
    return ORBX_OK;
}

int orbx_dev_kernel_time_enable(orbx_ctx* ctx, int enable)
{
    if (!ctx) return ORBX_ERR_ARG;
    ctx->timing = enable != 0;
    for (auto& t : ctx->timers) t.used = 0;
    return ORBX_OK;
}

int orbx_dev_kernel_time_select(orbx_ctx* ctx, const char* name)
{
    if (!ctx) return ORBX_ERR_ARG;
    ctx->timing_only = name ? name : "";
    return ORBX_OK;
}

int orbx_dev_kernel_time(orbx_ctx* ctx, const char* name, double* avg_ms, double* total_ms)
{
    if (!ctx || !name) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    for (auto& t : ctx->timers) {
        if (t.name != name) continue;
        double tot = 0;
        for (int i = 0; i < t.used; i++) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, t.start[i], t.stop[i]) == hipSuccess) tot += ms;
        }
        const int n = t.used;
        if (avg_ms) *avg_ms = n ? tot / n : 0.0;
        if (total_ms) *total_ms = tot;
        t.used = 0;
        return n;
    }
    if (avg_ms) *avg_ms = 0;
    if (total_ms) *total_ms = 0;
    return 0;
}

int orbx_dev_read_level(orbx_ctx* ctx, int slot, int level, int blurred, uint8_t* out, int cap, int* pw, int* ph)
{
    if (!ctx || level < 0 || level >= ctx->geom.nlevels) return ORBX_ERR_ARG;
    const int f = slot;   // work buffers are per slot
    if (f < 0 || f >= ctx->slots) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const LevelGeom& L = ctx->geom.levels[level];
    *pw = L.pw;
    *ph = L.ph;
    if (cap < L.pw * L.ph) return ORBX_ERR_CAPACITY;
    const uint8_t* src = (blurred ? ctx->pyr_blur : ctx->pyr_raw) + (size_t)f * ctx->geom.frame_pyr_bytes + L.off;
    ORBX_HIP_CHECK(hipMemcpy2D(out, L.pw, src, L.stride, L.pw, L.ph, hipMemcpyDeviceToHost));
    return ORBX_OK;
}

int orbx_extract(orbx_ctx* ctx, const uint8_t* img, int w, int h, size_t stride, orbx_keypoint* kps,
                 uint8_t* desc, int cap, int* n_out)
{
    if (!ctx || !n_out) return ORBX_ERR_ARG;
    if (w == 0 || h == 0 || img == nullptr) {   // _image.empty(): return untouched
        *n_out = 0;
        return ORBX_OK;
    }
    if (w < 0 || h < 0 || stride < (size_t)w) return ORBX_ERR_ARG;
    if (ctx->launch_mode == 0 || ctx->timing) {
        // stream launches: pageable upload, the extraction chain, read-backs
        int r = orbx_dev_upload(ctx, 0, 1, img, w, h, stride);
        if (r != ORBX_OK) return r;
        if ((r = orbx_dev_extract(ctx, 0, 1)) != ORBX_OK) return r;
        if ((r = orbx_dev_sync(ctx)) != ORBX_OK) return r;
        return orbx_dev_read_features(ctx, 0, kps, desc, cap, n_out);
    }
    // One graph launch per call: the image goes through a page-locked staging
    // buffer, the outputs come back into another (count, error flags,
    // nfeatures keypoint records and descriptors), one synchronisation.
    ctx_enter(ctx);
    int r = set_geometry(ctx, w, h);
    if (r != ORBX_OK) return r;
    const size_t nf = ctx->geom.nfeatures, in_bytes = (size_t)w * h;
    const size_t o_kps = 64, o_desc = o_kps + nf * sizeof(orbx_keypoint), out_bytes = o_desc + nf * 32;
    if (in_bytes > ctx->one_in_bytes) {
        drop_single_graph(ctx);
        if (ctx->one_in) (void)hipHostFree(ctx->one_in);
        ctx->one_in = nullptr;
        ctx->one_in_bytes = 0;
        if (hipHostMalloc(&ctx->one_in, in_bytes, hipHostMallocDefault) != hipSuccess) return ORBX_ERR_NOMEM;
        ctx->one_in_bytes = in_bytes;
    }
    if (out_bytes > ctx->one_out_bytes) {
        drop_single_graph(ctx);
        if (ctx->one_out) (void)hipHostFree(ctx->one_out);
        ctx->one_out = nullptr;
        ctx->one_out_bytes = 0;
        if (hipHostMalloc(&ctx->one_out, out_bytes, hipHostMallocDefault) != hipSuccess) return ORBX_ERR_NOMEM;
        ctx->one_out_bytes = out_bytes;
    }
    // everything a captured launch sequence depends on (each setting in a
    // field of its own)
    const orbx_ctx::GraphKey key{ctx->geom_gen, ctx->fp_contract, ctx->nth_pivot, true};
    // the call's device work on the context stream: the frame into slot 0,
    // the single-frame extraction launches (k_describe also writes the
    // read-back block)
    uint8_t* out_host = static_cast<uint8_t*>(ctx->one_out);
    auto enqueue = [&]() -> int {
        int cr = ORBX_OK;
        if (hipMemcpyAsync(ctx->frames, ctx->one_in, in_bytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
            cr = ORBX_ERR_HIP;
        ctx->single_frame = true;
        ctx->single_out = out_host;   // k_describe writes the read-back block (no pack launch)
        if (cr == ORBX_OK) cr = launch_extract(ctx, 0, 1);
        ctx->single_frame = false;
        ctx->single_out = nullptr;
        return cr;
    };
    if (!ctx->one_exec || !(ctx->one_key == key)) {
        drop_single_graph(ctx);
        ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        ORBX_HIP_CHECK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
        const int cr = enqueue();
        hipGraph_t graph = nullptr;
        const hipError_t ec = hipStreamEndCapture(ctx->stream, &graph);
        if (cr != ORBX_OK || ec != hipSuccess || !graph) {
            if (graph) (void)hipGraphDestroy(graph);
            (void)hipGetLastError();
            return cr != ORBX_OK ? cr : ORBX_ERR_HIP;
        }
        ctx->one_graph = graph;
        if (hipGraphInstantiate(&ctx->one_exec, graph, nullptr, nullptr, 0) != hipSuccess) {
            drop_single_graph(ctx);
            return ORBX_ERR_HIP;
        }
        ctx->one_key = key;
    }
    uint8_t* in = static_cast<uint8_t*>(ctx->one_in);
    if (stride == (size_t)w) {
        std::memcpy(in, img, in_bytes);
    } else {
        for (int y = 0; y < h; y++) std::memcpy(in + (size_t)y * w, img + (size_t)y * stride, (size_t)w);
    }
    // host-side effects of launch_extract that a graph replay does not repeat
    if (!ctx->bow_ready.empty()) ctx->bow_ready[0] = 0;
    ctx->last_first = 0;
    ctx->last_count = 1;
    ORBX_HIP_CHECK(hipGraphLaunch(ctx->one_exec, ctx->stream));
    ORBX_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const uint8_t* out = static_cast<const uint8_t*>(ctx->one_out);
    int32_t n = 0, flags = 0;
    std::memcpy(&n, out, 4);
    std::memcpy(&flags, out + 4, 4);
    if (flags) {
        (void)hipMemset(ctx->error_flags, 0, sizeof(int32_t));
        return ORBX_ERR_CAPACITY;
    }
    *n_out = n;
    if (n > cap) return ORBX_ERR_CAPACITY;
    if (n > 0 && kps) std::memcpy(kps, out + o_kps, (size_t)n * sizeof(orbx_keypoint));
    if (n > 0 && desc) std::memcpy(desc, out + o_desc, (size_t)n * 32);
    return ORBX_OK;
}

int orbx_dev_set_image_bounds(orbx_ctx* ctx, const float* bounds)
{
    if (!ctx) return ORBX_ERR_ARG;
    if (bounds && !(bounds[1] > bounds[0] && bounds[3] > bounds[2])) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ctx->has_bounds = bounds != nullptr;
    for (int i = 0; i < 4; i++) ctx->bounds[i] = bounds ? bounds[i] : 0.f;
    return ORBX_OK;
}

int orbx_set_launch_mode(orbx_ctx* ctx, int mode)
{
    if (!ctx || mode < 0 || mode > 1) return ORBX_ERR_ARG;
    ctx_enter(ctx);
    ctx->launch_mode = mode;
    return ORBX_OK;
}

int orbx_get_launch_mode(const orbx_ctx* ctx) { return ctx ? ctx->launch_mode : ORBX_ERR_ARG; }

int orbx_host_alloc(size_t bytes, void** out)
{
    if (!out || bytes == 0) return ORBX_ERR_ARG;
    *out = nullptr;
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return ORBX_ERR_NOMEM;
    }
    return ORBX_OK;
}

void orbx_host_free(void* p)
{
    if (p) (void)hipHostFree(p);
}

int orbx_dev_upload_async(orbx_ctx* ctx, int first, int count, const uint8_t* imgs, int w, int h, size_t stride)
{
    if (!ctx || !imgs || count <= 0 || first < 0 || first + count > ctx->slots || stride < (size_t)w) return ORBX_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    if (w != ctx->geom_w || h != ctx->geom_h) return orbx_dev_upload(ctx, first, count, imgs, w, h, stride);
    if (!ctx->ustream && hipStreamCreateWithFlags(&ctx->ustream, hipStreamNonBlocking) != hipSuccess) {
        ctx->ustream = nullptr;
        return ORBX_ERR_HIP;
    }
    // the slots' previous frames are read by extractions queued before this
    // call: the copy starts after them
    int r = order_after_extraction(ctx, ctx->ustream);
    if (r != ORBX_OK) return r;
    uint8_t* dst = ctx->frames + (size_t)first * w * h;
    if (stride == (size_t)w)   // one linear copy (a 2-D copy of w-byte rows is much slower)
        ORBX_HIP_CHECK(hipMemcpyAsync(dst, imgs, (size_t)w * h * count, hipMemcpyHostToDevice, ctx->ustream));
    else
        ORBX_HIP_CHECK(hipMemcpy2DAsync(dst, (size_t)w, imgs, stride, (size_t)w, (size_t)h * count, hipMemcpyHostToDevice,
                                        ctx->ustream));
    if (ctx->n_uploads == orbx_ctx::kMaxUploads) {   // table full: the context stream takes the oldest
        ORBX_HIP_CHECK(hipStreamWaitEvent(ctx->stream, ctx->uploads[0].done, 0));
        for (int i = 1; i < ctx->n_uploads; i++) ctx->uploads[i - 1] = ctx->uploads[i];
        ctx->n_uploads--;
    }
    hipEvent_t ev = ctx->ev_upload[ctx->next_upload];
    ctx->next_upload = (ctx->next_upload + 1) % orbx_ctx::kMaxUploads;
    ORBX_HIP_CHECK(hipEventRecord(ev, ctx->ustream));
    ctx->uploads[ctx->n_uploads++] = orbx_ctx::PendingMatch{first, first + count, ev};
    return ORBX_OK;
}

int orbx_dev_download_async(orbx_ctx* ctx, int first, int count, orbx_keypoint* kps, uint8_t* desc, int32_t* n_kps,
                            int32_t* matches12, int32_t* n_matches)
{
    if (!ctx || count <= 0 || first < 0 || first + count > ctx->slots) return ORBX_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    // after the extraction of the slots (every stream it may run on) and, mstream
    // being in order, after their queued match
    int r = ensure_aux_streams(ctx);
    if (r != ORBX_OK) return r;
    r = order_after_extraction(ctx, ctx->mstream);
    if (r != ORBX_OK) return r;
    const size_t nf = ctx->geom.nfeatures, s0 = first, n = count;
    const hipStream_t st = ctx->mstream;
    if (kps)
        ORBX_HIP_CHECK(hipMemcpyAsync(kps, ctx->out_kps + s0 * nf, n * nf * sizeof(orbx_keypoint), hipMemcpyDeviceToHost, st));
    if (desc) ORBX_HIP_CHECK(hipMemcpyAsync(desc, ctx->out_desc + s0 * nf * 32, n * nf * 32, hipMemcpyDeviceToHost, st));
    if (n_kps) ORBX_HIP_CHECK(hipMemcpyAsync(n_kps, ctx->out_n + s0, n * 4, hipMemcpyDeviceToHost, st));
    if (matches12)
        ORBX_HIP_CHECK(hipMemcpyAsync(matches12, ctx->match12 + s0 * nf, n * nf * 4, hipMemcpyDeviceToHost, st));
    if (n_matches) ORBX_HIP_CHECK(hipMemcpyAsync(n_matches, ctx->match_n + s0, n * 4, hipMemcpyDeviceToHost, st));
    // a later extraction of these slots waits for the copies
    ORBX_HIP_CHECK(push_pending(ctx, first, first + count));
    return ORBX_OK;
}

int orbx_extract_batch(orbx_ctx* ctx, int B, const uint8_t* const* imgs, int w, int h, size_t stride,
                       orbx_keypoint* kps, uint8_t* desc, int cap, int32_t* n_out)
{
    if (!ctx || !imgs || !n_out || B <= 0 || B > ctx->slots) return ORBX_ERR_ARG;
    int r;
    for (int b = 0; b < B; b++)
        if ((r = orbx_dev_upload(ctx, b, 1, imgs[b], w, h, stride)) != ORBX_OK) return r;
    if ((r = orbx_dev_extract(ctx, 0, B)) != ORBX_OK) return r;
    if ((r = orbx_dev_sync(ctx)) != ORBX_OK) return r;
    for (int b = 0; b < B; b++) {
        int n = 0;
        r = orbx_dev_read_features(ctx, b, kps ? kps + (size_t)b * cap : nullptr,
                                   desc ? desc + (size_t)b * cap * 32 : nullptr, cap, &n);
        n_out[b] = n;
        if (r != ORBX_OK) return r;
    }
    return ORBX_OK;
}

int orbx_describe_levels(int nfeatures, float scale_factor, int nlevels, int fast_th, int w, int h, int32_t* out,
                         int cap)
{
    if (nfeatures <= 0 || nlevels <= 0 || nlevels > kMaxLevels || !(scale_factor > 1.0f) || !out) return ORBX_ERR_ARG;
    Geometry g;
    init_extractor_tables(g, nfeatures, scale_factor, nlevels, fast_th);
    const int r = compute_geometry(g, w, h);
    if (r != ORBX_OK) return r;
    if (cap < 8 * nlevels) return ORBX_ERR_CAPACITY;
    for (int l = 0; l < nlevels; l++) {
        const LevelGeom& L = g.levels[l];
        int valid = 0;
        for (int c = 0; c < L.n_cells; c++) valid += g.cells[L.cell_base + c].valid;
        const int32_t v[8] = {L.w, L.h, L.n_desired, L.level_cols, L.level_rows, L.nfeatures_cell, L.n_cells, valid};
        for (int k = 0; k < 8; k++) out[8 * l + k] = v[k];
    }
    return nlevels;
}

int orbx_descriptor_distance(const uint8_t* a, const uint8_t* b)
{
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

}  // extern "C"
