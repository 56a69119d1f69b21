// Host-side tables of the extractor: everything that depends only on the
// configuration and the image size, computed once per size the way the
// reference (and OpenCV) compute them on every call.
//
//   * ORBextractor constructor: scale factors, per-level feature quota, umax
//     (src/ORBextractor.cc:457-511).  Note `double scaleFactor`
//     (include/ORBextractor.h:66): the float argument is widened, so
//     1.0f/scaleFactor and (float)(1.0/scaleFactor) are double divisions.
//   * ComputePyramid level sizes (src/ORBextractor.cc:786).
//   * ComputeKeyPoints cell grid (src/ORBextractor.cc:527-640).
//   * cv::resize INTER_LINEAR coefficient tables (OpenCV 2.4 imgwarp.cpp):
//     xofs/ialpha, yofs/ibeta with 11-bit fixed-point weights.
// Built with -ffp-contract=off so every float expression rounds as written.
#include <algorithm>
#include <cmath>

#include "orbx_internal.h"

namespace orbx {

namespace {
inline int cv_round(double v) { return (int)std::nearbyint(v); }
inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
inline int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}
inline int16_t sat16(int v) { return (int16_t)std::min(32767, std::max(-32768, v)); }

int vec_count(int width, bool strict4)
{
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    if (strict4) { for (; x < width - 4; x += 4) {} }
    else { for (; x <= width - 4; x += 4) {} }
    return x;
}
}  // namespace

void init_extractor_tables(Geometry& g, int nfeatures, float scale_factor, int nlevels, int fast_th)
{
    g.nfeatures = nfeatures;
    g.nlevels = nlevels;
    g.fast_th = fast_th;
    g.scale_factor = scale_factor;
    const double sf = scale_factor;                       // double member
    g.scale.assign(nlevels, 1.0f);
    for (int i = 1; i < nlevels; i++) g.scale[i] = (float)(g.scale[i - 1] * sf);
    const float inv = (float)(1.0f / sf);
    g.inv_scale.assign(nlevels, 1.0f);
    for (int i = 1; i < nlevels; i++) g.inv_scale[i] = g.inv_scale[i - 1] * inv;

    g.features_per_level.assign(nlevels, 0);
    const float factor = (float)(1.0 / sf);
    float desired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        g.features_per_level[l] = cv_round(desired);
        sum += g.features_per_level[l];
        desired *= factor;
    }
    g.features_per_level[nlevels - 1] = std::max(nfeatures - sum, 0);

    g.umax.assign(kHalfPatch + 1, 0);
    const int vmax = cv_floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
    const double hp2 = kHalfPatch * kHalfPatch;
    int v, v0;
    for (v = 0; v <= vmax; ++v) g.umax[v] = cv_round(std::sqrt(hp2 - v * v));
    for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (g.umax[v0] == g.umax[v0 + 1]) ++v0;
        g.umax[v] = v0;
        ++v0;
    }
    g.w = g.h = 0;
}

// OpenCV 2.4 cv::resize coefficient tables for one level (src -> dst).
static int resize_tables(Geometry& g, int sw, int sh, int dw, int dh)
{
    const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
    const double sx_scale = 1. / inv_sx, sy_scale = 1. / inv_sy;
    const int isx = (int)std::lrint(sx_scale), isy = (int)std::lrint(sy_scale);
    const bool area_fast = std::fabs(sx_scale - isx) < 2.220446049250313e-16 &&
                           std::fabs(sy_scale - isy) < 2.220446049250313e-16;
    // At exactly 2x cv::resize takes INTER_AREA's fast path, (S00 + S01 +
    // S10 + S11 + 2) >> 2 (ResizeAreaFastVec<uchar>).  The INTER_LINEAR
    // tables built below are then fx = fy = 1/2 (weights 1024 / 1024) and
    // both of its roundings, ((S0 >> 4) * 1024 >> 16) + ... + 2 >> 2 and
    // (S0 * 1024 + S1 * 1024 + 2^21) >> 22, reduce to that same value, so
    // the linear kernels compute the area result bit for bit (OpenCV's own
    // comment at the switch: "INTER_AREA (fast) also is equal to
    // INTER_LINEAR" there).
    (void)area_fast;
    int xmax = dw;
    std::vector<int> xofs(dw);
    std::vector<int16_t> a0(dw), a1(dw);
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * sx_scale - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        a0[dx] = sat16(cv_round((1.f - fx) * 2048));
        a1[dx] = sat16(cv_round(fx * 2048));
    }
    for (int dx = 0; dx < dw; dx++) {
        ResizeCol c;
        if (dx < xmax) {
            c.sx0 = (int16_t)xofs[dx];
            c.sx1 = (int16_t)(xofs[dx] + 1);
            c.a0 = a0[dx];
            c.a1 = a1[dx];
        } else {   // HResizeLinear tail: S[sx] * ONE
            c.sx0 = c.sx1 = (int16_t)xofs[dx];
            c.a0 = 2048;
            c.a1 = 0;
        }
        g.res_cols.push_back(c);
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * sy_scale - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        auto clip = [&](int y) { return y >= 0 ? (y < sh ? y : sh - 1) : 0; };
        ResizeRow r;
        r.sy0 = (int16_t)clip(sy);
        r.sy1 = (int16_t)clip(sy + 1);
        r.b0 = sat16(cv_round((1.f - fy) * 2048));
        r.b1 = sat16(cv_round(fy * 2048));
        g.res_rows.push_back(r);
    }
    return ORBX_OK;
}

int compute_geometry(Geometry& g, int w, int h)
{
    if (w <= 0 || h <= 0 || w > 4095 || h > 4095) return ORBX_ERR_ARG;
    g.w = w;
    g.h = h;
    g.levels.assign(g.nlevels, LevelGeom{});
    g.cells.clear();
    g.res_cols.clear();
    g.res_rows.clear();
    long long off = 0;
    int list_off = 0, level_off = 0;
    g.max_tile_bytes = g.max_list_cap = g.max_level_cap = g.max_cells_per_level = 0;
    for (int l = 0; l < g.nlevels; l++) {
        LevelGeom& L = g.levels[l];
        L.w = cv_round((float)w * g.inv_scale[l]);
        L.h = cv_round((float)h * g.inv_scale[l]);
        if (L.w < 1 || L.h < 1) return ORBX_ERR_UNSUPPORTED;
        L.pw = L.w + 2 * kEdge;
        L.ph = L.h + 2 * kEdge;
        L.stride = (L.pw + 63) & ~63;
        L.off = off;
        off += (long long)L.stride * L.ph;
        off = (off + 255) & ~255LL;
        L.nvec_resize = vec_count(L.w, true);
        L.nvec_blur = vec_count(L.w, false);
        L.scale = g.scale[l];
        L.patch_size = (float)(int)(kPatch * g.scale[l]);
        L.n_desired = g.features_per_level[l];
        while (g.res_cols.size() % 4) g.res_cols.push_back(ResizeCol{0, 0, 0, 0});   // 32-byte aligned runs
        L.res_col_off = (int)g.res_cols.size();
        L.res_row_off = (int)g.res_rows.size();
        L.res_span = 0;
        if (l > 0) {
            const int r = resize_tables(g, g.levels[l - 1].w, g.levels[l - 1].h, L.w, L.h);
            if (r != ORBX_OK) return r;
            // source rows feeding each strip of kResRows padded output rows
            for (int py0 = 0; py0 < L.ph; py0 += kResRows) {
                int lo = 1 << 30, hi = -1;
                for (int py = py0; py < std::min(py0 + kResRows, L.ph); py++) {
                    const ResizeRow& rr = g.res_rows[L.res_row_off + reflect101(py - kEdge, L.h)];
                    lo = std::min(lo, (int)std::min(rr.sy0, rr.sy1));
                    hi = std::max(hi, (int)std::max(rr.sy0, rr.sy1));
                }
                L.res_span = std::max(L.res_span, hi - lo + 1);
            }
        }
    }
    g.frame_pyr_bytes = off;
    // per (level >= 1, strip of kResRows padded rows): the first source row
    // the strip reads, appended to the row table so the resize kernel can
    // start its staging loads without a dependent table read
    for (int l = 1; l < g.nlevels; l++) {
        LevelGeom& L = g.levels[l];
        L.res_strip_off = (int)g.res_rows.size();
        for (int py0 = 0; py0 < L.ph; py0 += kResRows) {
            int lo = 1 << 30;
            for (int py = py0; py < std::min(py0 + kResRows, L.ph); py++) {
                const ResizeRow& rr = g.res_rows[L.res_row_off + reflect101(py - kEdge, L.h)];
                lo = std::min(lo, (int)std::min(rr.sy0, rr.sy1));
            }
            g.res_rows.push_back(ResizeRow{(int16_t)lo, 0, 0, 0});
        }
    }

    const float imageRatio = (float)g.levels[0].w / g.levels[0].h;
    for (int l = 0; l < g.nlevels; l++) {
        LevelGeom& L = g.levels[l];
        const int nDesired = L.n_desired;
        const int levelCols = (int)std::sqrt((float)nDesired / (5 * imageRatio));
        const int levelRows = (int)(imageRatio * levelCols);
        if (levelCols <= 0 || levelRows <= 0) return ORBX_ERR_UNSUPPORTED;
        const int minBorderX = kEdge, minBorderY = kEdge;
        const int maxBorderX = L.w - kEdge, maxBorderY = L.h - kEdge;
        const int W = maxBorderX - minBorderX, H = maxBorderY - minBorderY;
        const int cellW = (int)std::ceil((float)W / levelCols);
        const int cellH = (int)std::ceil((float)H / levelRows);
        const int nCells = levelRows * levelCols;
        L.level_cols = levelCols;
        L.level_rows = levelRows;
        L.n_cells = nCells;
        L.cell_base = (int)g.cells.size();
        L.nfeatures_cell = (int)std::ceil((float)nDesired / nCells);
        std::vector<int> iniXCol(levelCols, 0);
        std::vector<CellGeom> row_cells;
        float hY = cellH + 6;
        for (int i = 0; i < levelRows; i++) {
            const float iniY = minBorderY + i * cellH - 3;
            bool row_valid = true;
            if (i == levelRows - 1) {
                hY = maxBorderY + 3 - iniY;
                if (hY <= 0) row_valid = false;
            }
            float hX = cellW + 6;
            for (int j = 0; j < levelCols; j++) {
                CellGeom c{};
                c.level = l;
                c.i = i;
                c.j = j;
                float iniX = 0;
                if (row_valid) {
                    if (i == 0) {
                        iniX = minBorderX + j * cellW - 3;
                        iniXCol[j] = (int)iniX;
                    } else {
                        iniX = iniXCol[j];
                    }
                }
                c.valid = row_valid ? 1 : 0;
                if (row_valid && j == levelCols - 1) {
                    hX = maxBorderX + 3 - iniX;
                    if (hX <= 0) c.valid = 0;
                }
                c.ini_x = (int)iniX;
                c.ini_y = (int)iniY;
                c.hx = c.valid ? (int)(iniX + hX) - (int)iniX : 0;
                c.hy = c.valid ? (int)(iniY + hY) - (int)iniY : 0;
                if (c.valid) {
                    if (c.ini_x < 0 || c.ini_y < 0 || c.ini_x + c.hx > L.w || c.ini_y + c.hy > L.h)
                        return ORBX_ERR_UNSUPPORTED;
                }
                const int iw = std::max(c.hx - 6, 0), ih = std::max(c.hy - 6, 0);
                c.list_cap = ((iw + 1) / 2) * ((ih + 1) / 2);
                c.list_off = list_off;
                list_off += c.list_cap;
                // FAST tile: 16-byte aligned rows (up to 15 bytes of lead-in)
                g.max_tile_bytes = std::max(g.max_tile_bytes, c.hy * ((c.hx + 30) & ~15));
                g.max_list_cap = std::max(g.max_list_cap, c.list_cap);
                g.cells.push_back(c);
            }
        }
        // iniXCol for rows > 0 is read from row 0 (same as the reference);
        // cells of later rows were pushed with iniXCol values already set
        // because row 0 is always processed first.
        // Bound on the retained cell lists of a level, Σ_c min(nTotal_c,
        // nToRetain_c) (src/ORBextractor.cc:622-670): with q the quota of the
        // cells still distributing and D the surplus to distribute, a round
        // maps (Σ retained + D) to at most itself + m (1 + nfeaturesCell - q)
        // over its m open cells (q' <= nfeaturesCell + D / m + 1).  Only the
        // first round has q = nfeaturesCell; later ones have q >= it + 1.
        // Start: nCells * nfeaturesCell <= nDesired + nCells - 1.  So the
        // total stays <= nDesired + 2 nCells - 1 (slack: + 64).
        L.level_cap = nDesired + 2 * nCells + 64;
        L.level_off = level_off;
        level_off += L.level_cap;   // the cell pass writes up to level_cap entries
        g.max_level_cap = std::max(g.max_level_cap, L.level_cap);
        g.max_cells_per_level = std::max(g.max_cells_per_level, nCells);
    }
    g.list_entries = list_off;
    g.level_entries = level_off;
    return ORBX_OK;
}

// k_pyr_cascade's bands: band j owns ROI rows [h j / B, h (j + 1) / B) of
// every level (and the border rows that reflect to them) and computes those
// rows plus every ROI row the next level's computed rows read (their
// row-table sources), so each level's rows are derived from the previous
// level's in LDS and the bands of consecutive levels stay aligned.  The
// smallest band count whose two ping-pong buffers (rows x stride of the even
// and of the odd levels) fit lds_target.
void plan_cascade(Geometry& g, int lds_target)
{
    g.cascade.clear();
    g.cascade_bands = g.cascade_buf_x = g.cascade_lds = 0;
    g.cascade_tab_cols = g.cascade_tab_rows = 0;
    const int nl = g.nlevels;
    if (g.w % 16 != 0 || nl < 1) return;
    std::vector<int4> tab;
    for (int B = 1; B <= 512; B++) {
        tab.assign((size_t)B * nl, make_int4(0, 0, 0, -1));
        int bx = 0, by = 0;
        for (int j = 0; j < B; j++) {
            int need_lo = 1 << 30, need_hi = -1;
            for (int l = nl - 1; l >= 0; l--) {
                const LevelGeom& L = g.levels[l];
                const int o0 = (int)((long long)L.h * j / B), o1 = (int)((long long)L.h * (j + 1) / B);
                int lo = std::min(need_lo, o0), hi = std::max(need_hi, o1 - 1);
                if (o0 >= o1) lo = need_lo, hi = need_hi;
                if (lo > hi) lo = 0, hi = -1;
                tab[(size_t)j * nl + l] = make_int4(o0, o1, lo, hi);
                const int bytes = (hi - lo + 1) * L.stride;
                (l % 2 == 0 ? bx : by) = std::max(l % 2 == 0 ? bx : by, bytes);
                need_lo = 1 << 30;
                need_hi = -1;
                if (l > 0)
                    for (int r = lo; r <= hi; r++) {
                        const ResizeRow& rr = g.res_rows[L.res_row_off + r];
                        need_lo = std::min(need_lo, (int)std::min(rr.sy0, rr.sy1));
                        need_hi = std::max(need_hi, (int)std::max(rr.sy0, rr.sy1));
                    }
            }
        }
        bx = (bx + 15) & ~15;
        if (bx + by <= lds_target) {
            // the halo rows computed twice: a plan that would recompute more
            // than half again of the resized levels' pixels is not taken
            long long comp = 0, roi = 0;
            for (int l = 1; l < nl; l++) {
                roi += (long long)g.levels[l].w * g.levels[l].h;
                for (int j = 0; j < B; j++) comp += (long long)g.levels[l].w * (tab[(size_t)j * nl + l].w - tab[(size_t)j * nl + l].z + 1);
            }
            if (comp * 2 > roi * 3) return;
            g.cascade = tab;
            g.cascade_bands = B;
            g.cascade_buf_x = bx;
            g.cascade_lds = bx + by;
            for (int l = 1; l < nl; l++) g.cascade_tab_cols += g.levels[l].w;
            for (int j = 0; j < B; j++) {
                int rows = 0;
                for (int l = 1; l < nl; l++) rows += std::max(0, tab[(size_t)j * nl + l].w - tab[(size_t)j * nl + l].z + 1);
                g.cascade_tab_rows = std::max(g.cascade_tab_rows, rows);
            }
            return;
        }
    }
}

}  // namespace orbx
