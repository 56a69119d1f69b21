// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// CPU restatement of ORB_SLAM::ORBextractor (src/ORBextractor.cc) together
// with the OpenCV 2.4 routines it calls (resize INTER_LINEAR, FAST-9/16 with
// non-max suppression, KeyPointsFilter::retainBest, GaussianBlur 7x7,
// copyMakeBorder REFLECT_101).  OpenCV semantics follow the 2.4 generic C++
// code with the x86-64 SSE2 kernels that change rounding (the VResize and
// SymmColumn vector paths); see DESIGN.md section 3 for the pinned choices.
// Compile with -ffp-contract=off: every float expression is evaluated as
// written.
#include "ref_common.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

namespace orbref {

namespace {

const int kPatchSize = 31;       // PATCH_SIZE      (src/ORBextractor.cc:75)
const int kHalfPatch = 15;       // HALF_PATCH_SIZE (:76)
const int kEdge = 16;            // EDGE_THRESHOLD  (:77)


// cvRound/cvFloor/cvCeil of OpenCV 2.4 on x86-64 (cvtsd2si under the default
// round-to-nearest-even MXCSR mode).
inline int cvRound(double v) { return (int)std::nearbyint(v); }
inline int cvFloor(double v) { int i = (int)v; return i - (i > v); }
inline uint8_t satU8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
inline int16_t satS16(int v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }

// cv::borderInterpolate for BORDER_REFLECT_101.
int reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// Column count handled by an SSE2 loop pair "for(;x<=w-16;x+=16)" followed
// by a 4-wide loop whose bound is `x < w-4` (VResizeLinearVec_32s8u) or
// `x <= w-4` (SymmColumnVec_32s8u).
int vecCount(int width, bool strict4)
{
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    if (strict4) { for (; x < width - 4; x += 4) {} }
    else { for (; x <= width - 4; x += 4) {} }
    return x;
}

}  // namespace

// ---------------------------------------------------------------------------
// cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR) for CV_8UC1 (OpenCV 2.4
// imgwarp.cpp: coefficient tables in cv::resize, HResizeLinear<uchar,int,
// short,2048>, VResizeLinear<uchar,int,short,FixedPtCast<int,uchar,22>,
// VResizeLinearVec_32s8u>).  Called at src/ORBextractor.cc:800.
// ---------------------------------------------------------------------------
void cv24_resize_linear_u8(const uint8_t* src, int sstep, int sw, int sh,
                           uint8_t* dst, int dstep, int dw, int dh)
{
    const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    const int iscale_x = (int)std::lrint(scale_x), iscale_y = (int)std::lrint(scale_y);
    const bool area_fast = std::fabs(scale_x - iscale_x) < 2.220446049250313e-16 &&
                           std::fabs(scale_y - iscale_y) < 2.220446049250313e-16;
    if (area_fast && iscale_x == 2 && iscale_y == 2) {
        // cv::resize reroutes INTER_LINEAR at exactly 2x to INTER_AREA's fast
        // path: resizeAreaFast_ with ResizeAreaFastVec<uchar> in fast mode
        // (scale 2, cn 1): D = (S00 + S01 + S10 + S11 + 2) >> 2 over the
        // dwidth1 = sw / 2 columns and rows whose two source rows exist --
        // all of them when sw = 2 dw and sh = 2 dh.
        for (int dy = 0; dy < dh; dy++) {
            const uint8_t* S = src + (size_t)(2 * dy) * sstep;
            const uint8_t* T = S + sstep;
            uint8_t* D = dst + (size_t)dy * dstep;
            for (int dx = 0; dx < dw; dx++)
                D[dx] = (uint8_t)((S[2 * dx] + S[2 * dx + 1] + T[2 * dx] + T[2 * dx + 1] + 2) >> 2);
        }
        return;
    }

    const int kScale = 2048;  // INTER_RESIZE_COEF_SCALE
    std::vector<int> xofs(dw);
    std::vector<int16_t> ialpha(2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cvFloor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        const float c0 = 1.f - fx, c1 = fx;
        ialpha[2 * dx] = satS16(cvRound(c0 * kScale));
        ialpha[2 * dx + 1] = satS16(cvRound(c1 * kScale));
    }
    std::vector<int> yofs(dh);
    std::vector<int16_t> ibeta(2 * dh);
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cvFloor(fy);
        fy -= sy;
        yofs[dy] = sy;
        const float c0 = 1.f - fy, c1 = fy;
        ibeta[2 * dy] = satS16(cvRound(c0 * kScale));
        ibeta[2 * dy + 1] = satS16(cvRound(c1 * kScale));
    }

    std::vector<int> row0(dw), row1(dw);
    auto hresize = [&](const uint8_t* S, int* D) {
        for (int dx = 0; dx < xmax; dx++) {
            const int sx = xofs[dx];
            D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
        }
        for (int dx = xmax; dx < dw; dx++) D[dx] = S[xofs[dx]] * kScale;
    };
    const int nvec = vecCount(dw, true);
    for (int dy = 0; dy < dh; dy++) {
        const int sy0 = yofs[dy];
        auto clip = [&](int y) { return y >= 0 ? (y < sh ? y : sh - 1) : 0; };
        hresize(src + (size_t)clip(sy0) * sstep, row0.data());
        hresize(src + (size_t)clip(sy0 + 1) * sstep, row1.data());
        const int b0 = ibeta[2 * dy], b1 = ibeta[2 * dy + 1];
        uint8_t* D = dst + (size_t)dy * dstep;
        for (int x = 0; x < dw; x++) {
            if (x < nvec) {
                // SSE2: (S>>4) packed to int16, _mm_mulhi_epi16 with beta,
                // saturating add, +2, arithmetic >>2, packus to u8.
                const int s0 = satS16(row0[x] >> 4), s1 = satS16(row1[x] >> 4);
                const int m0 = (s0 * b0) >> 16, m1 = (s1 * b1) >> 16;
                int v = satS16(m0 + m1);
                v = satS16(v + 2) >> 2;
                D[x] = satU8(v);
            } else {
                D[x] = satU8((row0[x] * b0 + row1[x] * b1 + (1 << 21)) >> 22);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// FAST-9/16 with non-max suppression (OpenCV 2.4 features2d/src/fast.cpp,
// FAST_t<16> scalar form and cornerScore<16>).  Called per cell at
// src/ORBextractor.cc:607 and :613.
// ---------------------------------------------------------------------------
int cv24_corner_score16(const uint8_t* ptr, const int pixel[25], int threshold)
{
    const int K = 8, N = 25;
    const int v = ptr[0];
    int d[N];
    for (int k = 0; k < N; k++) d[k] = v - ptr[pixel[k]];
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(d[k + 1], d[k + 2]);
        a = std::min(a, d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, d[k + 4]);
        a = std::min(a, d[k + 5]);
        a = std::min(a, d[k + 6]);
        a = std::min(a, d[k + 7]);
        a = std::min(a, d[k + 8]);
        a0 = std::max(a0, std::min(a, d[k]));
        a0 = std::max(a0, std::min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max(d[k + 1], d[k + 2]);
        b = std::max(b, d[k + 3]);
        b = std::max(b, d[k + 4]);
        b = std::max(b, d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, d[k + 6]);
        b = std::max(b, d[k + 7]);
        b = std::max(b, d[k + 8]);
        b0 = std::min(b0, std::max(b, d[k]));
        b0 = std::min(b0, std::max(b, d[k + 9]));
    }
    (void)K;
    return -b0 - 1;
}

void cv24_fast16(const uint8_t* img, int step, int rows, int cols, int threshold,
                 bool nonmax, std::vector<KeyPoint>& kps)
{
    static const int kOffsets[16][2] = {
        {0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
        {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    const int K = 8, N = 25;
    int pixel[25];
    for (int k = 0; k < 16; k++) pixel[k] = kOffsets[k][0] + kOffsets[k][1] * step;
    for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
    kps.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t tab[512];
    for (int i = -255; i <= 255; i++)
        tab[i + 255] = (uint8_t)(i < -threshold ? 1 : (i > threshold ? 2 : 0));

    if (cols < 1) return;
    std::vector<uint8_t> sbuf(3 * (size_t)cols, 0);
    std::vector<int> cbuf(3 * ((size_t)cols + 1), 0);
    uint8_t* buf[3] = {sbuf.data(), sbuf.data() + cols, sbuf.data() + 2 * cols};
    int* cpbuf[3] = {cbuf.data() + 1, cbuf.data() + 1 + (cols + 1), cbuf.data() + 1 + 2 * (cols + 1)};

    for (int i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = img + (size_t)i * step + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        std::memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; j++, ptr++) {
                const int v = ptr[0];
                const uint8_t* t = &tab[0] - v + 255;
                int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
                d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
                d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
                d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
                d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
                d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
                if (d & 1) {
                    const int vt = v - threshold;
                    int count = 0;
                    for (int k = 0; k < N; k++) {
                        const int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                if (nonmax) curr[j] = (uint8_t)cv24_corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else {
                            count = 0;
                        }
                    }
                }
                if (d & 2) {
                    const int vt = v + threshold;
                    int count = 0;
                    for (int k = 0; k < N; k++) {
                        const int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                if (nonmax) curr[j] = (uint8_t)cv24_corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else {
                            count = 0;
                        }
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            const int j = cornerpos[k];
            const int score = prev[j];
            if (!nonmax ||
                (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                 score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                 score > curr[j] && score > curr[j + 1])) {
                KeyPoint kp;
                kp.x = (float)j;
                kp.y = (float)(i - 1);
                kp.size = 7.f;
                kp.angle = -1.f;
                kp.response = (float)score;
                kp.octave = 0;
                kp.class_id = -1;
                kps.push_back(kp);
            }
        }
    }
}

// std::nth_element as libstdc++ implements it (bits/stl_algo.h
// __introselect, __heap_select, __insertion_sort, __unguarded_partition),
// restated so the pivot step can follow either era of the library:
//   NTH_PIVOT_GCC49: __move_median_to_first(first, first + 1, mid,
//       last - 1) -- the median of those three swapped into *first (GCC >= 4.9,
//       PR libstdc++/58437; the GCC 11.4 of this image);
//   NTH_PIVOT_GCC48: __move_median_first(first, mid, last - 1) -- the median
//       of (first, mid, last - 1) moved to *first, *first left in place when
//       it is the median (GCC 4.6 .. 4.8, the compilers of the reference's
//       era: Ubuntu 12.04 / 14.04, README.md:46) -- the default.
// Everything else (depth limit 2 floor(log2 n), the Hoare partition from
// first + 1, heap select, insertion sort below 4 elements) is common to both.
// With NTH_PIVOT_GCC49 it is checked against this image's std::nth_element
// (orbx_ref_nth_element_check, tests/test_sort_era.py).
// ---------------------------------------------------------------------------
static int g_nth_pivot = NTH_PIVOT_GCC48;   // the default era, as the product's (include/orbx.h)
void set_nth_pivot(int mode) { g_nth_pivot = mode; }
int get_nth_pivot() { return g_nth_pivot; }

namespace {
template <class T, class Less>
void adjust_heap(T* first, long hole, long len, T value, Less less)
{
    const long top = hole;
    long child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (less(first[child], first[child - 1])) child--;
        first[hole] = first[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        first[hole] = first[child - 1];
        hole = child - 1;
    }
    long parent = (hole - 1) / 2;   // __push_heap
    while (hole > top && less(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

template <class T, class Less>
void heap_select(T* first, T* middle, T* last, Less less)
{
    const long len = middle - first;
    if (len >= 2)   // __make_heap
        for (long parent = (len - 2) / 2;; parent--) {
            adjust_heap(first, parent, len, first[parent], less);
            if (parent == 0) break;
        }
    for (T* i = middle; i < last; ++i)
        if (less(*i, *first)) {   // __pop_heap(first, middle, i)
            T value = *i;
            *i = *first;
            adjust_heap(first, 0, len, value, less);
        }
}

template <class T, class Less>
void insertion_sort(T* first, T* last, Less less)
{
    if (first == last) return;
    for (T* i = first + 1; i != last; ++i) {
        T val = *i;
        if (less(val, *first)) {
            for (T* k = i; k != first; --k) *k = *(k - 1);
            *first = val;
        } else {   // __unguarded_linear_insert
            T* k = i;
            while (less(val, *(k - 1))) {
                *k = *(k - 1);
                --k;
            }
            *k = val;
        }
    }
}

template <class T, class Less>
T* unguarded_partition(T* first, T* last, T* pivot, Less less)
{
    while (true) {
        while (less(*first, *pivot)) ++first;
        --last;
        while (less(*pivot, *last)) --last;
        if (!(first < last)) return first;
        std::swap(*first, *last);
        ++first;
    }
}

template <class T, class Less>
void pivot_to_first(T* first, T* last, Less less, int mode)
{
    T* mid = first + (last - first) / 2;
    if (mode == NTH_PIVOT_GCC48) {   // __move_median_first(first, mid, last - 1)
        T *a = first, *b = mid, *c = last - 1;
        if (less(*a, *b)) {
            if (less(*b, *c)) std::swap(*a, *b);
            else if (less(*a, *c)) std::swap(*a, *c);
        } else if (less(*a, *c)) {
            return;
        } else if (less(*b, *c)) {
            std::swap(*a, *c);
        } else {
            std::swap(*a, *b);
        }
        return;
    }
    // __move_median_to_first(first, first + 1, mid, last - 1)
    T *a = first + 1, *b = mid, *c = last - 1, *t;
    if (less(*a, *b)) {
        if (less(*b, *c)) t = b;
        else if (less(*a, *c)) t = c;
        else t = a;
    } else if (less(*a, *c)) {
        t = a;
    } else if (less(*b, *c)) {
        t = c;
    } else {
        t = b;
    }
    std::swap(*first, *t);
}
}  // namespace

template <class T, class Less>
void libstdcxx_nth_element(T* first, T* nth, T* last, Less less, int mode)
{
    if (first == last || nth == last) return;
    long depth = 0;
    for (long n = last - first; n > 1; n >>= 1) depth++;   // __lg
    depth *= 2;
    while (last - first > 3) {
        if (depth == 0) {
            heap_select(first, nth + 1, last, less);
            std::swap(*first, *nth);
            return;
        }
        --depth;
        pivot_to_first(first, last, less, mode);
        T* cut = unguarded_partition(first + 1, last, first, less);
        if (cut <= nth) first = cut;
        else last = cut;
    }
    insertion_sort(first, last, less);
}
template void libstdcxx_nth_element<KeyPoint>(KeyPoint*, KeyPoint*, KeyPoint*,
                                              bool (*)(const KeyPoint&, const KeyPoint&), int);

static bool response_greater(const KeyPoint& a, const KeyPoint& b) { return a.response > b.response; }

// KeyPointsFilter::retainBest (OpenCV 2.4 features2d/src/keypoint.cpp).
// Called at src/ORBextractor.cc:683 and :699.  The surviving set and order is
// the libstdc++ introselect permutation (std::nth_element, era as above).
// ---------------------------------------------------------------------------
void cv24_retain_best(std::vector<KeyPoint>& kps, int n_points)
{
    if (n_points >= 0 && kps.size() > (size_t)n_points) {
        if (n_points == 0) {
            kps.clear();
            return;
        }
        libstdcxx_nth_element(kps.data(), kps.data() + n_points, kps.data() + kps.size(), response_greater,
                              g_nth_pivot);
        const float ambiguous = kps[n_points - 1].response;
        auto newEnd = std::partition(kps.begin() + n_points, kps.end(),
                                     [ambiguous](const KeyPoint& k) { return k.response >= ambiguous; });
        kps.resize(newEnd - kps.begin());
    }
}

// ---------------------------------------------------------------------------
// GaussianBlur(level, level, Size(7,7), 2, 2, BORDER_REFLECT_101) in place
// on a pyramid ROI (src/ORBextractor.cc:760).  OpenCV 2.4: float kernel from
// getGaussianKernel(7, 2, CV_32F), converted to int with scale 256 (the
// 8U smoothing fixed-point path of createSeparableLinearFilter); row pass =
// exact int sums; column pass = SymmColumnFilter<FixedPtCastEx<int,uchar>>
// whose SSE2 vector op (SymmColumnVec_32s8u) evaluates in float and rounds
// with cvtps2dq, and whose scalar tail uses (s + 2^15) >> 16.  The ROI is not
// isolated, so the unblurred padded border feeds the filter and stays
// unblurred in the output.
// ---------------------------------------------------------------------------
static std::vector<int> gaussian_kernel_int()
{
    const int n = 7;
    const double sigma = 2.0;
    float cf[7];
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    for (int i = 0; i < n; i++) {
        const double x = i - (n - 1) * 0.5;
        cf[i] = (float)std::exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    std::vector<int> k(n);
    for (int i = 0; i < n; i++) {
        cf[i] = (float)(cf[i] * sum);
        k[i] = cvRound(cf[i] * 256.0f);   // convertTo(CV_32S, 1<<8)
    }
    return k;
}

void cv24_gaussian_blur7_roi(const PaddedImage& src, PaddedImage& dst)
{
    static const std::vector<int> k = gaussian_kernel_int();
    dst = src;  // border bytes stay as in the source
    const int w = src.w, h = src.h;
    // Row pass over ROI rows -3..h+2 (parent pixels supply the border).
    std::vector<int> rows((size_t)(h + 6) * w);
    for (int y = -3; y < h + 3; y++) {
        const uint8_t* s = src.roi(0, y);
        int* r = &rows[(size_t)(y + 3) * w];
        for (int x = 0; x < w; x++) {
            int acc = 0;
            for (int i = 0; i < 7; i++) acc += k[i] * s[x + i - 3];
            r[x] = acc;
        }
    }
    float ky[4];
    for (int i = 0; i < 4; i++) ky[i] = (float)(k[3 + i] * (1.0 / 65536));  // convertTo(CV_32F, 1/2^16)
    const int nvec = vecCount(w, false);
    for (int y = 0; y < h; y++) {
        uint8_t* d = dst.roi(0, y);
        const int* R[7];
        for (int i = 0; i < 7; i++) R[i] = &rows[(size_t)(y + i) * w];
        for (int x = 0; x < w; x++) {
            if (x < nvec) {
                float s = (float)R[3][x] * ky[0] + 0.0f;
                for (int j = 1; j <= 3; j++)
                    s = s + (float)(R[3 + j][x] + R[3 - j][x]) * ky[j];
                const int iv = (int)std::nearbyint(s);   // _mm_cvtps_epi32
                d[x] = satU8(satS16(iv));                // packs_epi32 + packus_epi16
            } else {
                int s = k[3] * R[3][x];
                for (int j = 1; j <= 3; j++) s += k[3 + j] * (R[3 + j][x] + R[3 - j][x]);
                d[x] = satU8((s + (1 << 15)) >> 16);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// ORBextractor::ORBextractor (src/ORBextractor.cc:457-511)
// ---------------------------------------------------------------------------
ORBextractorRef::ORBextractorRef(int _nfeatures, float _scaleFactor, int _nlevels,
                                 int _scoreType, int _fastTh)
    : nlevels(_nlevels), nfeatures(_nfeatures), scaleFactor(_scaleFactor),
      scoreType(_scoreType), fastTh(_fastTh)
{
    mvScaleFactor.resize(nlevels);
    mvScaleFactor[0] = 1;
    for (int i = 1; i < nlevels; i++) mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);
    const float invScaleFactor = (float)(1.0f / scaleFactor);
    mvInvScaleFactor.resize(nlevels);
    mvInvScaleFactor[0] = 1;
    for (int i = 1; i < nlevels; i++) mvInvScaleFactor[i] = mvInvScaleFactor[i - 1] * invScaleFactor;

    mnFeaturesPerLevel.resize(nlevels);
    const float factor = (float)(1.0 / scaleFactor);
    float nDesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int level = 0; level < nlevels - 1; level++) {
        mnFeaturesPerLevel[level] = cvRound(nDesired);
        sum += mnFeaturesPerLevel[level];
        nDesired *= factor;
    }
    mnFeaturesPerLevel[nlevels - 1] = std::max(nfeatures - sum, 0);

    umax.resize(kHalfPatch + 1);
    const int vmax = cvFloor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
    const double hp2 = kHalfPatch * kHalfPatch;
    int v, v0;
    for (v = 0; v <= vmax; ++v) umax[v] = cvRound(std::sqrt(hp2 - v * v));
    for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
}

// ---------------------------------------------------------------------------
// ComputePyramid (src/ORBextractor.cc:781-822).  The mask path is dead for
// the caller (Frame passes cv::Mat(), src/Frame.cc:59) and is not restated.
// ---------------------------------------------------------------------------
void ORBextractorRef::computePyramid(const uint8_t* img, int w, int h, size_t stride)
{
    pyramid.assign(nlevels, PaddedImage());
    for (int level = 0; level < nlevels; ++level) {
        const float scale = mvInvScaleFactor[level];
        const int lw = cvRound((float)w * scale), lh = cvRound((float)h * scale);
        PaddedImage& L = pyramid[level];
        L.w = lw;
        L.h = lh;
        L.pw = lw + 2 * kEdge;
        L.ph = lh + 2 * kEdge;
        L.buf.assign((size_t)L.pw * L.ph, 0);
        if (level != 0) {
            const PaddedImage& P = pyramid[level - 1];
            cv24_resize_linear_u8(P.roi(0, 0), P.step(), P.w, P.h, L.roi(0, 0), L.step(), lw, lh);
        } else {
            for (int y = 0; y < lh; y++) std::memcpy(L.roi(0, y), img + (size_t)y * stride, lw);
        }
        // copyMakeBorder(..., BORDER_REFLECT_101[+ISOLATED]): border from the
        // level itself (the level-0 input is a whole image, not a ROI).
        for (int y = -kEdge; y < lh + kEdge; y++) {
            const int sy = reflect101(y, lh);
            for (int x = -kEdge; x < lw + kEdge; x++) {
                if (y >= 0 && y < lh && x >= 0 && x < lw) continue;
                *L.roi(x, y) = *L.roi(reflect101(x, lw), sy);
            }
        }
    }
}

// IC_Angle (src/ORBextractor.cc:124-151)
static float ic_angle(const PaddedImage& image, float px, float py, const std::vector<int>& u_max)
{
    int m_01 = 0, m_10 = 0;
    const uint8_t* center = image.roi(cvRound(px), cvRound(py));
    for (int u = -kHalfPatch; u <= kHalfPatch; ++u) m_10 += u * center[u];
    const int step = image.step();
    for (int v = 1; v <= kHalfPatch; ++v) {
        int v_sum = 0;
        const int d = u_max[v];
        for (int u = -d; u <= d; ++u) {
            const int val_plus = center[u + v * step], val_minus = center[u - v * step];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return fast_atan2_cv24((float)m_01, (float)m_10);
}

// ---------------------------------------------------------------------------
// ComputeKeyPoints (src/ORBextractor.cc:522-707)
// ---------------------------------------------------------------------------
void ORBextractorRef::computeKeyPoints(std::vector<std::vector<KeyPoint>>& allKeypoints)
{
    allKeypoints.assign(nlevels, {});
    cellTotals.assign(nlevels, {});
    const float imageRatio = (float)pyramid[0].w / pyramid[0].h;
    for (int level = 0; level < nlevels; ++level) {
        PaddedImage& L = pyramid[level];
        const int nDesired = mnFeaturesPerLevel[level];
        const int levelCols = (int)std::sqrt((float)nDesired / (5 * imageRatio));
        const int levelRows = (int)(imageRatio * levelCols);
        const int minBorderX = kEdge, minBorderY = kEdge;
        const int maxBorderX = L.w - kEdge, maxBorderY = L.h - kEdge;
        const int W = maxBorderX - minBorderX, H = maxBorderY - minBorderY;
        if (levelCols <= 0 || levelRows <= 0)
            throw std::runtime_error("ComputeKeyPoints: empty cell grid (reference divides by zero)");
        const int cellW = (int)std::ceil((float)W / levelCols);
        const int cellH = (int)std::ceil((float)H / levelRows);
        const int nCells = levelRows * levelCols;
        const int nfeaturesCell = (int)std::ceil((float)nDesired / nCells);

        std::vector<std::vector<std::vector<KeyPoint>>> cellKeys(levelRows, std::vector<std::vector<KeyPoint>>(levelCols));
        std::vector<std::vector<int>> nToRetain(levelRows, std::vector<int>(levelCols, 0));
        std::vector<std::vector<int>> nTotal(levelRows, std::vector<int>(levelCols, 0));
        std::vector<std::vector<bool>> bNoMore(levelRows, std::vector<bool>(levelCols, false));
        std::vector<int> iniXCol(levelCols), iniYRow(levelRows);
        int nNoMore = 0, nToDistribute = 0;
        float hY = cellH + 6;
        for (int i = 0; i < levelRows; i++) {
            const float iniY = minBorderY + i * cellH - 3;
            iniYRow[i] = (int)iniY;
            if (i == levelRows - 1) {
                hY = maxBorderY + 3 - iniY;
                if (hY <= 0) continue;
            }
            float hX = cellW + 6;
            for (int j = 0; j < levelCols; j++) {
                float iniX;
                if (i == 0) {
                    iniX = minBorderX + j * cellW - 3;
                    iniXCol[j] = (int)iniX;
                } else {
                    iniX = iniXCol[j];
                }
                if (j == levelCols - 1) {
                    hX = maxBorderX + 3 - iniX;
                    if (hX <= 0) continue;
                }
                const int r0 = (int)iniY, r1 = (int)(iniY + hY);
                const int c0 = (int)iniX, c1 = (int)(iniX + hX);
                if (r0 < 0 || c0 < 0 || r1 > L.h || c1 > L.w)
                    throw std::runtime_error("ComputeKeyPoints: cell ROI outside the level");
                const uint8_t* cell = L.roi(c0, r0);
                std::vector<KeyPoint>& ck = cellKeys[i][j];
                cv24_fast16(cell, L.step(), r1 - r0, c1 - c0, fastTh, true, ck);
                if (ck.size() <= 3) {
                    ck.clear();
                    cv24_fast16(cell, L.step(), r1 - r0, c1 - c0, 7, true, ck);
                }
                // ORB::HARRIS_SCORE == 0 (:616-620, HARRIS_K = 0.04f :73)
                if (scoreType == 0) cv24_harris_responses(cell, L.step(), ck, 7, 0.04f);
                const int nKeys = (int)ck.size();
                nTotal[i][j] = nKeys;
                if (nKeys > nfeaturesCell) {
                    nToRetain[i][j] = nfeaturesCell;
                    bNoMore[i][j] = false;
                } else {
                    nToRetain[i][j] = nKeys;
                    nToDistribute += nfeaturesCell - nKeys;
                    bNoMore[i][j] = true;
                    nNoMore++;
                }
            }
        }

        while (nToDistribute > 0 && nNoMore < nCells) {
            const int nNewFeaturesCell = nfeaturesCell + (int)std::ceil((float)nToDistribute / (nCells - nNoMore));
            nToDistribute = 0;
            for (int i = 0; i < levelRows; i++) {
                for (int j = 0; j < levelCols; j++) {
                    if (!bNoMore[i][j]) {
                        if (nTotal[i][j] > nNewFeaturesCell) {
                            nToRetain[i][j] = nNewFeaturesCell;
                            bNoMore[i][j] = false;
                        } else {
                            nToRetain[i][j] = nTotal[i][j];
                            nToDistribute += nNewFeaturesCell - nTotal[i][j];
                            bNoMore[i][j] = true;
                            nNoMore++;
                        }
                    }
                }
            }
        }

        std::vector<KeyPoint>& keypoints = allKeypoints[level];
        keypoints.reserve(nDesired * 2);
        const int scaledPatchSize = (int)(kPatchSize * mvScaleFactor[level]);
        for (int i = 0; i < levelRows; i++) {
            for (int j = 0; j < levelCols; j++) {
                cellTotals[level].push_back(nTotal[i][j]);
                std::vector<KeyPoint>& keysCell = cellKeys[i][j];
                cv24_retain_best(keysCell, nToRetain[i][j]);
                if ((int)keysCell.size() > nToRetain[i][j]) keysCell.resize(nToRetain[i][j]);
                for (size_t k = 0; k < keysCell.size(); k++) {
                    keysCell[k].x += iniXCol[j];
                    keysCell[k].y += iniYRow[i];
                    keysCell[k].octave = level;
                    keysCell[k].size = (float)scaledPatchSize;
                    keypoints.push_back(keysCell[k]);
                }
            }
        }
        if ((int)keypoints.size() > nDesired) {
            cv24_retain_best(keypoints, nDesired);
            keypoints.resize(nDesired);
        }
    }
    for (int level = 0; level < nlevels; ++level)
        for (KeyPoint& kp : allKeypoints[level]) kp.angle = ic_angle(pyramid[level], kp.x, kp.y, umax);
}

// ---------------------------------------------------------------------------
// ORBextractor::operator() (src/ORBextractor.cc:718-779)
// ---------------------------------------------------------------------------
bool ORBextractorRef::extract(const uint8_t* img, int w, int h, size_t stride,
                              std::vector<KeyPoint>& kps, std::vector<uint8_t>& desc)
{
    if (w <= 0 || h <= 0 || img == nullptr) return false;
    computePyramid(img, w, h, stride);
    std::vector<std::vector<KeyPoint>> allKeypoints;
    computeKeyPoints(allKeypoints);
    int nkeypoints = 0;
    for (int level = 0; level < nlevels; ++level) nkeypoints += (int)allKeypoints[level].size();
    desc.assign((size_t)nkeypoints * 32, 0);
    kps.clear();
    kps.reserve(nkeypoints);
    blurred.assign(nlevels, PaddedImage());
    levelKeys = allKeypoints;
    int offset = 0;
    for (int level = 0; level < nlevels; ++level) {
        std::vector<KeyPoint>& keypoints = allKeypoints[level];
        const int n = (int)keypoints.size();
        cv24_gaussian_blur7_roi(pyramid[level], blurred[level]);
        if (n == 0) continue;
        for (int i = 0; i < n; i++) orb_descriptor(keypoints[i], blurred[level], &desc[(size_t)(offset + i) * 32]);
        offset += n;
        if (level != 0) {
            const float scale = mvScaleFactor[level];
            for (KeyPoint& kp : keypoints) {
                kp.x *= scale;
                kp.y *= scale;
            }
        }
        kps.insert(kps.end(), keypoints.begin(), keypoints.end());
    }
    return true;
}

}  // namespace orbref
