// ============================================================================
// ORACLE -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference hot path (worxli/ORB_SLAM) used as the
// parity checker for the HIP implementation.  Only tests/, __graft_entry__.
// smoke() and bench.py's cpu_baseline leg may load it.  It is never linked
// into the product library (orb_slam_amd/liborbx.so).
//
// Parity status: the reference cannot be built here (OpenCV 2.4, Eigen3 and
// CHOLMOD are absent) and ships no tests or fixtures,
// so this restatement is "parity unpinned" against the reference binary.  It
// restates the reference sources line by line (file:line cited at each
// function) plus the OpenCV-2.4 / libstdc++ / libm semantics recorded in
// DESIGN.md section 3.
// ============================================================================
#pragma once
#include <cstdint>
#include <cstddef>
#include <vector>

namespace orbref {

// cv::KeyPoint (OpenCV 2.4), 28 bytes -- identical layout to orbx_keypoint.
struct KeyPoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

// Padded 8-bit image: the (w+32)x(h+32) buffer ORBextractor::ComputePyramid
// allocates per level (src/ORBextractor.cc:786-789); the level is the ROI at
// (16,16).
struct PaddedImage {
    int w = 0, h = 0;      // ROI size
    int pw = 0, ph = 0;    // padded size
    std::vector<uint8_t> buf;
    uint8_t* roi(int x, int y) { return buf.data() + (size_t)(y + 16) * pw + (x + 16); }
    const uint8_t* roi(int x, int y) const { return buf.data() + (size_t)(y + 16) * pw + (x + 16); }
    int step() const { return pw; }
};

// ---- libm / OpenCV numeric helpers (ref_math.cpp) ----
float fast_atan2_cv24(float y, float x);     // cv::fastAtan2 (OpenCV 2.4)
float cr_cosf(float x);                      // correctly rounded cosf
float cr_sinf(float x);                      // correctly rounded sinf

// ---- extraction (ref_extract.cpp) ----
class ORBextractorRef {
public:
    ORBextractorRef(int nfeatures, float scaleFactor, int nlevels, int scoreType, int fastTh);
    // ORBextractor::operator() (src/ORBextractor.cc:718-779).  Returns false
    // when the image is empty (outputs untouched).
    bool extract(const uint8_t* img, int w, int h, size_t stride,
                 std::vector<KeyPoint>& kps, std::vector<uint8_t>& desc);

    int nlevels;
    int nfeatures;
    double scaleFactor;       // NB: double member (include/ORBextractor.h:66)
    int scoreType, fastTh;
    std::vector<int> mnFeaturesPerLevel;
    std::vector<int> umax;
    std::vector<float> mvScaleFactor, mvInvScaleFactor;
    std::vector<PaddedImage> pyramid;   // raw levels (after extract())
    std::vector<PaddedImage> blurred;   // blurred copies (after extract())
    // per-level keypoints in level coordinates, before the final scaling
    std::vector<std::vector<KeyPoint>> levelKeys;
    // per-cell FAST counts and chosen thresholds of the last call (debug)
    std::vector<std::vector<int>> cellTotals;
private:
    void computePyramid(const uint8_t* img, int w, int h, size_t stride);
    void computeKeyPoints(std::vector<std::vector<KeyPoint>>& allKeypoints);
};

// OpenCV-2.4 primitives exposed for unit tests
void cv24_resize_linear_u8(const uint8_t* src, int sstep, int sw, int sh,
                           uint8_t* dst, int dstep, int dw, int dh);
void cv24_fast16(const uint8_t* img, int step, int rows, int cols, int threshold,
                 bool nonmax, std::vector<KeyPoint>& kps);
int  cv24_corner_score16(const uint8_t* ptr, const int pixel[25], int threshold);
void cv24_gaussian_blur7_roi(const PaddedImage& src, PaddedImage& dst);
void cv24_retain_best(std::vector<KeyPoint>& kps, int n_points);
// libstdc++ nth_element restated with either era's pivot step (ref_extract.cpp)
enum { NTH_PIVOT_GCC49 = 0, NTH_PIVOT_GCC48 = 1 };
void set_nth_pivot(int mode);
int get_nth_pivot();
template <class T, class Less>
void libstdcxx_nth_element(T* first, T* nth, T* last, Less less, int mode);
// ---- reference-compiled float expressions (ref_orbsites.cpp; built with
//      and without FMA contraction) ----
void cv24_harris_responses(const uint8_t* img, int step, std::vector<KeyPoint>& pts, int blockSize, float harris_k);
void orb_descriptor(const KeyPoint& kpt, const PaddedImage& img, uint8_t* desc);
int orbsites_contracted();

// ---- matching (ref_match.cpp) ----
int descriptor_distance(const uint8_t* a, const uint8_t* b);

struct FrameRef {
    std::vector<KeyPoint> keys;     // mvKeysUn (== mvKeys: no distortion)
    std::vector<uint8_t> desc;      // N x 32
    float minX = 0, maxX = 0, minY = 0, maxY = 0;
    float gridWInv = 0, gridHInv = 0;
    std::vector<float> scaleFactors;
    std::vector<int> grid[64][48];
    void build(const KeyPoint* k, const uint8_t* d, int n, float minx, float maxx,
               float miny, float maxy, int nlevels, float scale);
    std::vector<size_t> featuresInArea(float x, float y, float r, int minLevel, int maxLevel) const;
};

int search_for_initialization(const FrameRef& F1, const FrameRef& F2,
                              std::vector<float>& prevMatched, std::vector<int>& matches12,
                              int windowSize, float nnratio, bool checkOri);
int window_search(const FrameRef& F1, const FrameRef& F2, const uint8_t* f1_mp,
                  int windowSize, int minLevel, int maxLevel, float nnratio,
                  bool checkOri, std::vector<int>& matches21);
int search_by_projection_pair(const FrameRef& F1, const FrameRef& F2,
                              const float* mp_xyz, const uint8_t* mp_valid,
                              const uint8_t* f2_assigned, const float* Tcw,
                              const float* cam, int windowSize, float nnratio,
                              std::vector<int>& matches21);
int search_by_projection_motion(const FrameRef& Cur, const FrameRef& Last,
                                const float* mp_xyz, const uint8_t* mp_valid,
                                const uint8_t* cur_assigned, const float* Tcw,
                                const float* cam, float th, bool checkOri,
                                std::vector<int>& matchesCur);
int search_by_projection_local(const FrameRef& F, int n_mp, const uint8_t* in_view,
                               const float* proj_xy, const int32_t* pred_level,
                               const float* view_cos, const uint8_t* mp_desc,
                               const uint8_t* f_assigned, float th, float nnratio,
                               std::vector<int>& matchesF);
bool is_in_frustum(const FrameRef& F, const float* Rcw, const float* tcw, const float* Ow, const float* cam,
                   const float* P, const float* Pn, float minDistance, float maxDistance, float viewingCosLimit,
                   float& u_out, float& v_out, int& level_out, float& cos_out);
void hamming_bf(const uint8_t* dA, int nA, const uint8_t* dB, int nB,
                int32_t* best_idx, int32_t* best, int32_t* second);

}  // namespace orbref
