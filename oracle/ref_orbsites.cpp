// ORACLE -- TEST INFRASTRUCTURE ONLY (see ref_common.h).
//
// The floating-point expressions of the extractor that live in the
// reference's OWN source (src/ORBextractor.cc), as opposed to OpenCV's.
// The reference is built with -O3 -march=native (CMakeLists.txt:12-13) and
// GCC contracts a*b + c*d into fused multiply-adds by default
// (-ffp-contract=fast outside ISO mode) on any FMA-capable host, while the
// OpenCV 2.4 library it links was built separately, without that.  So this
// one file is compiled twice by oracle/Makefile:
//   build/ref_orbsites.o          -ffp-contract=off  (ISO evaluation; liborbx_ref.so)
//   build/ref_orbsites_contract.o -ffp-contract=fast -march=haswell
//                                  (GCC's own contraction of the same
//                                   expressions; liborbx_ref_contract.so)
// and everything else in the oracle is shared.  The contraction choice is
// left to GCC on the reference's expression shapes, restated verbatim.
#include "ref_common.h"

#include <cmath>

namespace orbref {

namespace {

const int kPattern[256 * 4] = {
#include "ref_pattern.inc"
};

inline int cvRound(double v) { return (int)std::nearbyint(v); }

}  // namespace

// HarrisResponses (src/ORBextractor.cc:79-120): 7x7 block of 3x3 Sobel
// products around each keypoint of the cell image (pt in cell coordinates;
// the Sobel taps read one pixel past the block, inside the level buffer).
// Integer sums, then the float response in the source's evaluation order
// (src/ORBextractor.cc:117-118).
void cv24_harris_responses(const uint8_t* img, int step, std::vector<KeyPoint>& pts, int blockSize, float harris_k)
{
    const int r = blockSize / 2;
    float scale = (1 << 2) * blockSize * 255.0f;
    scale = 1.0f / scale;
    const float scale_sq_sq = scale * scale * scale * scale;
    for (KeyPoint& kp : pts) {
        const int x0 = cvRound(kp.x - r), y0 = cvRound(kp.y - r);
        const uint8_t* ptr0 = img + (ptrdiff_t)y0 * step + x0;
        int a = 0, b = 0, c = 0;
        for (int i = 0; i < blockSize; i++) {
            for (int j = 0; j < blockSize; j++) {
                const uint8_t* p = ptr0 + (ptrdiff_t)i * step + j;
                const int Ix = (p[1] - p[-1]) * 2 + (p[-step + 1] - p[-step - 1]) + (p[step + 1] - p[step - 1]);
                const int Iy = (p[step] - p[-step]) * 2 + (p[step - 1] - p[-step - 1]) + (p[step + 1] - p[-step + 1]);
                a += Ix * Ix;
                b += Iy * Iy;
                c += Ix * Iy;
            }
        }
        kp.response = ((float)a * b - (float)c * c - harris_k * ((float)a + b) * ((float)a + b)) * scale_sq_sq;
    }
}

// computeOrbDescriptor (src/ORBextractor.cc:155-194): a = cos, b = sin of
// the keypoint angle (:159-160, std::cos(float) / std::sin(float) = glibc
// cosf / sinf); sample (x, y) of the pattern is read at
// center[cvRound(x*b + y*a) * step + cvRound(x*a - y*b)] (GET_VALUE, :165-167),
// the pattern's int coordinates converted to float.
void orb_descriptor(const KeyPoint& kpt, const PaddedImage& img, uint8_t* desc)
{
    const float factorPI = (float)(M_PI / 180.f);
    const float angle = (float)kpt.angle * factorPI;
    const float a = cr_cosf(angle), b = cr_sinf(angle);
    const uint8_t* center = img.roi(cvRound(kpt.x), cvRound(kpt.y));
    const int step = img.step();
    const int* pattern = kPattern;
    for (int i = 0; i < 32; ++i, pattern += 32) {
        int val = 0;
        for (int bit = 0; bit < 8; bit++) {
            const int* p0 = pattern + 4 * bit;
            const int* p1 = p0 + 2;
            const int t0 = center[cvRound(p0[0] * b + p0[1] * a) * step + cvRound(p0[0] * a - p0[1] * b)];
            const int t1 = center[cvRound(p1[0] * b + p1[1] * a) * step + cvRound(p1[0] * a - p1[1] * b)];
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

// 1 when this translation unit was built with FMA contraction
int orbsites_contracted()
{
#ifdef ORBREF_CONTRACT
    return 1;
#else
    return 0;
#endif
}

}  // namespace orbref
