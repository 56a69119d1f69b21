// Device layout of a PoseOptimization problem (orbx_pose.hip's k_pose_opt),
// shared with the tracking chain (orbx_search.hip), which builds problems on
// the device.
#pragma once

#include <cstdint>

struct orbx_ctx;

namespace orbx {

struct PoseHdr {
    long long e0;        // first edge in the SoA arrays
    int nE;              // edges (keypoints with a map point)
    int pad;
    float T[12];         // initial Tcw rows 0..2
    float cam[4];        // fx fy cx cy
};

struct PoseOut {
    float T[12];
    int n_inliers;
    int rounds;
    int iterations[4];
    int trials[4];
    int n_bad[4];
    int not_posdef;
    int pad;
    double chi2_final[4];
};

// Edge arrays (SoA): observation, information, fixed point
struct PoseEdgeArrays {
    const float* ox;
    const float* oy;
    const float* isig;
    const float* px;
    const float* py;
    const float* pz;
};

// Launches PoseOptimization on P problems resident in device memory
// (orbx_pose.hip; the kernel orbx_pose_run selects for the context).
int launch_pose_device(orbx_ctx* ctx, const PoseHdr* hdrs, const PoseEdgeArrays& ed, uint8_t* flags, PoseOut* outs,
                       int P);

}  // namespace orbx
