/*
 * orbx.h -- C ABI of the MI355X-native ORB-SLAM front end + local-BA kernels.
 *
 * Every entry point below replaces one reference interface on the hot path
 * named by BASELINE.json's north_star.  The reference is
 * a single C++ executable with no FFI layer, so the "binding" is a C++ adapter
 * (orb_slam_amd/adapters/, shown in INTEGRATION.md) that keeps the reference
 * class signatures and calls these functions.  Signatures use plain pointers
 * and sizes only; all device memory is owned by an orbx_ctx.
 *
 * Conventions
 *   - return 0 (ORBX_OK) on success, a negative ORBX_ERR_* code otherwise.
 *     The reference has no error codes (it asserts or returns silently); the
 *     adapter maps codes back to that behaviour.
 *   - host pointers are caller-allocated; "cap" arguments bound outputs.
 *   - an orbx_ctx owns one HIP stream and its buffers; it is NOT thread-safe
 *     (mirrors ORBextractor, whose pyramid is member state:
 *     include/ORBextractor.h:74).  Use one context per calling thread.
 */
#ifndef ORBX_H
#define ORBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI revision of this header.  A caller compares orbx_abi_version() with the
 * ORBX_ABI_VERSION it was compiled against before its first call (the C++
 * adapter does, in every constructor) and refuses a library of another
 * revision instead of calling through a changed signature.
 *   1: rounds 1-3.
 *   2: orbx_lba_solve_batch / orbx_lba_run take per-problem abort flags
 *      (the `aborts` argument after iters1).
 *   3: single-frame graph path (orbx_set_launch_mode), host-fed pipeline
 *      (orbx_host_alloc, orbx_dev_upload_async, orbx_dev_download_async),
 *      image bounds of device-resident frames (orbx_dev_set_image_bounds),
 *      multi-workgroup single local-BA problems (orbx_lba_set_workgroups);
 *      additions only.
 *   4: orbx_pose_set_exact / orbx_pose_get_exact; additions only.
 *   5: the measured-slower opt-in modes removed (orbx_dev_set_pyramid_mode,
 *      orbx_dev_pyramid_fused / _kind, orbx_dev_set_fast_chunk / get, launch
 *      modes 2 and 3); orbx_lba_last_workgroups, orbx_debug_lba_split;
 *      orbx_track_frame (one Tracking frame on the device); PoseOptimization
 *      sums sequentially in g2o's order by default (orbx_pose_set_exact). */
#define ORBX_ABI_VERSION 5
int orbx_abi_version(void);

#define ORBX_OK               0
#define ORBX_ERR_ARG         -1  /* invalid argument / shape                      */
#define ORBX_ERR_HIP         -2  /* HIP runtime failure (device missing, launch)  */
#define ORBX_ERR_CAPACITY    -3  /* caller buffer or context capacity too small   */
#define ORBX_ERR_UNSUPPORTED -4  /* configuration outside the implemented subset  */
#define ORBX_ERR_NOMEM       -5  /* device or host allocation failed              */
#define ORBX_ERR_NOT_POSDEF  -6  /* reduced camera system not positive definite   */

/* cv::KeyPoint layout (OpenCV 2.4 core/types.hpp): 28 bytes. */
typedef struct {
    float x, y;        /* pt                                 */
    float size;        /* diameter of the meaningful region  */
    float angle;       /* degrees in [0,360)                 */
    float response;    /* FAST score                         */
    int32_t octave;    /* pyramid level                      */
    int32_t class_id;  /* always -1                          */
} orbx_keypoint;

typedef struct orbx_ctx orbx_ctx;

/* ------------------------------------------------------------------------ */
/* Context / extractor construction                                          */
/* ------------------------------------------------------------------------ */

/* Replaces ORBextractor::ORBextractor(int nfeatures, float scaleFactor,
 * int nlevels, int scoreType, int fastTh)  (src/ORBextractor.cc:457-511,
 * include/ORBextractor.h:37).  max_w/max_h/max_batch size the device
 * buffers (frames larger than max_w x max_h are rejected); max_batch is the
 * number of frames one batched launch may carry and also the number of
 * device-resident frame slots available to orbx_dev_* (see below).
 * score_type: 0 = ORB::HARRIS_SCORE (HarrisResponses re-scores the FAST
 * corners before retainBest, src/ORBextractor.cc:79-120, :616-620; keypoint
 * responses are the Harris values), any other value = FAST_SCORE (the FAST
 * score; the reference tests only == HARRIS_SCORE). */
int  orbx_create(orbx_ctx** out, int device, int nfeatures, float scale_factor,
                 int nlevels, int score_type, int fast_th,
                 int max_w, int max_h, int max_batch);
void orbx_destroy(orbx_ctx* ctx);

/* ORBextractor::GetLevels / GetScaleFactor (include/ORBextractor.h:47-51). */
int   orbx_get_levels(const orbx_ctx* ctx);
float orbx_get_scale_factor(const orbx_ctx* ctx);
/* mnFeaturesPerLevel (src/ORBextractor.cc:476-487) and mvScaleFactor. */
int   orbx_get_features_per_level(const orbx_ctx* ctx, int32_t* out, int cap);
int   orbx_get_scale_factors(const orbx_ctx* ctx, float* out, int cap);

/* Host-side extractor tables for a frame size, computed without a device:
 * per level 8 ints {w, h, n_desired, level_cols, level_rows, nfeatures_cell,
 * n_cells, n_valid_cells} (src/ORBextractor.cc:462-487, 527-547, 786).
 * Returns the number of levels or a negative error. */
int orbx_describe_levels(int nfeatures, float scale_factor, int nlevels, int fast_th,
                         int w, int h, int32_t* out, int cap);

/* ------------------------------------------------------------------------ */
/* A. Extraction                                                             */
/* ------------------------------------------------------------------------ */

/* Replaces ORBextractor::operator()(image, mask=Mat(), keypoints, descriptors)
 * (src/ORBextractor.cc:718-779).  img: w x h mono8 with row stride `stride`.
 * Outputs keypoints in reference order (level-major, retainBest order within
 * a level; coordinates scaled to level 0) and N x 32 descriptor bytes.
 * An empty image (w==0 || h==0) returns ORBX_OK with *n_out = 0 -- the
 * reference returns without touching its outputs (:721-722). */
int orbx_extract(orbx_ctx* ctx, const uint8_t* img, int w, int h, size_t stride,
                 orbx_keypoint* kps, uint8_t* desc, int cap, int* n_out);
/* How orbx_extract issues its work (Frame::Frame calls the extractor once per
 * frame, synchronously: src/Frame.cc:59, src/Tracking.cc:206).
 *   1 (default): the call is one hipGraph launch -- the image copied through a
 *     page-locked staging buffer into its slot, the extraction kernels (the
 *     blur on a branch beside FAST and retainBest), then one kernel that
 *     stores the count, error flags, keypoints and descriptors into a
 *     page-locked buffer -- and one synchronisation.  The graph is captured
 *     on the first call of a configuration (frame size, fp-contract mode,
 *     nth_element era) and replayed after that.
 *   0: the kernels launched one by one on the context stream, with pageable
 *     copies (rounds 1-4).
 * Both produce identical outputs; kernel timing (orbx_dev_kernel_time_enable)
 * takes the stream launches.  (Modes 2 -- the pyramid reading the staging
 * buffer in place -- and 3 -- the single-frame launches without a graph --
 * measured within noise of 1 and were removed in ABI 5.) */
int orbx_set_launch_mode(orbx_ctx* ctx, int mode);
int orbx_get_launch_mode(const orbx_ctx* ctx);

/* Batched form: B frames of identical size, host in / host out.
 * kps: B*cap records, desc: B*cap*32 bytes, n_out: B counts. */
int orbx_extract_batch(orbx_ctx* ctx, int B, const uint8_t* const* imgs,
                       int w, int h, size_t stride,
                       orbx_keypoint* kps, uint8_t* desc, int cap, int32_t* n_out);

/* ------------------------------------------------------------------------ */
/* Device-resident pipeline (inputs already in HBM; used by bench/tests).     */
/* A context owns `max_batch` frame slots.  Frames are uploaded once, then    */
/* extracted and matched without host round-trips.                            */
/* ------------------------------------------------------------------------ */

/* Copy `count` host frames (w x h, contiguous rows of `stride` bytes, frame k
 * at imgs + k*h*stride) into slots [first, first+count).  All slots of one
 * context share one frame size (set by the first upload). */
int orbx_dev_upload(orbx_ctx* ctx, int first, int count, const uint8_t* imgs,
                    int w, int h, size_t stride);
/* Extract slots [first, first+count) (async, on the context stream).
 * Batches of 32+ frames run as two halves on two internal streams (joined
 * before the call's later work) unless disabled with orbx_dev_set_split. */
int orbx_dev_extract(orbx_ctx* ctx, int first, int count);
/* Floating-point evaluation of the expressions that live in the reference's
 * own source rather than in OpenCV: computeOrbDescriptor's sample coordinates
 * x*b + y*a, x*a - y*b (src/ORBextractor.cc:165-167) and HarrisResponses'
 * response (:117-118).  0 (default): each operation rounded as written (ISO
 * C++, the reference built with -ffp-contract=off or on a host without FMA).
 * 1: as GCC evaluates them when it builds the reference with its own flags
 * (-O3 -march=native, CMakeLists.txt:12-13) on an FMA host, where GCC's
 * default -ffp-contract=fast fuses them: fma(x, b, y*a), fma(x, a, -(y*b));
 * fma(-(k*(a+b)), a+b, fma(a, b, -(c*c))).  Applies to extractions launched
 * after the call (DESIGN.md section 4 has the measured effect). */
int orbx_set_fp_contract(orbx_ctx* ctx, int enable);
int orbx_get_fp_contract(const orbx_ctx* ctx);
/* libstdc++ era of retainBest's std::nth_element (KeyPointsFilter::retainBest,
 * called at src/ORBextractor.cc:683, :699).  The surviving keypoints and their
 * order are nth_element's permutation, and libstdc++ changed its introselect
 * pivot step in GCC 4.9 (PR libstdc++/58437):
 *   ORBX_NTH_PIVOT_GCC49 (0): median of (first + 1, mid, last - 1) swapped
 *     into first -- GCC >= 4.9;
 *   ORBX_NTH_PIVOT_GCC48 (1, default): median of (first, mid, last - 1)
 *     moved to first -- GCC 4.6 .. 4.8, the compilers of the platforms the
 *     reference documents (Ubuntu 12.04 / 14.04, README.md:46), whose OpenCV
 *     2.4 packages instantiate retainBest's nth_element.
 * Applies to extractions launched after the call (DESIGN.md section 4 has the
 * measured effect). */
enum { ORBX_NTH_PIVOT_GCC49 = 0, ORBX_NTH_PIVOT_GCC48 = 1 };
int orbx_set_nth_pivot(orbx_ctx* ctx, int mode);
int orbx_get_nth_pivot(const orbx_ctx* ctx);
/* enable: 0 = one stream; 1 = split with the default three parts;
 * 2..4 = split, and the asynchronous extract_match pipeline runs its batch
 * in that many parts on as many streams, part i released by part i-1's
 * FAST pass. */
int orbx_dev_set_split(orbx_ctx* ctx, int enable);
/* orbx_dev_extract followed by matching every slot of the batch against its
 * predecessor (mode 1: orbx_dev_match_prev with window / nnratio / check_ori;
 * mode 2: orbx_dev_match_bf_prev with th_low / nnratio), pipelined: with the
 * two-stream split each half's internal pairs are matched while the other
 * half is still being extracted.  Results as for the separate calls. */
int orbx_dev_extract_match(orbx_ctx* ctx, int first, int count, int seq_len, int mode,
                           int window, int th_low, float nnratio, int check_ori);
/* Asynchronous matching for orbx_dev_extract_match: the batch's matching is
 * queued on an internal stream after its extraction, and the call returns;
 * a later extract_match of *other* slots overlaps it (a stream of batches
 * alternating between two slot ranges keeps extraction and matching of
 * consecutive batches concurrent).  Any other call on the context, or an
 * extraction into slots the pending match reads, waits for it first. */
int orbx_dev_set_async_match(orbx_ctx* ctx, int enable);
/* (ABI 5 removed the opt-in pyramid modes -- one fused pyramid + blur
 * launch per batch, and the band-cascade raw pyramid for batches -- and
 * chunked FAST workgroups: each measured slower than the default at every
 * frame size.  The band cascade remains the pyramid of
 * orbx_extract's single-frame graph, where it is the fastest.) */
/* SearchForInitialization (B3) for slots [first, first+count): slot s is
 * matched against slot s-1 unless s % seq_len == 0 (sequence start).  Frame
 * s-1 plays F1 (initial frame), s plays F2; vbPrevMatched = F1 keypoints. */
int orbx_dev_match_prev(orbx_ctx* ctx, int first, int count, int seq_len,
                        int window, float nnratio, int check_ori);
/* Image bounds of the slots' keypoints for the device-resident matchers
 * (orbx_dev_match_prev and the extract_match pipeline): Frame's static
 * mnMinX, mnMaxX, mnMinY, mnMaxY (src/Frame.cc:320-348), which also scale its
 * 64x48 grid (:76-77).  After orbx_dev_undistort with a distorting camera,
 * pass orbx_compute_image_bounds' result; NULL (the default) is 0..w x 0..h,
 * the reference's bounds without distortion (:341-347). */
int orbx_dev_set_image_bounds(orbx_ctx* ctx, const float* bounds);
/* Brute-force matching (config C3) of slots [first, first+count) against
 * their predecessors, same slot pairing as orbx_dev_match_prev: every
 * keypoint of s-1 against every keypoint of s, accepted when best <= th_low
 * and best < nnratio * second (rule of src/ORBmatcher.cc:640-654); results
 * via orbx_dev_read_matches. */
int orbx_dev_match_bf_prev(orbx_ctx* ctx, int first, int count, int seq_len,
                           int th_low, float nnratio);
int orbx_dev_sync(orbx_ctx* ctx);
/* Host-fed pipeline: frames that arrive in host memory and results that must
 * leave it, overlapped with the extraction of other slots.
 * orbx_host_alloc / orbx_host_free: page-locked host memory (the copies below
 * overlap device work only from such memory).
 * orbx_dev_upload_async: like orbx_dev_upload, but queued on an internal copy
 * stream and returning at once; the copy waits for the extractions queued
 * before the call (which may still read the slots' previous frames), and a
 * later extraction of these slots waits for the copy.  The frame size must be
 * the context's current one (otherwise the call is orbx_dev_upload).
 * orbx_dev_download_async: queue read-backs of slots [first, first+count)
 * after their queued extraction and match: keypoints (count x nfeatures
 * records, slot-major), descriptors (count x nfeatures x 32), keypoint counts
 * (count), match vectors (count x nfeatures) and match counts (count); any
 * pointer may be NULL.  A later extraction of these slots waits for the
 * copies; the host buffers are complete after orbx_dev_sync. */
int  orbx_host_alloc(size_t bytes, void** out);
void orbx_host_free(void* p);
int  orbx_dev_upload_async(orbx_ctx* ctx, int first, int count, const uint8_t* imgs,
                           int w, int h, size_t stride);
int  orbx_dev_download_async(orbx_ctx* ctx, int first, int count, orbx_keypoint* kps,
                             uint8_t* desc, int32_t* n_kps, int32_t* matches12,
                             int32_t* n_matches);
/* Read back one slot's features / its match result (after sync). */
int orbx_dev_read_features(orbx_ctx* ctx, int slot, orbx_keypoint* kps,
                           uint8_t* desc, int cap, int* n_out);
int orbx_dev_read_matches(orbx_ctx* ctx, int slot, int32_t* matches12, int cap,
                          int* n_matches, int* n1);
/* Timing of the dominant kernels over the launches issued since the last
 * reset, measured with hipEvents on the context stream.  name: "pyr0",
 * "resize", "fast", "retain", "blur", "describe", "match".  Returns the number of
 * timed launches; *avg_ms receives the mean duration. */
int orbx_dev_kernel_time(orbx_ctx* ctx, const char* name, double* avg_ms,
                         double* total_ms);
int orbx_dev_kernel_time_enable(orbx_ctx* ctx, int enable);
/* Restrict kernel timing to the launches of one timer name (NULL or "":
 * all), so a timed region carries only the events it reports. */
int orbx_dev_kernel_time_select(orbx_ctx* ctx, const char* name);

/* Debug / parity taps: padded pyramid level (raw or blurred) of a slot.
 * Writes (w_l+32)*(h_l+32) bytes; *pw, *ph receive the padded size. */
int orbx_dev_read_level(orbx_ctx* ctx, int slot, int level, int blurred,
                        uint8_t* out, int cap, int* pw, int* ph);

/* ------------------------------------------------------------------------ */
/* B. Matching                                                               */
/* ------------------------------------------------------------------------ */

/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1794-1810), host side. */
int orbx_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Frame view consumed by the matchers: mvKeysUn, mDescriptors, image bounds
 * (Frame::ComputeImageBounds, src/Frame.cc:320-348) and the scale pyramid
 * (mvScaleFactors, src/Frame.cc:94-102).  The 64x48 cell grid
 * (src/Frame.cc:108-122) is rebuilt on the device from keys_un. */
typedef struct {
    const orbx_keypoint* keys_un;
    const uint8_t* desc;          /* n x 32 */
    int n;
    float min_x, max_x, min_y, max_y;
    int nlevels;
    float scale_factor;
} orbx_frame_view;

/* All-pairs Hamming (B8 primitive): for every row a of dA, the first index of
 * the smallest distance over dB, that distance and the second smallest value
 * of the multiset of distances (reference best/second rule, ORBmatcher.cc:
 * 640-649).  Distances are DescriptorDistance. */
int orbx_hamming_bf(orbx_ctx* ctx, const uint8_t* dA, int nA, const uint8_t* dB,
                    int nB, int32_t* best_idx, int32_t* best, int32_t* second);
/* Brute-force matcher (C3): best/second rule + accept best <= th_low and
 * best < nnratio*second.  m12[a] = matched b or -1. */
int orbx_match_bf(orbx_ctx* ctx, const uint8_t* dA, int nA, const uint8_t* dB,
                  int nB, int th_low, float nnratio, int32_t* m12, int* n_matches);

/* ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:598-713).
 * prev_matched: 2*F1->n floats (vbPrevMatched), updated in place.
 * matches12: F1->n entries (vnMatches12). */
int orbx_search_for_initialization(orbx_ctx* ctx, const orbx_frame_view* F1,
                                   const orbx_frame_view* F2, float* prev_matched,
                                   int32_t* matches12, int window, float nnratio,
                                   int check_ori, int* n_matches);

/* ORBmatcher::WindowSearch (src/ORBmatcher.cc:409-516).
 * f1_mp: per F1 keypoint, 1 if F1.mvpMapPoints[i1] is set and not bad.
 * matches21 (out, F2->n): i1 whose map point was assigned to F2 keypoint i2,
 * or -1 (vpMapPointMatches2 / vnMatches21).  max_level < 0 means INT_MAX. */
int orbx_window_search(orbx_ctx* ctx, const orbx_frame_view* F1,
                       const orbx_frame_view* F2, const uint8_t* f1_mp,
                       int window, int min_level, int max_level, float nnratio,
                       int check_ori, int32_t* matches21, int* n_matches);

/* ORBmatcher::SearchByProjection(Frame& F1, Frame& F2, int windowSize,
 * vector<MapPoint*>&) (src/ORBmatcher.cc:519-594).
 * f1_mp_xyz: 3 floats per F1 keypoint (world position of its map point);
 * f1_mp_valid: 1 if the point exists, is not bad and is not already in F2
 * (spMapPointsAlreadyFound).  f2_assigned (in): F2.mvpMapPoints non-null.
 * Tcw2: F2 pose, 12 floats row-major [R|t].  cam: fx, fy, cx, cy.
 * matches21 (out): F1 index assigned to each F2 keypoint or -1 (new only). */
int orbx_search_by_projection_pair(orbx_ctx* ctx, const orbx_frame_view* F1,
                                   const orbx_frame_view* F2,
                                   const float* f1_mp_xyz, const uint8_t* f1_mp_valid,
                                   const uint8_t* f2_assigned, const float* Tcw2,
                                   const float* cam, int window, float nnratio,
                                   int32_t* matches21, int* n_matches);

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame,
 * float th) (src/ORBmatcher.cc:1507-1620), motion-model tracking.
 * last_mp_xyz / last_mp_valid: per LastFrame keypoint (pMP && !mvbOutlier).
 * cur_assigned (in): CurrentFrame.mvpMapPoints non-null.
 * matches_cur (out, Cur->n): LastFrame index assigned to each current
 * keypoint by this call, or -1. */
int orbx_search_by_projection_motion(orbx_ctx* ctx, const orbx_frame_view* Cur,
                                     const orbx_frame_view* Last,
                                     const float* last_mp_xyz,
                                     const uint8_t* last_mp_valid,
                                     const uint8_t* cur_assigned, const float* Tcw,
                                     const float* cam, float th, int check_ori,
                                     int32_t* matches_cur, int* n_matches);

/* ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&, float th)
 * (src/ORBmatcher.cc:49-125), local-map tracking.  Per map point m (n_mp):
 * in_view (mbTrackInView && !isBad), proj_xy (mTrackProjX/Y), pred_level
 * (mnTrackScaleLevel), view_cos (mTrackViewCos), mp_desc (32 B).
 * f_assigned (in): F.mvpMapPoints non-null.  matches_f (out, F->n): index of
 * the map point assigned to each keypoint by this call, or -1. */
int orbx_search_by_projection_local(orbx_ctx* ctx, const orbx_frame_view* F,
                                    int n_mp, const uint8_t* in_view,
                                    const float* proj_xy, const int32_t* pred_level,
                                    const float* view_cos, const uint8_t* mp_desc,
                                    const uint8_t* f_assigned, float th, float nnratio,
                                    int32_t* matches_f, int* n_matches);

/* Tracking::SearchReferencePointsInFrustum (src/Tracking.cc:701-752) without a
 * host pass over the local map: Frame::isInFrustum(pMP, view_cos_limit)
 * (src/Frame.cc:136-197) for every local map point on the device, then
 * ORBmatcher(nnratio).SearchByProjection(F, mvpLocalMapPoints, th)
 * (src/ORBmatcher.cc:49-125) over the points found in view.  The frame's
 * pose matrices are Frame state (UpdatePoseMatrices, src/Frame.cc:129-134)
 * and are passed as such.  Outputs per point are what isInFrustum writes into
 * the MapPoint (mbTrackInView, mTrackProjX/Y, mnTrackScaleLevel,
 * mTrackViewCos); the caller applies IncreaseVisible() to the points in view
 * and the matches to mvpMapPoints, as the reference's loops do. */
typedef struct {
    const orbx_frame_view* frame;   /* F: mvKeysUn, mDescriptors, bounds, scale pyramid   */
    const float* Rcw;               /* 9, row-major (Frame::mRcw)                          */
    const float* tcw;               /* 3 (mtcw)                                            */
    const float* Ow;                /* 3 (mOw, the camera centre)                          */
    const float* cam;               /* fx, fy, cx, cy                                      */
    int n_mp;                       /* local map points                                    */
    const float* mp_pos;            /* n_mp x 3: GetWorldPos()                             */
    const float* mp_normal;         /* n_mp x 3: GetNormal()                               */
    const float* mp_dist;           /* n_mp x 2: GetMinDistanceInvariance(), GetMaxDistanceInvariance() */
    const uint8_t* mp_skip;         /* n_mp or NULL: 1 = not projected (isBad(), or
                                       mnLastFrameSeen == this frame: already matched)    */
    const uint8_t* mp_desc;         /* n_mp x 32: GetDescriptor()                          */
    const uint8_t* f_assigned;      /* F->n: mvpMapPoints non-null                         */
    float view_cos_limit;           /* 0.5 (src/Tracking.cc:738)                           */
    float th;                       /* 1, or 5 just after relocalisation (:745-748)        */
    float nnratio;                  /* 0.8 (:744)                                          */
    uint8_t* in_view;               /* out, n_mp or NULL: mbTrackInView                    */
    float* proj_xy;                 /* out, n_mp x 2 or NULL: mTrackProjX/Y                */
    int32_t* pred_level;            /* out, n_mp or NULL: mnTrackScaleLevel                */
    float* view_cos;                /* out, n_mp or NULL: mTrackViewCos                    */
    int32_t* matches_f;             /* out, F->n: map point assigned to each keypoint, or -1 */
    int n_in_view;                  /* out: points in view (nToMatch)                      */
    int n_matches;                  /* out: SearchByProjection's return value              */
} orbx_local_map_query;

int orbx_search_local_map(orbx_ctx* ctx, orbx_local_map_query* q);

/* One Tracking frame on the device (Tracking::TrackWithMotionModel then
 * Tracking::TrackLocalMap, src/Tracking.cc:573-600, 604-627): the current
 * frame's keypoints are read where extraction left them (slot `slot`; with
 * `image` set, the image is uploaded and extracted into that slot first),
 * and the chain
 *   SearchByProjection(current, last, 15)            (src/ORBmatcher.cc:1507)
 *   -> < 20 matches: status 1 (the reference then tries TrackPreviousFrame)
 *   -> PoseOptimization, outliers discarded          (src/Optimizer.cc:154)
 *   -> < 10 matches left: status 2
 *   -> SearchReferencePointsInFrustum: isInFrustum of the local map points
 *      not already matched, SearchByProjection(F, local map, th)
 *   -> PoseOptimization on all matches
 * (mode 0) or, mode 1, TrackPreviousFrame's
 *   WindowSearch(last, current, 200, minOctave), < 10: WindowSearch(100)
 *   -> >= 10: PoseOptimization from mLastFrame.mTcw, outliers discarded,
 *      SearchByProjection(last, current, 15); else SearchByProjection(.., 50)
 *   -> < 10 matches: status 3; PoseOptimization, outliers discarded; < 10: 4
 * followed by the same local-map search and PoseOptimization,
 * runs without a host round trip: one upload (last frame, local map, pose
 * prediction, image) and one read-back.  The last frame's map points are
 * named by their index in the map-point arrays.  The local map is an input:
 * the reference rebuilds it (UpdateReference, src/Tracking.cc:754-790) from
 * the keyframes that observe the motion search's matches, between the two
 * searches; a caller passes the one it holds (the previous frame's), which
 * is the reference's whenever those keyframes are unchanged, or runs the two
 * halves with the host-array calls (orbx_search_by_projection_motion,
 * orbx_pose_optimization, orbx_search_local_map).  The camera centre for the frustum
 * test is Frame::UpdatePoseMatrices' mOw = -Rcw^T tcw evaluated in float
 * left to right (the adapter's host glue does the same).  The undistorted
 * keypoints of the slot are its extracted keypoints (k1 = 0) or those
 * orbx_dev_undistort wrote; the frame bounds those of
 * orbx_dev_set_image_bounds (default 0..w, 0..h). */
typedef struct {
    int mode;                       /* 0: TrackWithMotionModel (src/Tracking.cc:572-611);
                                       1: TrackPreviousFrame (:497-569, the reference's
                                       fallback after status 1); both then TrackLocalMap  */
    int min_octave;                 /* mode 1: WindowSearch's minOctave (maxOctave / 2 + 1
                                       when KeyFramesInMap() > 5, else 0, :505-507)        */
    int slot;                       /* current frame's slot                                */
    const uint8_t* image;           /* NULL (slot already extracted) or the mono8 image    */
    int w, h;                       /* image size (also the default bounds)                */
    size_t stride;
    int last_slot;                  /* >= 0: LastFrame is that slot's extraction (the previous
                                       call's slot; `last` unused), else -1              */
    int last_cap;                   /* last_slot >= 0: entries of last_mp / last_outlier (at
                                       least that frame's n_cur, at most nfeatures)       */
    const orbx_frame_view* last;    /* last_slot < 0: LastFrame's mvKeysUn, mDescriptors,
                                       bounds, pyramid                                    */
    const int32_t* last_mp;         /* local-map index of LastFrame.mvpMapPoints[i], or -1 */
    const uint8_t* last_outlier;    /* LastFrame.mvbOutlier                                */
    int n_mp;                       /* map points of the arrays below                      */
    int n_local_mp;                 /* the first n_local_mp of them are mvpLocalMapPoints (the
                                       frustum search's); the rest only LastFrame's. <= 0: all */
    const float* mp_pos;            /* n_mp x 3                                            */
    const float* mp_normal;         /* n_mp x 3                                            */
    const float* mp_dist;           /* n_mp x 2: min, max distance invariance              */
    const uint8_t* mp_desc;         /* n_mp x 32                                           */
    const uint8_t* mp_skip;         /* n_mp or NULL: isBad()                               */
    const float* Tcw_pred;          /* 12: mode 0 rows 0..2 of mVelocity * mLastFrame.mTcw,
                                       mode 1 of mLastFrame.mTcw                          */
    const float* cam;               /* fx, fy, cx, cy                                      */
    const float* inv_level_sigma2;  /* nlevels (mvInvLevelSigma2)                          */
    int nlevels;
    float th_local;                 /* 1, or 5 just after relocalisation                   */
    /* outputs */
    float Tcw[12];                  /* final pose (rows 0..2): after the last PoseOptimization
                                       that ran (the prediction for status 1)              */
    int32_t* cur_mp;                /* cap: local-map index per current keypoint, or -1     */
    uint8_t* cur_outlier;           /* cap: mvbOutlier after the last PoseOptimization      */
    int cap;                        /* capacity of cur_mp / cur_outlier                    */
    int n_cur;                      /* current frame's keypoints                           */
    int status;                     /* 0 tracked (TrackLocalMap ran); mode 0: 1 / 2 above;
                                       mode 1: 3 < 10 matches after the window and pair
                                       searches, 4 < 10 left after their PoseOptimization */
    int n_motion;                   /* mode 0: SearchByProjection(current, last) matches;
                                       mode 1: the WindowSearch's (200, else 100)         */
    int n_pair;                     /* mode 1: SearchByProjection(last, current, 15 / 50)  */
    int n_after_pose;               /* matches left after the PoseOptimization before the
                                       local-map search                                   */
    int n_in_view;                  /* local map points in view (nToMatch)                  */
    int n_local;                    /* SearchByProjection(F, local map) matches            */
    int n_inliers;                  /* the last PoseOptimization's return value            */
} orbx_track_query;
int orbx_track_frame(orbx_ctx* ctx, orbx_track_query* q);
/* B independent frames (each with its own local map) in one upload, two
 * launches (all frustum tests, then one search wavefront per frame) and one
 * readback. */
int orbx_search_local_map_batch(orbx_ctx* ctx, int B, orbx_local_map_query* qs);

/* Vocabulary-node searches.  A keyframe or frame as
 * the BoW matchers read it: keypoints (angle; pt and octave for the
 * epipolar test), descriptors, the map-point state of every keypoint and
 * its DBoW2::FeatureVector (node id -> feature indices, std::map order) as
 * CSR arrays.  mp: 0 = no map point, 1 = map point, 2 = map point isBad().
 * Every feature index appears in at most one node (DBoW2 transform). */
typedef struct {
    const orbx_keypoint* keys;      /* [n] mvKeysUn (Frame side of
                                       SearchByBoW(KF, F): mvKeys)          */
    const uint8_t* desc;            /* [n][32] mDescriptors                  */
    int n;
    const uint8_t* mp;              /* [n] map-point state                   */
    int n_nodes;                    /* FeatureVector entries                 */
    const uint32_t* node_id;        /* [n_nodes] ascending                   */
    const int32_t* node_ptr;        /* [n_nodes + 1] offsets into feat_idx   */
    const int32_t* feat_idx;        /* feature indices of each node, as stored */
} orbx_bow_view;

/* ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>&)
 * (src/ORBmatcher.cc:155-283).  matches_f (out, F->n): the KF keypoint whose
 * map point was assigned to each F keypoint (vpMapPointMatches), or -1. */
int orbx_search_by_bow_frame(orbx_ctx* ctx, const orbx_bow_view* KF, const orbx_bow_view* F,
                             float nnratio, int check_ori, int32_t* matches_f, int* n_matches);
/* ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>&)
 * (src/ORBmatcher.cc:715-850).  matches12 (out, KF1->n): the KF2 keypoint
 * whose map point matched each KF1 keypoint (vpMatches12), or -1. */
int orbx_search_by_bow_kf(orbx_ctx* ctx, const orbx_bow_view* KF1, const orbx_bow_view* KF2,
                          float nnratio, int check_ori, int32_t* matches12, int* n_matches);
/* ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12, ...) (src/ORBmatcher.cc:
 * 852-1014).  F12: 3x3 row-major fundamental matrix (float, as cv::Mat);
 * sigma2_2: KF2's mvLevelSigma2 (nlevels entries).  matches12 (out, KF1->n):
 * vMatches12 (KF2 index or -1); vMatchedPairs are its non-negative entries
 * in KF1 order. */
int orbx_search_for_triangulation(orbx_ctx* ctx, const orbx_bow_view* KF1, const orbx_bow_view* KF2,
                                  const float* F12, const float* sigma2_2, int nlevels, int check_ori,
                                  int32_t* matches12, int* n_matches);
/* Batched forms for LocalMapping's per-neighbour loops: one keyframe KF1
 * against n keyframes KF2s[k] in one upload, one launch (a workgroup per
 * pair) and one readback; results as n separate calls would give.
 * SearchForTriangulation: CreateNewMapPoints (src/LocalMapping.cc:220-260,
 * F12s n x 9, sigma2_2s n x nlevels).  SearchByBoW(KF1, KF2): the loop
 * candidates of LoopClosing::ComputeSim3 (src/LoopClosing.cc:240).
 * matches12[k] (out, KF1->n) and n_matches[k] per pair. */
int orbx_search_for_triangulation_batch(orbx_ctx* ctx, const orbx_bow_view* KF1, int n,
                                        const orbx_bow_view* KF2s, const float* F12s,
                                        const float* sigma2_2s, int nlevels, int check_ori,
                                        int32_t* const* matches12, int* n_matches);
int orbx_search_by_bow_kf_batch(orbx_ctx* ctx, const orbx_bow_view* KF1, int n, const orbx_bow_view* KF2s,
                                float nnratio, int check_ori, int32_t* const* matches12, int* n_matches);

/* Keyframe projection searches.  Map points as they
 * read them, one entry per point (SoA). */
typedef struct {
    int n;
    const float* pos;        /* [n][3] GetWorldPos()                        */
    const float* normal;     /* [n][3] GetNormal() (Fuse; may be NULL else)  */
    const float* min_dist;   /* [n] GetMinDistanceInvariance()               */
    const float* max_dist;   /* [n] GetMaxDistanceInvariance()               */
    const uint8_t* desc;     /* [n][32] GetDescriptor()                      */
} orbx_mappoint_view;

/* ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>&, th) (src/ORBmatcher.cc:
 * 1016-1134; sim3 = 0, T = the keyframe's Tcw) and Fuse(KeyFrame*, Scw,
 * vector<MapPoint*>&, th) (:1136-1265; sim3 = 1, T = Scw), 4x4 row-major
 * float.  Computes the state-free part for every map point -- projection,
 * image / distance / viewing-angle gates, predicted level, and the best
 * keyframe keypoint within th * scale[level] at levels [pred - 1, pred]:
 * best_idx (-1 when gated out or no candidate) and best_dist.  The caller
 * replays the graph updates in map-point order (isBad / IsInKeyFrame /
 * already-found checks, bestDist <= TH_LOW, Replace or AddObservation),
 * which depend on the earlier points' updates. */
int orbx_fuse_candidates(orbx_ctx* ctx, const orbx_frame_view* KF, const float* cam,
                         const orbx_mappoint_view* mps, const float* T, int sim3, float th,
                         int32_t* best_idx, int32_t* best_dist);
/* Fuse candidates for n keyframes in one upload / launch / readback:
 * SearchInNeighbors' loop over the target keyframes (src/LocalMapping.cc:
 * 403-416), KFs[k] with camera cams[4k..], pose Ts[16k..] and map points
 * *mps[k] (views that are the same object are uploaded once: the loop fuses
 * the current keyframe's points into every neighbour).  The candidates are
 * state-free, so computing all of them before the caller replays the graph
 * updates neighbour by neighbour gives the sequential loop's result (a point
 * replaced or already in the keyframe is skipped at replay, as there). */
int orbx_fuse_candidates_batch(orbx_ctx* ctx, int n_kf, const orbx_frame_view* KFs, const float* cams,
                               const orbx_mappoint_view* const* mps, const float* Ts, int sim3, float th,
                               int32_t* const* best_idx, int32_t* const* best_dist);
/* orbx_fuse_candidates_batch against keyframes that stay in their extraction
 * slots: keyframe k is the frame in slots[k] (keypoints as the slot holds
 * them -- mvKeysUn after orbx_dev_undistort -- descriptors, the extractor's
 * scale pyramid), with image bounds bounds[4k..4k+3] (min_x, max_x, min_y,
 * max_y; Frame::ComputeImageBounds) or, bounds NULL, 0..w x 0..h.  Only the
 * map points, cameras and poses are uploaded; results as the batch form. */
int orbx_dev_fuse_candidates(orbx_ctx* ctx, int n_kf, const int* slots, const float* bounds, const float* cams,
                             const orbx_mappoint_view* const* mps, const float* Ts, int sim3, float th,
                             int32_t* const* best_idx, int32_t* const* best_dist);
/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
 * (src/ORBmatcher.cc:1267-1505).  mp1 / valid1: the map point of each KF1
 * keypoint (valid = pMP && !isBad()); mp2 / valid2 likewise for KF2.  T1w,
 * T2w: keyframe poses (4x4 row-major); R12 3x3 row-major, t12 3.  prior12
 * (in, KF1->n): -2 where vpMatches12[i] is NULL, else the KF2 index of that
 * map point (GetIndexInKeyFrame(pKF2), -1 if not observed).  new12 (out):
 * the KF2 keypoint whose map point this call assigns (vpMatches12[i1] =
 * vpMapPoints2[new12[i1]]), or -1.  cam: pKF1's fx, fy, cx, cy. */
int orbx_search_by_sim3(orbx_ctx* ctx, const orbx_frame_view* KF1, const orbx_frame_view* KF2,
                        const float* cam, const orbx_mappoint_view* mp1, const uint8_t* valid1,
                        const orbx_mappoint_view* mp2, const uint8_t* valid2, const float* T1w,
                        const float* T2w, float s12, const float* R12, const float* t12, float th,
                        const int32_t* prior12, int32_t* new12, int* n_found);
/* The same with both keyframes resident in their extraction slots (keypoints
 * as the slots hold them; bounds1 / bounds2: min_x, max_x, min_y, max_y, or
 * NULL for 0..w x 0..h; mp1 / valid1 / prior12 one entry per slot1 keypoint,
 * mp2 / valid2 per slot2 keypoint).  new12: cap >= slot1's keypoint count. */
int orbx_dev_search_by_sim3(orbx_ctx* ctx, int slot1, const float* bounds1, int slot2, const float* bounds2,
                            const float* cam, const orbx_mappoint_view* mp1, const uint8_t* valid1,
                            const orbx_mappoint_view* mp2, const uint8_t* valid2, const float* T1w,
                            const float* T2w, float s12, const float* R12, const float* t12, float th,
                            const int32_t* prior12, int32_t* new12, int cap, int* n_found);
/* ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const
 * vector<MapPoint*>& vpPoints, vector<MapPoint*>& vpMatched, int th)
 * (src/ORBmatcher.cc:286-407), loop closing.  mps: vpPoints; mp_skip:
 * pMP->isBad() or already in vpMatched (spAlreadyFound).  matched (in/out,
 * KF->n): vpMatched as an index into mps (any value >= 0 for an entry set by
 * the caller), -1 where NULL; the call writes the entries it assigns. */
int orbx_search_by_projection_kf_sim3(orbx_ctx* ctx, const orbx_frame_view* KF, const float* cam,
                                      const orbx_mappoint_view* mps, const uint8_t* mp_skip,
                                      const float* Scw, int th, int32_t* matched, int* n_matches);
/* The same against a keyframe resident in its extraction slot (keypoints as
 * the slot holds them, mvKeysUn after orbx_dev_undistort; bounds: min_x,
 * max_x, min_y, max_y, or NULL for 0..w x 0..h).  matched (in / out): cap >=
 * the slot's keypoint count entries, as above. */
int orbx_dev_search_by_projection_kf_sim3(orbx_ctx* ctx, int slot, const float* bounds, const float* cam,
                                          const orbx_mappoint_view* mps, const uint8_t* mp_skip, const float* Scw,
                                          int th, int32_t* matched, int cap, int* n_matches);
/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const
 * set<MapPoint*>& sAlreadyFound, float th, int ORBdist) (src/ORBmatcher.cc:
 * 1622-1746), relocalisation.  KF: pKF's keypoints (mvKeysUn); kf_mps: the
 * map point of each KF keypoint (pos, min_dist, desc); kf_valid: pMP &&
 * !isBad() && !sAlreadyFound.count(pMP).  F: CurrentFrame; f_assigned:
 * CurrentFrame.mvpMapPoints[i] != NULL; Tcw: CurrentFrame.mTcw (4x4
 * row-major); cam: CurrentFrame's fx, fy, cx, cy.  matches_f (out, F->n):
 * the KF keypoint whose map point this call assigns, or -1. */
int orbx_search_by_projection_frame_kf(orbx_ctx* ctx, const orbx_frame_view* F, const orbx_frame_view* KF,
                                       const float* cam, const orbx_mappoint_view* kf_mps,
                                       const uint8_t* kf_valid, const uint8_t* f_assigned,
                                       const float* Tcw, float th, int orb_dist, int check_ori,
                                       int32_t* matches_f, int* n_matches);
/* The same with the current frame in f_slot (bounds: min_x, max_x, min_y,
 * max_y, or NULL for 0..w x 0..h) and the candidate keyframe in kf_slot
 * (its keypoints from the slot; kf_mps / kf_valid: one entry per keyframe
 * keypoint), both as extraction / orbx_dev_undistort left them.
 * matches_f: cap >= the frame's keypoint count entries. */
int orbx_dev_search_by_projection_frame_kf(orbx_ctx* ctx, int f_slot, const float* f_bounds, int kf_slot,
                                           const float* cam, const orbx_mappoint_view* kf_mps,
                                           const uint8_t* kf_valid, const uint8_t* f_assigned, const float* Tcw,
                                           float th, int orb_dist, int check_ori, int32_t* matches_f, int cap,
                                           int* n_matches);
/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:185-250) for
 * n_mp map points at once: point m's observed descriptors (non-bad
 * keyframes, observation order) are rows obs_ptr[m] .. obs_ptr[m+1]-1 of
 * desc.  best (out): the row (relative to obs_ptr[m]) with the least median
 * distance to the others, -1 for a point without descriptors. */
int orbx_distinctive_descriptors(orbx_ctx* ctx, int n_mp, const int32_t* obs_ptr,
                                 const uint8_t* desc, int32_t* best);

/* Frame construction.  Frame::UndistortKeyPoints
 * (src/Frame.cc:288-318): cv::undistortPoints with P = K, K = (fx, fy, cx,
 * cy), dist = (k1, k2, p1, p2, k3) (mDistCoef; k3 = 0 for 4 coefficients).
 * A zero k1 copies the keypoints (:290-294), as the reference does. */
int orbx_undistort_keypoints(orbx_ctx* ctx, int n, const orbx_keypoint* keys, const float* K,
                             const float* dist, orbx_keypoint* keys_un);
/* Frame::ComputeImageBounds (src/Frame.cc:320-348): bounds = mnMinX,
 * mnMaxX, mnMinY, mnMaxY for a w x h image (host only, four points). */
int orbx_compute_image_bounds(int w, int h, const float* K, const float* dist, float* bounds);
/* Device-resident form: undistort the keypoints of extracted slots
 * [first, first+count) in place (after orbx_dev_extract, before matching). */
int orbx_dev_undistort(orbx_ctx* ctx, int first, int count, const float* K, const float* dist);

/* DBoW2 vocabulary: the tree as
 * TemplatedVocabulary::loadFromTextFile builds it (Thirdparty/DBoW2/DBoW2/
 * TemplatedVocabulary.h:1338-1420) -- node 0 the root, node i (1..n-1) a
 * child of parent[i] (children in increasing id order), word ids given to
 * the nodes flagged is_leaf in id order, a 32-byte descriptor and a weight
 * (idf) per node.  Kept in HBM for the vocabulary's lifetime. */
typedef struct orbx_vocab orbx_vocab;
int orbx_vocab_create(orbx_ctx* ctx, int k, int L, int n_nodes, const int32_t* parent,
                      const uint8_t* is_leaf, const uint8_t* desc, const double* weight,
                      orbx_vocab** out);
void orbx_vocab_destroy(orbx_vocab* voc);
int orbx_vocab_n_words(const orbx_vocab* voc);
/* TemplatedVocabulary::transform(features, BowVector&, FeatureVector&,
 * levelsup) (:1127-1259) as Frame::ComputeBoW calls it (src/Frame.cc:
 * 279-286, levelsup 4), TF-IDF weighting with L1 scoring (ORBvoc.txt's).
 * The tree descent of the n descriptors runs on the device; per feature:
 * word_id, weight and the level-(L - levelsup) node (node_id, -1 if the
 * descent ended above that level).  BowVector: n_words (word, value) pairs,
 * words ascending, values L1-normalised.  FeatureVector: n_fv_nodes node
 * ids ascending with CSR offsets fv_ptr (n_fv_nodes + 1) into fv_feat.
 * Stopped words (weight 0) are left out of both.  Capacities: n entries
 * (fv_ptr: n + 1). */
int orbx_vocab_transform(orbx_ctx* ctx, const orbx_vocab* voc, int n, const uint8_t* desc,
                         int levelsup, int32_t* word_id, double* weight, int32_t* node_id,
                         uint32_t* bow_words, double* bow_values, int* n_words,
                         uint32_t* fv_nodes, int32_t* fv_ptr, int32_t* fv_feat, int* n_fv_nodes);

/* Device-resident form for extracted slots: Frame::ComputeBoW (src/Frame.cc:
 * 279-286) of slots [first, first+count) -- the descent of every extracted
 * descriptor and the slot's BowVector / FeatureVector built on the device,
 * kept in HBM until the slot is extracted again (async, context stream).
 * Frames of up to 4096 features (ORBX_ERR_UNSUPPORTED above). */
int orbx_dev_compute_bow(orbx_ctx* ctx, const orbx_vocab* voc, int first, int count, int levelsup);
/* Read one slot's BoW (after orbx_dev_compute_bow; syncs), the arrays of
 * orbx_vocab_transform with the same meaning.  Any output may be NULL;
 * cap >= the slot's feature count (ORBX_ERR_CAPACITY otherwise). */
int orbx_dev_read_bow(orbx_ctx* ctx, int slot, int cap, int32_t* word_id, double* weight, int32_t* node_id,
                      uint32_t* bow_words, double* bow_values, int* n_words, uint32_t* fv_nodes,
                      int32_t* fv_ptr, int32_t* fv_feat, int* n_fv_nodes);
/* Tracking::Relocalisation's matching loop (src/Tracking.cc:904-925):
 * ORBmatcher::SearchByBoW(pKF, F) (src/ORBmatcher.cc:155-283) of n
 * candidate keyframes against the frame in `slot`, its keypoints,
 * descriptors and FeatureVector read where orbx_dev_extract /
 * orbx_dev_compute_bow left them.  matches_f[k] (cap >= nfeatures entries):
 * per frame keypoint the KF keypoint index or -1, as orbx_search_by_bow_frame. */
int orbx_dev_search_by_bow(orbx_ctx* ctx, int slot, int n, const orbx_bow_view* KFs, float nnratio,
                           int check_ori, int32_t* const* matches_f, int cap, int* n_matches);
/* The keyframe-pair searches between device-resident frames, the keyframe
 * in slot1 against those in slots2[0, n) (keypoints as the slots hold them,
 * mvKeysUn after orbx_dev_undistort; FeatureVectors from
 * orbx_dev_compute_bow on every slot named): SearchByBoW(KF1, KF2)
 * (src/ORBmatcher.cc:715-850) as LoopClosing::ComputeSim3's candidate loop
 * (src/LoopClosing.cc:240) runs it, and SearchForTriangulation (:852-1014)
 * as LocalMapping::CreateNewMapPoints' neighbour loop (src/LocalMapping.cc:
 * 220-260) does (F12s n x 9, sigma2_2s n x nlevels, nlevels the
 * extractor's).  Only the map-point states travel: mp1 and mp2s[k] hold one
 * state per keypoint of the slot (0 none, 1 map point, 2 isBad()).
 * matches12[k] (cap >= nfeatures entries): per slot1 keypoint the slots2[k]
 * keypoint or -1, as the host-array forms. */
int orbx_dev_search_by_bow_kf(orbx_ctx* ctx, int slot1, const uint8_t* mp1, int n, const int* slots2,
                              const uint8_t* const* mp2s, float nnratio, int check_ori,
                              int32_t* const* matches12, int cap, int* n_matches);
int orbx_dev_search_for_triangulation(orbx_ctx* ctx, int slot1, const uint8_t* mp1, int n, const int* slots2,
                                      const uint8_t* const* mp2s, const float* F12s, const float* sigma2_2s,
                                      int nlevels, int check_ori, int32_t* const* matches12, int cap,
                                      int* n_matches);

/* ------------------------------------------------------------------------ */
/* C. Local bundle adjustment                                                */
/* ------------------------------------------------------------------------ */

/* SoA local-BA problem (Optimizer::LocalBundleAdjustment, src/Optimizer.cc:
 * 287-536).  Poses are SE3Quat (g2o se3quat.h) as unit quaternion (x,y,z,w)
 * + translation; ids are the g2o vertex ids (KF mnId; points mnId+maxKFid+1)
 * which fix the Hessian ordering (sparse_optimizer.cpp:166-190, 482-487).
 * Edges are EdgeSE3ProjectXYZ in insertion order (points in local-list order,
 * observations in the caller's map<KeyFrame*,size_t> order). */
typedef struct {
    int n_poses, n_points, n_edges;
    double* pose_q;             /* [n_poses][4] x,y,z,w   (in/out)           */
    double* pose_t;             /* [n_poses][3]           (in/out)           */
    const uint8_t* pose_fixed;  /* [n_poses]                                  */
    const int64_t* pose_id;     /* [n_poses] g2o vertex id                    */
    const double* pose_cam;     /* [n_poses][4] fx, fy, cx, cy                */
    double* points;             /* [n_points][3]          (in/out)           */
    const int64_t* point_id;    /* [n_points]                                 */
    const int32_t* point_nobs;  /* [n_points] MapPoint::Observations() at call*/
    const int32_t* edge_point;  /* [n_edges] index into points                */
    const int32_t* edge_pose;   /* [n_edges] index into poses                 */
    const double* edge_obs;     /* [n_edges][2] undistorted keypoint          */
    const double* edge_inv_sigma2; /* [n_edges] information = I * invSigma2   */
    double huber_delta;         /* sqrt(5.991) as float, widened              */
    double chi2_threshold;      /* 5.991                                      */
} orbx_ba_problem;

typedef struct {
    int iterations[2];          /* LM iterations executed per optimize() call */
    int levenberg_trials[2];    /* inner LM trials summed                     */
    double chi2_initial[2];     /* robust chi2 at the first linearisation     */
    double chi2_final[2];       /* robust chi2 of the accepted state          */
    int n_outliers[2];          /* edges erased by each outlier pass          */
    int not_posdef;             /* Cholesky failures (step rejected)          */
} orbx_ba_stats;

/* Runs optimize(iters0), the first outlier pass (edge erased and removed from
 * the graph), optimize(iters1) and the second outlier pass.  edge_status
 * (out, n_edges): 0 inlier, 1 erased in pass 1, 2 erased in pass 2.
 * point_bad (out, n_points): MapPoint became bad through EraseObservation.
 * abort: polled between LM iterations (mbAbortBA; may be NULL).  g2o also
 * tests its stop flag between the trials of an iteration (levenberg.cpp:149);
 * here an iteration that has started runs its trials to the end, so a flag
 * raised mid-iteration stops the solve at the same iteration boundary but
 * possibly after more trials.
 * One problem runs over several workgroups when it qualifies
 * (orbx_lba_set_workgroups), with the same result bits. */
int orbx_lba_solve(orbx_ctx* ctx, orbx_ba_problem* p, int iters0, int iters1,
                   const volatile uint8_t* abort, uint8_t* edge_status,
                   uint8_t* point_bad, orbx_ba_stats* stats);

/* Workgroups that share one problem (orbx_lba_solve, and batches of one):
 * 0 (default) = automatic (one per 32 points, at most 64, when the reduced
 * system fits a workgroup's LDS); 1 = one workgroup, as in a batch; n > 1 =
 * n workgroups.  Every setting gives the same bits (k_lba_split sums in the
 * single-workgroup kernel's order); more workgroups cut the latency of the
 * call LocalMapping makes once per keyframe (src/LocalMapping.cc:83).
 * The workgroups of one problem meet at grid barriers, so they must all be
 * resident at once: the count is capped at what the device holds of that
 * kernel (occupancy x CUs: a partitioned device, or a setting of 256, gets
 * fewer), and a solve whose barrier still times out (another context's
 * kernels holding the CUs) is run again on one workgroup -- same bits,
 * longer call.  (A cooperative launch, available through
 * orbx_debug_lba_split, gives the same bits but measured to delay other
 * contexts' calls beside it.) */
int orbx_lba_set_workgroups(orbx_ctx* ctx, int n);
int orbx_lba_get_workgroups(const orbx_ctx* ctx);
/* Workgroups the last local-BA launch of ctx ran with (after the cap and any
 * one-workgroup re-run). */
int orbx_lba_last_workgroups(const orbx_ctx* ctx);
/* Test hooks of that residency handling (fail: the next n split launches
 * see a barrier timeout; fallback 0: no re-run, ORBX_ERR_HIP with the
 * caller's arrays untouched; cap > 0: capacity capped; coop -1 / 0 / 1:
 * the device's choice / plain (default) / cooperative launch; arguments
 * below those ranges leave the setting unchanged). */
int orbx_debug_lba_split(orbx_ctx* ctx, int fail, int fallback, int cap, int coop);

/* Batched throughput form: P independent problems, one workgroup each.
 * aborts: NULL, or P flags (entries may be NULL), each polled between LM
 * iterations like orbx_lba_solve's: problem i stops its optimize() calls
 * when *aborts[i] is set (its own LocalMapping's mbAbortBA,
 * src/LocalMapping.cc:83, :125), the others continue.  With flags each
 * iteration is a launch and the call waits for it to poll; without flags
 * each optimize() pass is one launch of all its iterations and nothing
 * waits.  Results are the same bits either way. */
int orbx_lba_solve_batch(orbx_ctx* ctx, int P, orbx_ba_problem* problems,
                         int iters0, int iters1, const volatile uint8_t* const* aborts,
                         uint8_t* const* edge_status, uint8_t* const* point_bad,
                         orbx_ba_stats* stats);
/* Device-resident form of the batch (bench/tests; the pose API's shape):
 * stage P problems in HBM once (validated as orbx_lba_solve_batch does),
 * run both optimize() passes from the staged state any number of times
 * (asynchronous, on the context stream; kernel timers "lba_iter" /
 * "lba_outliers"), fetch the last run's poses, points, flags and statistics
 * into problems laid out like the staged ones (ORBX_ERR_ARG before a run or
 * on a size mismatch).  orbx_lba_run's aborts are orbx_lba_solve_batch's
 * (NULL: asynchronous; with flags the call returns when the run is done). */
int orbx_lba_stage(orbx_ctx* ctx, int P, const orbx_ba_problem* problems);
int orbx_lba_run(orbx_ctx* ctx, int iters0, int iters1, const volatile uint8_t* const* aborts);
int orbx_lba_fetch(orbx_ctx* ctx, orbx_ba_problem* problems, uint8_t* const* edge_status,
                   uint8_t* const* point_bad, orbx_ba_stats* stats);

/* ------------------------------------------------------------------------ */
/* D. Motion-only pose optimisation                   */
/* ------------------------------------------------------------------------ */

/* One Frame as Optimizer::PoseOptimization(Frame*) reads and writes it
 * (src/Optimizer.cc:154-285).  Keypoints with a map point become
 * EdgeSE3ProjectXYZ edges to fixed points (information = I *
 * mvInvLevelSigma2[octave], Huber delta sqrt(5.991)); four robust rounds
 * (chi2 9.210 / 7.378 / 5.991 / 5.991, LM iterations 10 / 10 / 7 / 5)
 * classify outliers. */
typedef struct {
    int n;                           /* N = mvpMapPoints.size() (= keypoints)    */
    const float* kp_un;              /* [n][2] mvKeysUn[i].pt                    */
    const int32_t* octave;           /* [n] mvKeysUn[i].octave                   */
    const float* inv_level_sigma2;   /* [nlevels] mvInvLevelSigma2               */
    int nlevels;
    const uint8_t* has_mp;           /* [n] mvpMapPoints[i] != NULL              */
    const float* mp_xyz;             /* [n][3] mvpMapPoints[i]->GetWorldPos()    */
    float cam[4];                    /* fx, fy, cx, cy                           */
    float Tcw[16];                   /* mTcw, row-major 4x4 (in/out)             */
    uint8_t* outlier;                /* [n] mvbOutlier (in/out: entries with a map
                                        point are written, the rest untouched)   */
} orbx_pose_frame;

typedef struct {
    int rounds;                      /* robust rounds run (stops after round 0
                                        when the frame has < 10 edges)           */
    int iterations[4];               /* LM iterations per round                  */
    int levenberg_trials[4];         /* inner LM trials per round                */
    int n_bad[4];                    /* outliers after each round                */
    double chi2_final[4];            /* robust chi2 of the accepted state        */
    int not_posdef;                  /* LDLT failures (step rejected)            */
} orbx_pose_stats;

/* Replaces Optimizer::PoseOptimization(Frame*): updates f->Tcw and
 * f->outlier, *n_inliers = the function's return value
 * (nInitialCorrespondences - nBad).  stats may be NULL. */
int orbx_pose_optimization(orbx_ctx* ctx, orbx_pose_frame* f, int* n_inliers,
                           orbx_pose_stats* stats);
/* Batched form: P independent frames (one wavefront each, one launch). */
int orbx_pose_optimization_batch(orbx_ctx* ctx, int P, orbx_pose_frame* frames,
                                 int32_t* n_inliers, orbx_pose_stats* stats);
/* Device-resident form of the batch (bench/tests): stage P frames in HBM
 * once, run the optimisation from the staged initial poses any number of
 * times (asynchronous, on the context stream; kernel timer "pose"), fetch
 * the results of the last run into the frames' Tcw / outlier. */
int orbx_pose_stage(orbx_ctx* ctx, int P, const orbx_pose_frame* frames);
int orbx_pose_run(orbx_ctx* ctx);
int orbx_pose_fetch(orbx_ctx* ctx, orbx_pose_frame* frames, int32_t* n_inliers,
                    orbx_pose_stats* stats);
/* Summation mode of the pose optimisation (default 1).  1: every chi2 / H /
 * b sum runs sequentially in g2o's active-edge order (the edge terms are
 * computed in parallel, accumulated edge by edge), so the whole LM
 * trajectory -- accept / reject of every trial, lambda, iterations -- and
 * the returned pose are the sequential reference's bit for bit, for every
 * batch size.  0 (opt-in, faster: about 1.03x one call, 1.4x a batch): each
 * wavefront sums its edges' terms lane-strided and then through a fixed DPP
 * tree -- deterministic, but in another order than g2o, so LM steps decided
 * on rounding noise (a converged pose restarted in a later robust round) may
 * count differently: poses within 1e-5, and the result of a frame may differ
 * between a lone call (a workgroup per frame) and a batch (a wavefront per
 * frame).  Takes effect at the next orbx_pose_run.  Returns ORBX_ERR_ARG for
 * a null context or a mode outside 0..1; orbx_pose_get_exact returns the
 * mode (ORBX_ERR_ARG for NULL). */
int orbx_pose_set_exact(orbx_ctx* ctx, int exact);
int orbx_pose_get_exact(const orbx_ctx* ctx);

/* Library identification. */
const char* orbx_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ORBX_H */
