/*
 * orbhip.h — C-ABI of liborbhip.so, the MI355X (gfx950) ORB front-end + BA back-end.
 *
 * Drop-in boundary for the hot path of EricPedley/ORB_SLAM3_ROS2.
 * Each entry point names the reference interface it replaces:
 *   R:src/imu_mono_realsense.cpp:337   System::TrackMonocular -> Frame(mono) -> Frame::ExtractORB
 *   U:src/Frame.cc::Frame::ExtractORB  calls ORBextractor::operator()(im, Mat(), kps, desc, {0,1000})
 *   U:src/ORBextractor.cc::ORBextractor::operator()          -> orbhip_extract / orbhip_extract_batch_device
 *   U:src/ORBextractor.cc::ORBextractor::ORBextractor(...)   -> orbhip_create (orbhip_orb_params)
 *   U:src/ORBmatcher.cc::ORBmatcher::DescriptorDistance      -> orbhip_descriptor_distance
 *   U:src/ORBmatcher.cc  best/second + ratio + TH_LOW + rotation histogram -> orbhip_match_bf*
 *   U:src/Optimizer.cc::Optimizer::LocalBundleAdjustment / BundleAdjustment -> orbhip_ba_solve
 *
 * Conventions:
 *  - Plain pointers and sizes only; no C++ types, no exceptions cross this ABI.
 *  - The caller owns every host buffer. A context owns its device memory, pinned
 *    staging and one HIP stream (used by the host-buffer entry points). The *_device entry
 *    points run on the caller's `stream` argument; NULL is the HIP null stream. One context
 *    per calling thread; a context is not re-entrant; distinct contexts are safe to use
 *    concurrently.
 *  - Status: 0 ok, < 0 error (orbhip_status).
 *  - Parity contract: keypoints/descriptors bit-exact with the CPU restatement in
 *    oracle/ (the reference's own path cannot be built here: SURVEY.md §0, §8c).
 */
#ifndef ORBHIP_H
#define ORBHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBHIP_ABI_VERSION 1

typedef enum {
    ORBHIP_OK = 0,
    ORBHIP_ERR_ARG = -1,          /* bad argument (null pointer, bad size, ...) */
    ORBHIP_ERR_CAPACITY = -2,     /* caller buffer too small; *n_out holds the required count */
    ORBHIP_ERR_DEVICE = -3,       /* HIP runtime failure / no device */
    ORBHIP_ERR_NOT_PD = -4,       /* reduced camera system not positive definite */
    ORBHIP_ERR_UNSUPPORTED = -5,  /* configuration outside the supported envelope */
    ORBHIP_ERR_EMPTY = -6,        /* empty image: ORBextractor::operator() returns -1 */
    ORBHIP_ERR_TIMEOUT = -7       /* a persistent-solver hand-off timed out (ORBHIP_DAG_RERUN=0) */
} orbhip_status;

typedef struct orbhip_ctx orbhip_ctx;

/* ORBextractor ctor arguments; YAML keys ORBextractor.{nFeatures, scaleFactor, nLevels,
 * iniThFAST, minThFAST} (R:config/Monocular/MilkV.yaml:42-55). */
typedef struct {
    int32_t n_features;
    float scale_factor;
    int32_t n_levels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
} orbhip_orb_params;

/* cv::KeyPoint as produced by ORBextractor (class_id is always -1 there, omitted). */
typedef struct {
    float x, y;       /* level-0 pixel coordinates (pt *= mvScaleFactor[octave]) */
    float size;       /* (int)(31 * mvScaleFactor[octave]) */
    float angle;      /* IC_Angle, degrees [0, 360) */
    float response;   /* FAST score */
    int32_t octave;   /* pyramid level */
} orbhip_kp;

/* ---- context ------------------------------------------------------------------- */
int orbhip_abi_version(void);
/* device: HIP ordinal, or < 0 for the calling thread's current device (hipGetDevice: one process
   per GPU). params may be NULL -> ORB_SLAM3 defaults (1000, 1.2, 8, 20, 7). */
int orbhip_create(orbhip_ctx** out, int device, const orbhip_orb_params* params);
int orbhip_destroy(orbhip_ctx* ctx);
/* Per-level tables of the ORBextractor ctor: mvScaleFactor, mnFeaturesPerLevel. */
int orbhip_level_info(orbhip_ctx* ctx, int w, int h, int32_t* level_w, int32_t* level_h,
                      int32_t* n_feat, float* scale);
/* Max keypoints one frame can yield for this context at size w x h (cap for outputs). */
int orbhip_max_keypoints(orbhip_ctx* ctx, int w, int h);

/* ---- ORB extraction --------------------------------------------------------------
 * orbhip_extract: ORBextractor::operator()(img, Mat(), kps, desc, {lap0, lap1}).
 * Host image (CV_8UC1, row stride in bytes), host outputs (cap entries). *mono_index
 * receives the return value of operator() (kps with lap0 <= x <= lap1 fill the array
 * from the end, the rest from the front). Empty image -> ORBHIP_ERR_EMPTY (reference: -1). */
int orbhip_extract(orbhip_ctx* ctx, const uint8_t* img, int w, int h, int stride, int lap0, int lap1,
                   orbhip_kp* kps, uint8_t* desc32, int cap, int* n_out, int* mono_index);

/* Batched, fully device-resident form (torch-ROCm ingest, benchmarks). d_imgs: B frames,
 * frame f at d_imgs + f*frame_stride, rows `stride` bytes apart. Outputs per frame f:
 * d_kps[f*cap ...], d_desc[(f*cap ...)*32], d_n[f], d_mono[f]. Asynchronous on `stream`
 * (hipStream_t; NULL = the HIP null stream, as in every HIP API — torch's default stream). */
int orbhip_extract_batch_device(orbhip_ctx* ctx, const uint8_t* d_imgs, int B, int w, int h, int stride,
                                int64_t frame_stride, int lap0, int lap1, orbhip_kp* d_kps, uint8_t* d_desc,
                                int cap, int32_t* d_n, int32_t* d_mono, void* stream);

/* ---- distorted pinhole camera -----------------------------------
 * U:src/CameraModels/Pinhole (fx fy cx cy) + U:src/Frame.cc mDistCoef (k1 k2 p1 p2 [k3]), as the
 * node's camera file gives them (R:config/Monocular/MilkV.yaml:10-25). k1 == 0 means no
 * distortion (the reference's test: mDistCoef.at<float>(0) == 0). */
typedef struct orbhip_pinhole {
    float fx, fy, cx, cy;
    float k1, k2, p1, p2, k3;
} orbhip_pinhole;

/* U:src/Frame.cc::Frame::UndistortKeyPoints: mvKeysUn from mvKeys through cv::undistortPoints
 * (OpenCV 4.5.4, 5 fixed-point rounds, fp64), bit-exact. Host buffers; out may alias kps.
 * k1 == 0: out = kps. Replaces the cv::undistortPoints call inside Frame(mono) after ExtractORB. */
int orbhip_undistort_keypoints(orbhip_ctx* ctx, const orbhip_pinhole* cam, const orbhip_kp* kps, int n,
                               orbhip_kp* out);
/* The same on the device over an extraction batch: d_kps[b*cap + i] for i < d_n[b] -> d_out
 * (may alias). Asynchronous on `stream` (NULL = the HIP null stream). */
int orbhip_undistort_keypoints_device(orbhip_ctx* ctx, const orbhip_pinhole* cam, const orbhip_kp* d_kps,
                                      const int32_t* d_n, int B, int cap, orbhip_kp* d_out, void* stream);
/* U:src/Frame.cc::Frame::ComputeImageBounds: bounds = {mnMinX, mnMaxX, mnMinY, mnMaxY} from the
 * undistorted image corners ({0, cols, 0, rows} when k1 == 0). These bounds define the 64 x 48
 * frame grid the projection / initialisation searches use (orbhip_frame.min_x ...). */
int orbhip_image_bounds(orbhip_ctx* ctx, const orbhip_pinhole* cam, int cols, int rows, float bounds[4]);

/* ---- ingest (a23) -------------------------------------------------------------------
 * cv_bridge::toCvShare(bgr8 msg, MONO8) -> cvtColor(COLOR_BGR2GRAY) (R:src/imu_mono_realsense.cpp:298)
 * on the device, bit-exact: Y = (B*1868 + G*9617 + R*4899 + 2^13) >> 14. B frames of w x h
 * BGR (3 bytes/px, rows `src_stride` bytes apart, frames `src_fstride` apart) -> u8 gray
 * (rows `dst_stride`, frames `dst_fstride`), ready for orbhip_extract_batch_device.
 * Asynchronous on `stream` (NULL = the HIP null stream). */
int orbhip_bgr_to_gray_device(orbhip_ctx* ctx, const uint8_t* d_bgr, int B, int w, int h, int src_stride,
                              int64_t src_fstride, uint8_t* d_gray, int dst_stride, int64_t dst_fstride,
                              void* stream);

/* ---- Hamming matching ------------------------------------------------------------- */
/* ORBmatcher::DescriptorDistance (host helper, popcount of xor over 32 bytes). */
int orbhip_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Brute-force top-2 over the whole train set (order-free: no greedy vnMatches21 pass),
 * accept best <= th_low && (float)best < ratio*(float)second, then (if check_orientation)
 * the rotation-histogram filter (HISTO_LENGTH 30, ComputeThreeMaxima). best/second start at
 * 256 (SearchByBoW). match[i] = train index or -1. Host buffers. Returns #matches >= 0. */
int orbhip_match_bf(orbhip_ctx* ctx, const uint8_t* q_desc, const float* q_angle, int nq,
                    const uint8_t* t_desc, const float* t_angle, int nt, int th_low, float ratio,
                    int check_orientation, int32_t* match, int32_t* best_d, int32_t* second_d);

/* Device form over extractor outputs: pairs (frame p, frame p+1) for p in [0, B-1), each
 * frame's kps/desc at f*cap as written by orbhip_extract_batch_device. Outputs at p*cap;
 * d_nmatch[p] = #matches. Asynchronous. */
int orbhip_match_pairs_device(orbhip_ctx* ctx, const orbhip_kp* d_kps, const uint8_t* d_desc,
                              const int32_t* d_n, int B, int cap, int th_low, float ratio,
                              int check_orientation, int32_t* d_match, int32_t* d_best,
                              int32_t* d_second, int32_t* d_nmatch, void* stream);

/* Device form over two arbitrary frames (e.g. frame t vs t-1 in a 2-slot ring): query
 * set (d_q_kps/d_q_desc, count *d_nq) vs train set (d_t_kps/d_t_desc, count *d_nt), both laid
 * out like one frame of orbhip_extract_batch_device (cap entries). Outputs (cap entries) and
 * *d_nmatch on the device. Asynchronous; no host synchronisation. */
int orbhip_match_frames_device(orbhip_ctx* ctx, const orbhip_kp* d_q_kps, const uint8_t* d_q_desc,
                               const int32_t* d_nq, const orbhip_kp* d_t_kps, const uint8_t* d_t_desc,
                               const int32_t* d_nt, int cap, int th_low, float ratio, int check_orientation,
                               int32_t* d_match, int32_t* d_best, int32_t* d_second, int32_t* d_nmatch,
                               void* stream);

/* ---- camera front-end stream -------------------------------------------------------
 * One camera's frames, as Tracking receives them (Frame ctor -> ExtractORB, then matching
 * against the last frame), pipelined on the device: frame k is extracted at batch 1 on
 * context k % frames_in_flight (each context = its own HIP stream / hardware queue) into
 * output slot k % slots (slots = 2 * frames_in_flight, 2 for 1), then the previous frame
 * (queries) is matched to it (train) as orbhip_match_frames_device does with (th_low, ratio,
 * check_orientation). Cross-frame hand-offs are device events; push never blocks the host.
 * Same kernels and results as the one-frame calls. Frame 0 has no match (*nmatch = -1).
 *   push: d_img = device u8 frame (w x h, rows `stride` bytes apart), vLappingArea
 *         {lap0, lap1}; returns the slot index (>= 0) or an error (< 0). The caller keeps
 *         d_img unchanged until the frame completes.
 *   view: device pointers of a slot's outputs (valid until the slot is reused, `slots`
 *         pushes later); frame = number of the frame held (-1 none).
 *   wait: the frame in `slot` complete: host-blocking (stream NULL) or stream-ordered. With
 *         one frame in flight the stream is one in-order HIP stream and push records no event:
 *         the first wait that needs one records it then (covering every frame pushed so far).
 *   context: context j (0 <= j < frames_in_flight), e.g. for orbhip_profile_stage. */
typedef struct orbhip_frontend orbhip_frontend;
typedef struct {
    int64_t frame;
    int32_t cap, slots;
    orbhip_kp* kps;          /* cap entries */
    uint8_t* desc;           /* cap x 32 */
    int32_t* n;              /* 1 */
    int32_t* mono;           /* 1: operator()'s return value */
    int32_t* match;          /* cap: previous frame's keypoint i -> this frame's index or -1 */
    int32_t* best;           /* cap */
    int32_t* second;         /* cap */
    int32_t* nmatch;         /* 1 */
} orbhip_frontend_slot;
int orbhip_frontend_create(orbhip_frontend** out, int device, const orbhip_orb_params* params, int w, int h,
                           int frames_in_flight, int th_low, float ratio, int check_orientation);
int orbhip_frontend_destroy(orbhip_frontend* fe);
int orbhip_frontend_push(orbhip_frontend* fe, const uint8_t* d_img, int stride, int lap0, int lap1);
int orbhip_frontend_view(orbhip_frontend* fe, int slot, orbhip_frontend_slot* out);
int orbhip_frontend_wait(orbhip_frontend* fe, int slot, void* stream);
int orbhip_frontend_context(orbhip_frontend* fe, int j, orbhip_ctx** out);

/* ---- diagnostics: live kernel timing ----------------------------------------------
 * orbhip_profile_stage selects ONE stage whose launches are bracketed by hipEvents on the
 * stream they run on (0 off, 1 pyramid resize, 2 FAST cells, 3 octree, 4 orientation +
 * descriptor, 5 Hamming top-2, 6 rotation filter). orbhip_profile_collect synchronises and
 * returns the summed duration (ms) and the number of bracketed launches, then resets. The one-launch
 * pyramid (k_pyr_cone) and the octree also time themselves on the device (first workgroup start to
 * last workgroup end, s_memrealtime: the span rocprofv3's kernel trace reports); their stages
 * return that span when every launch recorded it, the event pairs otherwise. */
int orbhip_profile_stage(orbhip_ctx* ctx, int stage);
int orbhip_profile_collect(orbhip_ctx* ctx, double* total_ms, int32_t* count);

/* With ORBHIP_GRAPH=1 in the environment, repeated calls of orbhip_extract_batch_device /
 * orbhip_match_*_device with identical arguments on a non-NULL stream are replayed from a
 * captured hipGraph (from the second such call on: one hipGraphLaunch instead of the kernel
 * launches). Same kernels, same results. Off by default (the replay adds device time on this
 * runtime); always direct while a profile stage is selected or on a capturing stream.
 * Returns the number of launch graphs the context holds. */
int orbhip_launch_graphs(orbhip_ctx* ctx);

/* ---- bundle adjustment ------------------------------------------------------------
 * Optimizer::LocalBundleAdjustment / BundleAdjustment problem (SoA, host memory).
 * Poses are Tcw = (q, t): q = unit quaternion (x, y, z, w), t translation, float, as
 * Sophus::SE3f stores them. Edges are EdgeSE3ProjectXYZ mono observations. */
typedef struct {
    int32_t n_poses, n_points, n_edges;
    const float* pose_q;        /* n_poses x 4 (x,y,z,w) */
    const float* pose_t;        /* n_poses x 3 */
    const uint8_t* pose_fixed;  /* n_poses (1 = fixed vertex) */
    const float* points;        /* n_points x 3 (world) */
    const int32_t* edge_pose;   /* n_edges */
    const int32_t* edge_point;  /* n_edges */
    const float* edge_uv;       /* n_edges x 2 (undistorted keypoint) */
    const int32_t* edge_octave; /* n_edges */
    const float* inv_sigma2;    /* per octave: information = I * invSigma2[octave] */
    int32_t n_octaves;
    float fx, fy, cx, cy;       /* Pinhole mvParameters (float) */
    float huber_delta;          /* sqrt(5.991) for LBA; <= 0 disables the robust kernel */
    int32_t iterations;         /* optimize(n): 10 for LBA */
    int32_t early_stop;         /* vendored-g2o chi2 stall stop, 0 = off */
} orbhip_ba_problem;

typedef struct {
    float* pose_q;              /* n_poses x 4 out (fixed poses copied through) */
    float* pose_t;              /* n_poses x 3 out */
    float* points;              /* n_points x 3 out */
    float* edge_chi2;           /* n_edges out: e->chi2() after optimize (for the 5.991 erase) */
    uint8_t* edge_depth_ok;     /* n_edges out: e->isDepthPositive() */
    double initial_chi2;        /* activeRobustChi2 before iteration 0 */
    double final_chi2;          /* activeRobustChi2 of the accepted state */
    int32_t iterations_done;    /* SparseOptimizer::optimize return value */
    int32_t lm_trials;          /* total Levenberg trials */
} orbhip_ba_result;

/* stop_flag: polled between LM iterations/trials (LocalMapping mbAbortBA -> g2o
 * setForceStopFlag). May be NULL. */
int orbhip_ba_solve(orbhip_ctx* ctx, const orbhip_ba_problem* prob, orbhip_ba_result* res,
                    const volatile int* stop_flag);

/* Concurrency: LocalMapping's LBA and LoopClosing's GBA (R:src/imu_mono_realsense.cpp:99-100
 * spawns both threads) may solve at the same time on two contexts. The persistent Cholesky
 * (one launch owning every CU) is serialised per device across contexts and streams, so two
 * solves never hold parts of the chip at once. A hand-off that still times out (its bounded spin,
 * ORBHIP_DAG_SPIN_MAX polls, runs out) never becomes a silently rejected LM trial: the solve is run
 * again on the non-persistent solvers (same g2o schedule), or, with ORBHIP_DAG_RERUN=0 in the
 * environment, returns ORBHIP_ERR_TIMEOUT.
 * orbhip_ba_stats: out[0] persistent solves launched on the context's device (every context),
 * out[1] of them launched after waiting for another stream's solve, out[2] hand-off timeouts this
 * context saw, out[3] solves it re-ran. */
int orbhip_ba_stats(orbhip_ctx* ctx, int64_t out[4]);

/* B independent problems solved together (SURVEY.md §8e replicas: concurrent maps / agents,
 * or a batch of local windows). Each problem follows its own exact LM schedule; all share the
 * kernel launches of a round. probs / res: arrays of B structs. */
int orbhip_ba_solve_batch(orbhip_ctx* ctx, const orbhip_ba_problem* probs, int B, orbhip_ba_result* res,
                          const volatile int* stop_flag);

/* ---- projection-guided matching ---------------------------
 * The current Frame as U:src/Frame.cc holds it after extraction: keypoints mvKeysUn (= mvKeys,
 * distortion k1 == 0), descriptors, image bounds mnMinX..mnMaxY (ComputeImageBounds), the
 * 64 x 48 grid implied by them (AssignFeaturesToGrid / PosInGrid / GetFeaturesInArea), the
 * scale tables and the pose Tcw. claimed[k] = mvpMapPoints[k] set (with observations) before
 * the call (NULL: none). At most 65535 keypoints. */
typedef struct {
    int32_t n;
    const orbhip_kp* kps;       /* n: mvKeysUn */
    const uint8_t* desc;        /* n x 32: mDescriptors */
    const uint8_t* claimed;     /* n or NULL */
    float min_x, max_x, min_y, max_y;
    const float* scale_factors; /* mvScaleFactors */
    int32_t n_levels;
    float log_scale_factor;     /* mfLogScaleFactor */
    float fx, fy, cx, cy;       /* Pinhole mvParameters */
    float pose_q[4];            /* Tcw rotation (x, y, z, w) */
    float pose_t[3];
} orbhip_frame;

/* U:src/ORBmatcher.cc::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th,
 * bMono = true) (TrackWithMotionModel). Queries: LastFrame entries i with a MapPoint that is
 * not an outlier, in index order: world position, pMP->GetDescriptor(), LastFrame keypoint
 * octave and angle. match[q] = CurrentFrame keypoint assigned to query q (the adapter sets
 * CurrentFrame.mvpMapPoints[match[q]] = pMP) or -1. Returns nmatches. */
typedef struct {
    int32_t n;
    const float* points;        /* n x 3 */
    const uint8_t* desc;        /* n x 32 */
    const int32_t* octave;      /* n */
    const float* angle;         /* n: LastFrame.mvKeysUn[i].angle */
} orbhip_proj_last;
int orbhip_search_by_projection_last(orbhip_ctx* ctx, const orbhip_frame* cur, const orbhip_proj_last* last,
                                     float th, int check_orientation, int32_t* match);

/* U:src/Tracking.cc::SearchLocalPoints: Frame::isInFrustum(pMP, view_cos_limit = 0.5) for every
 * local MapPoint not skipped, then U:src/ORBmatcher.cc::SearchByProjection(F, vpMapPoints, th,
 * bFarPoints, thFarPoints) in vpMapPoints order. Per point: GetWorldPos, GetNormal,
 * mfMinDistance, mfMaxDistance, GetDescriptor; skip[m] = bad / already matched in this frame.
 * Outputs: in_view[m] = mbTrackInView, level[m] = mnTrackScaleLevel, match[m] = F keypoint or -1.
 * Returns nmatches. */
typedef struct {
    int32_t n;
    const float* points;        /* n x 3 */
    const float* normals;       /* n x 3 */
    const float* min_dist;      /* n: mfMinDistance */
    const float* max_dist;      /* n: mfMaxDistance */
    const uint8_t* desc;        /* n x 32 */
    const uint8_t* skip;        /* n or NULL */
} orbhip_local_points;
int orbhip_search_local_points(orbhip_ctx* ctx, const orbhip_frame* frame, const orbhip_local_points* mps,
                               float view_cos_limit, float th, float nnratio, int far_points, float th_far,
                               uint8_t* in_view, int32_t* level, int32_t* match);

/* ---- monocular initialisation matching -------------------------------------------
 * U:src/ORBmatcher.cc::SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>&
 * vbPrevMatched, vector<int>& vnMatches12, int windowSize), called by
 * U:src/Tracking.cc::MonocularInitialization as ORBmatcher(0.9, true) with windowSize 100.
 * Exact greedy semantics: F1 keypoints of octave 0 in index order, F2.GetFeaturesInArea(
 * vbPrevMatched[i1], windowSize, 0, 0) on F2's 64 x 48 grid (bounds min_x..max_y), candidates
 * with vMatchedDistance <= dist skipped, TH_LOW = 50 and the nnratio test, later better matches
 * steal the F2 keypoint, rotation histogram over all pushes (ComputeThreeMaxima).
 * prev_matched (n1 x 2 floats) is updated in place for the surviving matches; matches12[n1]
 * receives vnMatches12. Returns nmatches. Octaves must be >= 0. Envelope: 4 * (F2 octave-0
 * keypoints) + 4 * (F1 octave-0 keypoints) <= 150 KiB (ORBHIP_ERR_UNSUPPORTED beyond). */
typedef struct {
    int32_t n;
    const orbhip_kp* kps;       /* n: mvKeysUn */
    const uint8_t* desc;        /* n x 32 */
    float min_x, max_x, min_y, max_y;   /* mnMinX, mnMaxX, mnMinY, mnMaxY (grid of F2) */
} orbhip_init_frame;
int orbhip_search_for_initialization(orbhip_ctx* ctx, const orbhip_init_frame* f1, const orbhip_init_frame* f2,
                                     float* prev_matched, int window_size, float nnratio, int check_orientation,
                                     int32_t* matches12);

/* ---- KeyFrameDatabase place recognition ---------------------
 * U:src/KeyFrameDatabase.cc. The database lives on the device: add/erase mirror
 * KeyFrameDatabase::add(pKF) / erase(pKF) with the KF's BowVector (ascending word ids, L1
 * values; slot = the adapter's KeyFrame index, < max_kf). The KeyFrame members the queries use
 * (mnRelocQuery/Words, mRelocScore, mnPlaceRecognitionQuery/Words/Score) persist in the
 * database between queries, as on the KeyFrames. Per query the adapter passes the query
 * BowVector (<= 3072 words), a unique query id (Frame / KeyFrame mnId), covis = max_kf x 10
 * slots of KeyFrame::GetBestCovisibilityKeyFrames(10) (-1 padded), and optionally the map id of
 * every slot (GetMap()) with the query's map, and flags (bit 0 isBad(), bit 1 GetMap()->IsBad()). */
typedef struct orbhip_kfdb orbhip_kfdb;
typedef struct {
    int64_t query_id;
    const int32_t* words;
    const double* values;
    int32_t n;
    const int32_t* covis;       /* max_kf x 10 */
    const int32_t* kf_map;      /* max_kf or NULL (one map) */
    int32_t query_map;
    const uint8_t* kf_flags;    /* max_kf or NULL */
} orbhip_kfdb_query;
int orbhip_kfdb_create(orbhip_ctx* ctx, int max_kf, orbhip_kfdb** out);
int orbhip_kfdb_destroy(orbhip_kfdb* db);
int orbhip_kfdb_add(orbhip_kfdb* db, int kf, const int32_t* words, const double* values, int n);
int orbhip_kfdb_erase(orbhip_kfdb* db, int kf);
/* DetectRelocalizationCandidates(F, pMap): writes up to cap slots, returns the full count. */
int orbhip_kfdb_detect_relocalization(orbhip_kfdb* db, const orbhip_kfdb_query* q, int32_t* out, int cap);
/* DetectNBestCandidates(pKF, vpLoopCand, vpMergeCand, n): connected = max_kf flags of
 * pKF->GetConnectedKeyFrames() (or NULL); n <= 32. Returns n_loop + n_merge. */
int orbhip_kfdb_detect_nbest(orbhip_kfdb* db, const orbhip_kfdb_query* q, const uint8_t* connected, int n,
                             int32_t* loop_out, int32_t* n_loop, int32_t* merge_out, int32_t* n_merge);

/* ---- motion-only bundle adjustment -------------------------
 * U:src/Optimizer.cc::Optimizer::PoseOptimization(Frame* pFrame), monocular observations:
 * one VertexSE3Expmap (Tcw), EdgeSE3ProjectXYZOnlyPose per matched MapPoint (information
 * I * mvInvLevelSigma2[octave], Huber sqrt(5.991)), 4 rounds of Levenberg optimize(10) each
 * from the frame's initial pose, chi2 > 5.991 -> outlier after every round, robust kernel
 * dropped after round 2, early stop after round 0 for < 10 edges. The adapter fills one
 * problem per Frame from its mvpMapPoints (non-NULL entries, mvuRight < 0) and writes back
 * SetPose(result) and mvbOutlier[i] = outlier[k]. Returns nInitialCorrespondences - nBad
 * (0, pose untouched, when < 3 correspondences). */
typedef struct {
    int32_t n;                  /* correspondences */
    const float* pose_q;        /* 4: initial Tcw rotation (x, y, z, w) = pFrame->GetPose() */
    const float* pose_t;        /* 3 */
    const float* points;        /* n x 3: MapPoint::GetWorldPos() */
    const float* uv;            /* n x 2: mvKeysUn[i].pt */
    const int32_t* octave;      /* n: mvKeysUn[i].octave */
    const float* inv_sigma2;    /* per octave: mvInvLevelSigma2 */
    int32_t n_octaves;
    float fx, fy, cx, cy;       /* Pinhole mvParameters */
} orbhip_pose_problem;

typedef struct {
    float pose_q[4];            /* optimised Tcw */
    float pose_t[3];
    uint8_t* outlier;           /* n out (caller-owned, may be NULL): mvbOutlier */
    int32_t n_inliers;          /* PoseOptimization return value */
    int32_t lm_trials;          /* total Levenberg trials over the 4 rounds */
} orbhip_pose_result;

int orbhip_pose_optimization(orbhip_ctx* ctx, const orbhip_pose_problem* prob, orbhip_pose_result* res);
/* B frames (e.g. every camera of a rig, or a batch of agents) in one launch, one wavefront each. */
int orbhip_pose_optimization_batch(orbhip_ctx* ctx, const orbhip_pose_problem* probs, int B,
                                   orbhip_pose_result* res);

/* ---- bag of words -----------------------------------------
 * DBoW2 vocabulary in the ORBvoc.txt node order (Thirdparty/DBoW2 TemplatedVocabulary):
 * node 0 = root, node i (i >= 1) = line i of the text file with (parent, is_leaf, 32-byte
 * descriptor, weight); children keep file order; word ids follow leaf order.
 *   orbhip_vocab_load_text   TemplatedVocabulary::loadFromTextFile ("k L scoring weighting" header)
 *   orbhip_bow_transform     per-descriptor transform(feature, word, weight, &node, levelsup)
 *                            (U:src/Frame.cc::ComputeBoW: levelsup 4); the caller builds the
 *                            BowVector (weights summed per word, L1-normalised) and FeatureVector
 *                            (node -> ascending feature indices, weight > 0 only)
 *   orbhip_search_bow        U:src/ORBmatcher.cc::SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches):
 *                            match[f] = KF feature index matched to frame feature f, or -1 (the
 *                            adapter maps it to the KF's MapPoint*); kf_valid[i] = the KF feature
 *                            has a good map point. Returns nmatches. n <= 2048 per side. */
typedef struct orbhip_vocab orbhip_vocab;
int orbhip_vocab_create(orbhip_ctx* ctx, int k, int L, int scoring, int weighting, int n_nodes,
                        const int32_t* parent, const uint8_t* is_leaf, const uint8_t* desc32,
                        const double* weight, orbhip_vocab** out);
int orbhip_vocab_load_text(orbhip_ctx* ctx, const char* path, orbhip_vocab** out);
int orbhip_vocab_destroy(orbhip_vocab* vocab);
int orbhip_vocab_info(const orbhip_vocab* vocab, int32_t* k, int32_t* L, int32_t* n_nodes, int32_t* n_words);
int orbhip_bow_transform(orbhip_ctx* ctx, const orbhip_vocab* vocab, const uint8_t* desc32, int n, int levelsup,
                         int32_t* word_id, int32_t* node_id, double* weight);
/* device form over extractor outputs: B frames, descriptors at f*cap, counts d_n[f]; outputs at f*cap */
int orbhip_bow_transform_device(orbhip_ctx* ctx, const orbhip_vocab* vocab, const uint8_t* d_desc,
                                const int32_t* d_n, int B, int cap, int levelsup, int32_t* d_word,
                                int32_t* d_node, double* d_weight, void* stream);
int orbhip_search_bow(orbhip_ctx* ctx, const uint8_t* kf_desc, const float* kf_angle, const int32_t* kf_node,
                      const double* kf_weight, const uint8_t* kf_valid, int nkf, const uint8_t* f_desc,
                      const float* f_angle, const int32_t* f_node, const double* f_weight, int nf,
                      float ratio, int check_orientation, int th_low, int32_t* match);

/* ---- multi-GPU BundleAdjustment (SURVEY.md §8e, C5 GlobalBundleAdjustment) --------
 * One process per GPU. Landmarks (with their edges) are partitioned across ranks; every rank
 * holds all poses. Per LM trial the ranks sum their Schur contributions (the reduced camera
 * system S, its right-hand side, Hpp, chi2 / scale terms) with RCCL all-reduces over xGMI, solve
 * the identical S redundantly and back-substitute their own landmarks; all ranks follow one LM
 * schedule and return identical poses.
 *   orbhip_comm_unique_id  rank 0 only; send the 128 bytes to every rank (any transport)
 *   orbhip_comm_init       collective over the ranks: creates the context's communicator
 *   orbhip_ba_solve_sharded  collective: this rank's shard (all poses, its landmarks/edges);
 *                            the stop flag is agreed on (max over ranks) at each iteration
 *   orbhip_ba_solve_sharded_segments  collective: this rank holds nlocal consecutive shards
 *                            (segments rank*nlocal .. rank*nlocal+nlocal-1 of nranks*nlocal; the
 *                            same nlocal on every rank, else ORBHIP_ERR_ARG); they are summed on
 *                            the device, then all-reduced over the ranks
 *   orbhip_ba_solve_shards_local  the same decomposition with all shards in one process on one
 *                            device (the sums run on the device): single-GPU model and test. */
int orbhip_comm_unique_id(uint8_t* id128);
int orbhip_comm_init(orbhip_ctx* ctx, int nranks, int rank, const uint8_t* id128);
int orbhip_ba_solve_sharded(orbhip_ctx* ctx, const orbhip_ba_problem* shard, orbhip_ba_result* res,
                            const volatile int* stop_flag);
int orbhip_ba_solve_sharded_segments(orbhip_ctx* ctx, const orbhip_ba_problem* shards, int nlocal,
                                     orbhip_ba_result* res, const volatile int* stop_flag);
int orbhip_ba_solve_shards_local(orbhip_ctx* ctx, const orbhip_ba_problem* shards, int nshards,
                                 orbhip_ba_result* res, const volatile int* stop_flag);

#ifdef __cplusplus
}
#endif
#endif /* ORBHIP_H */
