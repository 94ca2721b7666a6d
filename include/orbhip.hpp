// orbhip.hpp — C++ host mirror of the reference interfaces over the C-ABI of orbhip.h.
//
// Same names, argument meaning and error behaviour as the ORB_SLAM3 classes this path replaces
// (upstream ORB_SLAM3 v1.0, the gjcliff fork's submodule; cited U:file::Symbol because the
// submodule is empty in the reference tree):
//   U:include/ORBextractor.h  class ORBextractor   -> orbhip::ORBextractor
//   U:include/ORBmatcher.h    ORBmatcher::DescriptorDistance, TH_LOW / TH_HIGH / HISTO_LENGTH
//   U:include/Optimizer.h     Optimizer::LocalBundleAdjustment / BundleAdjustment (problem form)
// The reference types (cv::Mat, cv::KeyPoint, KeyFrame, MapPoint) stay on the adapter side
// (INTEGRATION.md). Here images are (pointer, w, h, stride) and keypoints are orbhip::KeyPoint
// with cv::KeyPoint's fields. Header-only: link liborbhip.so.
#ifndef ORBHIP_HPP
#define ORBHIP_HPP

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "orbhip.h"

namespace orbhip {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& what) : std::runtime_error(what + ": status " + std::to_string(code)), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

inline void check(int rc, const char* what) {
    if (rc < 0) throw Error(rc, what);
}

// cv::KeyPoint's fields as ORBextractor fills them (class_id is always -1 there).
struct KeyPoint {
    float x, y, size, angle, response;
    int octave;
    int class_id = -1;
};

// U:include/ORBextractor.h::ORBextractor
class ORBextractor {
public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0)
        : nfeatures_(nfeatures), scaleFactor_(scaleFactor), nlevels_(nlevels) {
        orbhip_orb_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
        check(orbhip_create(&ctx_, device, &p), "orbhip_create");
        // the ctor's tables (U:src/ORBextractor.cc): mvScaleFactor from the library (float,
        // accumulated through the double scaleFactor), sigma2 = s*s, inverses in float
        mvScaleFactor_.resize(nlevels);
        check(orbhip_level_info(ctx_, 640, 480, nullptr, nullptr, nullptr, mvScaleFactor_.data()), "orbhip_level_info");
        for (int l = 0; l < nlevels; l++) {
            mvLevelSigma2_.push_back(mvScaleFactor_[l] * mvScaleFactor_[l]);
            mvInvScaleFactor_.push_back(1.0f / mvScaleFactor_[l]);
            mvInvLevelSigma2_.push_back(1.0f / mvLevelSigma2_[l]);
        }
    }
    ~ORBextractor() { if (ctx_) orbhip_destroy(ctx_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // operator()(InputArray image, InputArray mask, vector<KeyPoint>&, OutputArray descriptors,
    //            vector<int>& vLappingArea) -> monoIndex; -1 on an empty image. The mask is
    //            ignored by the reference as well. descriptors: N rows of 32 bytes.
    int operator()(const uint8_t* image, int w, int h, int stride, std::vector<KeyPoint>& keypoints,
                   std::vector<uint8_t>& descriptors, const std::vector<int>& vLappingArea) {
        keypoints.clear();
        descriptors.clear();
        if (!image || w <= 0 || h <= 0) return -1;
        const int cap = orbhip_max_keypoints(ctx_, w, h);
        check(cap, "orbhip_max_keypoints");
        kp_.resize(cap);
        descriptors.resize((size_t)cap * 32);
        int n = 0, mono = 0;
        const int lap0 = vLappingArea.size() > 0 ? vLappingArea[0] : 0;
        const int lap1 = vLappingArea.size() > 1 ? vLappingArea[1] : 1000;
        const int rc = orbhip_extract(ctx_, image, w, h, stride, lap0, lap1, kp_.data(), descriptors.data(), cap, &n, &mono);
        if (rc == ORBHIP_ERR_EMPTY) return -1;
        check(rc, "orbhip_extract");
        keypoints.resize(n);
        for (int i = 0; i < n; i++)
            keypoints[i] = KeyPoint{kp_[i].x, kp_[i].y, kp_[i].size, kp_[i].angle, kp_[i].response, kp_[i].octave};
        descriptors.resize((size_t)n * 32);
        return mono;
    }

    int inline GetLevels() const { return nlevels_; }
    float inline GetScaleFactor() const { return scaleFactor_; }
    std::vector<float> inline GetScaleFactors() const { return mvScaleFactor_; }
    std::vector<float> inline GetInverseScaleFactors() const { return mvInvScaleFactor_; }
    std::vector<float> inline GetScaleSigmaSquares() const { return mvLevelSigma2_; }
    std::vector<float> inline GetInverseScaleSigmaSquares() const { return mvInvLevelSigma2_; }
    orbhip_ctx* context() const { return ctx_; }

private:
    orbhip_ctx* ctx_ = nullptr;
    int nfeatures_;
    float scaleFactor_;
    int nlevels_;
    std::vector<float> mvScaleFactor_, mvInvScaleFactor_, mvLevelSigma2_, mvInvLevelSigma2_;
    std::vector<orbhip_kp> kp_;
};

// U:include/ORBmatcher.h — the constants and the brute-force acceptance rule (a11/a12).
class ORBmatcher {
public:
    static const int TH_LOW = 50;
    static const int TH_HIGH = 100;
    static const int HISTO_LENGTH = 30;

    ORBmatcher(float nnratio = 0.6f, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orbhip_descriptor_distance(a, b); }

    // best/second over the whole train set; match[i] = train index or -1. Returns #matches.
    int MatchBruteForce(orbhip_ctx* ctx, const std::vector<uint8_t>& q, const std::vector<float>& qAngle,
                        const std::vector<uint8_t>& t, const std::vector<float>& tAngle, std::vector<int>& match,
                        int thLow = TH_LOW) const {
        const int nq = (int)(q.size() / 32), nt = (int)(t.size() / 32);
        match.assign(nq, -1);
        std::vector<int32_t> best(nq), second(nq);
        const int rc = orbhip_match_bf(ctx, q.data(), qAngle.data(), nq, t.data(), tAngle.data(), nt, thLow, mfNNratio,
                                       mbCheckOrientation ? 1 : 0, match.data(), best.data(), second.data());
        check(rc, "orbhip_match_bf");
        return rc;
    }

    // U:src/ORBmatcher.cc::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize):
    // keypoints/descriptors of both frames, F2's image bounds, vbPrevMatched as (x, y) pairs
    // (updated in place). Returns nmatches.
    int SearchForInitialization(orbhip_ctx* ctx, const std::vector<orbhip_kp>& kps1, const std::vector<uint8_t>& desc1,
                                const std::vector<orbhip_kp>& kps2, const std::vector<uint8_t>& desc2,
                                const float bounds2[4], std::vector<float>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10) const {
        vnMatches12.assign(kps1.size(), -1);
        const orbhip_init_frame f1{(int32_t)kps1.size(), kps1.data(), desc1.data(), 0.f, 1.f, 0.f, 1.f};
        const orbhip_init_frame f2{(int32_t)kps2.size(), kps2.data(), desc2.data(), bounds2[0], bounds2[1],
                                   bounds2[2], bounds2[3]};
        const int rc = orbhip_search_for_initialization(ctx, &f1, &f2, vbPrevMatched.data(), windowSize, mfNNratio,
                                                        mbCheckOrientation ? 1 : 0, vnMatches12.data());
        check(rc, "orbhip_search_for_initialization");
        return rc;
    }

    float mfNNratio;
    bool mbCheckOrientation;
};

// U:include/KeyFrameDatabase.h — the device database; slots stand for KeyFrames.
class KeyFrameDatabase {
public:
    KeyFrameDatabase(orbhip_ctx* ctx, int maxKF) : maxKF_(maxKF) { check(orbhip_kfdb_create(ctx, maxKF, &db_), "orbhip_kfdb_create"); }
    ~KeyFrameDatabase() { if (db_) orbhip_kfdb_destroy(db_); }
    KeyFrameDatabase(const KeyFrameDatabase&) = delete;
    KeyFrameDatabase& operator=(const KeyFrameDatabase&) = delete;
    void add(int kf, const std::vector<int32_t>& words, const std::vector<double>& values) {
        check(orbhip_kfdb_add(db_, kf, words.data(), values.data(), (int)words.size()), "orbhip_kfdb_add");
    }
    void erase(int kf) { check(orbhip_kfdb_erase(db_, kf), "orbhip_kfdb_erase"); }
    std::vector<int> DetectRelocalizationCandidates(const orbhip_kfdb_query& q) {
        std::vector<int32_t> out(maxKF_);
        const int n = orbhip_kfdb_detect_relocalization(db_, &q, out.data(), maxKF_);
        check(n, "orbhip_kfdb_detect_relocalization");
        return std::vector<int>(out.begin(), out.begin() + std::min(n, maxKF_));
    }
    void DetectNBestCandidates(const orbhip_kfdb_query& q, const std::vector<uint8_t>& connected, int n,
                               std::vector<int>& loopCand, std::vector<int>& mergeCand) {
        std::vector<int32_t> lo(n > 0 ? n : 1), me(n > 0 ? n : 1);
        int32_t nl = 0, nm = 0;
        check(orbhip_kfdb_detect_nbest(db_, &q, connected.empty() ? nullptr : connected.data(), n, lo.data(), &nl,
                                       me.data(), &nm), "orbhip_kfdb_detect_nbest");
        loopCand.assign(lo.begin(), lo.begin() + nl);
        mergeCand.assign(me.begin(), me.begin() + nm);
    }

private:
    orbhip_kfdb* db_ = nullptr;
    int maxKF_;
};

// U:include/Optimizer.h — the g2o problem of LocalBundleAdjustment in SoA form. The adapter
// fills it from the local KeyFrames / MapPoints and applies the result.
struct BAProblem {
    std::vector<float> pose_q, pose_t, points, edge_uv, inv_sigma2;
    std::vector<uint8_t> pose_fixed;
    std::vector<int32_t> edge_pose, edge_point, edge_octave;
    float fx = 0, fy = 0, cx = 0, cy = 0;
    float huber_delta = std::sqrt(5.991f);
    int iterations = 10;
    int early_stop = 0;
};

struct BAResult {
    std::vector<float> pose_q, pose_t, points, edge_chi2;
    std::vector<uint8_t> edge_depth_ok;
    double initial_chi2 = 0, final_chi2 = 0;
    int iterations_done = 0, lm_trials = 0;
};

class Optimizer {
public:
    // LocalBundleAdjustment's optimize(10) with Huber sqrt(5.991). The reference's bool*
    // pbStopFlag (LocalMapping::mbAbortBA -> g2o setForceStopFlag) is an int here, polled by
    // the solver between LM iterations and trials; NULL = never stop.
    static BAResult LocalBundleAdjustment(orbhip_ctx* ctx, const BAProblem& p, const volatile int* pbStopFlag = nullptr) {
        return solve(ctx, p, pbStopFlag);
    }
    // BundleAdjustment(vpKF, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust): robust -> sqrt(5.99)
    static BAResult BundleAdjustment(orbhip_ctx* ctx, BAProblem p, int nIterations = 5,
                                     const volatile int* pbStopFlag = nullptr, bool bRobust = true) {
        p.iterations = nIterations;
        p.huber_delta = bRobust ? std::sqrt(5.99f) : 0.0f;
        return solve(ctx, p, pbStopFlag);
    }

private:
    static BAResult solve(orbhip_ctx* ctx, const BAProblem& p, const volatile int* stop) {
        const int P = (int)p.pose_fixed.size(), M = (int)(p.points.size() / 3), E = (int)p.edge_pose.size();
        orbhip_ba_problem c{P, M, E, p.pose_q.data(), p.pose_t.data(), p.pose_fixed.data(), p.points.data(),
                            p.edge_pose.data(), p.edge_point.data(), p.edge_uv.data(), p.edge_octave.data(),
                            p.inv_sigma2.data(), (int)p.inv_sigma2.size(), p.fx, p.fy, p.cx, p.cy, p.huber_delta,
                            p.iterations, p.early_stop};
        BAResult r;
        r.pose_q.resize(4 * (size_t)P); r.pose_t.resize(3 * (size_t)P); r.points.resize(3 * (size_t)M);
        r.edge_chi2.resize(E); r.edge_depth_ok.resize(E);
        orbhip_ba_result o{r.pose_q.data(), r.pose_t.data(), r.points.data(), r.edge_chi2.data(), r.edge_depth_ok.data(),
                           0, 0, 0, 0};
        check(orbhip_ba_solve(ctx, &c, &o, stop), "orbhip_ba_solve");
        r.initial_chi2 = o.initial_chi2; r.final_chi2 = o.final_chi2;
        r.iterations_done = o.iterations_done; r.lm_trials = o.lm_trials;
        return r;
    }
};

// Camera front-end stream (orbhip_frontend_*): push device frames, read slots when needed.
class FrameStream {
public:
    FrameStream(int w, int h, int frames_in_flight = 8, int device = 0, orbhip_orb_params prm = {1000, 1.2f, 8, 20, 7},
                int th_low = 50, float nnratio = 0.9f, bool check_orientation = true) {
        check(orbhip_frontend_create(&fe_, device, &prm, w, h, frames_in_flight, th_low, nnratio,
                                     check_orientation ? 1 : 0),
              "orbhip_frontend_create");
    }
    ~FrameStream() {
        if (fe_) orbhip_frontend_destroy(fe_);
    }
    FrameStream(const FrameStream&) = delete;
    FrameStream& operator=(const FrameStream&) = delete;
    // returns the slot that will hold this frame's keypoints and its match to the previous frame
    int push(const uint8_t* d_gray, int stride, int lap0 = 0, int lap1 = 1000) {
        const int slot = orbhip_frontend_push(fe_, d_gray, stride, lap0, lap1);
        check(slot, "orbhip_frontend_push");
        return slot;
    }
    orbhip_frontend_slot view(int slot) const {
        orbhip_frontend_slot v{};
        check(orbhip_frontend_view(fe_, slot, &v), "orbhip_frontend_view");
        return v;
    }
    void wait(int slot, void* stream = nullptr) const { check(orbhip_frontend_wait(fe_, slot, stream), "orbhip_frontend_wait"); }

private:
    orbhip_frontend* fe_ = nullptr;
};

}  // namespace orbhip

#endif  // ORBHIP_HPP
