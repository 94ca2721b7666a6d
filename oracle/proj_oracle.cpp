// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see orb_oracle.cpp header for the rules).
//
// CPU restatement of the projection-guided matchers, float semantics as
// the reference computes them (recalled upstream; the ORB_SLAM3 submodule is empty here):
//   U:src/Frame.cc::Frame::AssignFeaturesToGrid / PosInGrid   FRAME_GRID_COLS 64 x ROWS 48,
//       mfGridElementWidthInv = 64.f / (mnMaxX - mnMinX), cell = round((pt - min) * inv)
//   U:src/Frame.cc::Frame::GetFeaturesInArea(x, y, r, minLevel, maxLevel)   cells ix (outer),
//       iy, then cell order; |dx| < r && |dy| < r
//   U:src/Frame.cc::Frame::isInFrustum(pMP, viewingCosLimit)   Pc = mRcw P + mtcw, project,
//       bounds, 0.8 minDist / 1.2 maxDist, viewCos, MapPoint::PredictScale (ceil(log(ratio) /
//       mfLogScaleFactor), clamped)
//   U:src/ORBmatcher.cc::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th,
//       bMono = true)   window th * scale[lastOctave], levels lastOctave-1 .. lastOctave+1, best
//       Hamming (strict <, first wins) <= TH_HIGH = 100, greedy claims in LastFrame index order,
//       30-bin rotation histogram + ComputeThreeMaxima
//   U:src/ORBmatcher.cc::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, th,
//       bFarPoints, thFarPoints)   RadiusByViewingCos (2.5 if viewCos > 0.998, else 4.0; x th
//       when th != 1), levels predicted-1 .. predicted, best/second with levels, ratio test only
//       when both lie on the same level; greedy claims in vpMapPoints order
//   U:src/ORBmatcher.cc::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
//       F1 keypoints of octave 0 in index order; F2.GetFeaturesInArea(prev, windowSize, 0, 0);
//       candidates with vMatchedDistance[i2] <= dist skipped; best/second (strict <);
//       bestDist <= TH_LOW = 50 && bestDist < (float)bestDist2 * mfNNratio; a better later match
//       steals i2 (the earlier vnMatches12 entry is reset, its rotHist entry stays); rotation
//       histogram of pushes + ComputeThreeMaxima; vbPrevMatched updated for the survivors
// Pose arithmetic: Sophus SE3f * p = q._transformVector(p) + t (Eigen, float); mRcw =
// q.toRotationMatrix(); mOw = Twc.translation() = conj(q)._transformVector(-t). No FMA
// contraction (-ffp-contract=off). The searches take mvKeysUn and the image bounds as given:
// orc_undistort_keypoints / orc_image_bounds (end of file) compute them for a distorted pinhole
// (R:config/Monocular/MilkV.yaml:22-25); with k1 == 0 they are mvKeys and [0, cols] x [0, rows].
// PARITY UNPINNED by the reference (no fixtures upstream).
// ============================================================================
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace proj {

constexpr int kCols = 64, kRows = 48, TH_HIGH = 100, HISTO_LENGTH = 30;

struct Kp { float x, y, size, angle, response; int32_t octave; };   // orbhip_kp layout

struct Frame {
    int n;
    const Kp* kps;
    const uint8_t* desc;
    float minx, maxx, miny, maxy, invw, invh;
    std::vector<int> grid[kCols][kRows];
    void build() {
        invw = (float)kCols / (maxx - minx);
        invh = (float)kRows / (maxy - miny);
        for (int i = 0; i < n; i++) {
            const int px = (int)std::round((kps[i].x - minx) * invw);
            const int py = (int)std::round((kps[i].y - miny) * invh);
            if (px < 0 || px >= kCols || py < 0 || py >= kRows) continue;
            grid[px][py].push_back(i);
        }
    }
    void features_in_area(float x, float y, float r, int minLevel, int maxLevel, std::vector<int>& out) const {
        out.clear();
        const int nMinCellX = std::max(0, (int)std::floor((x - minx - r) * invw));
        if (nMinCellX >= kCols) return;
        const int nMaxCellX = std::min(kCols - 1, (int)std::ceil((x - minx + r) * invw));
        if (nMaxCellX < 0) return;
        const int nMinCellY = std::max(0, (int)std::floor((y - miny - r) * invh));
        if (nMinCellY >= kRows) return;
        const int nMaxCellY = std::min(kRows - 1, (int)std::ceil((y - miny + r) * invh));
        if (nMaxCellY < 0) return;
        const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
                for (int j : grid[ix][iy]) {
                    const Kp& k = kps[j];
                    if (bCheckLevels) {
                        if (k.octave < minLevel) continue;
                        if (maxLevel >= 0 && k.octave > maxLevel) continue;
                    }
                    const float dx = k.x - x, dy = k.y - y;
                    if (std::fabs(dx) < r && std::fabs(dy) < r) out.push_back(j);
                }
    }
};

static inline int hamming(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

// Eigen QuaternionBase::_transformVector, float
static inline void qrot(const float q[4], const float v[3], float o[3]) {
    float uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    const float c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    o[0] = v[0] + q[3] * uv[0] + c[0];
    o[1] = v[1] + q[3] * uv[1] + c[1];
    o[2] = v[2] + q[3] * uv[2] + c[2];
}

static inline void qtomat(const float q[4], float R[9]) {   // Eigen toRotationMatrix, float
    const float tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const float twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const float txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const float tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

static void three_maxima(const int* h, int& i1, int& i2, int& i3) {
    int m1 = 0, m2 = 0, m3 = 0;
    i1 = i2 = i3 = -1;
    for (int i = 0; i < HISTO_LENGTH; i++) {
        const int s = h[i];
        if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
        else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
        else if (s > m3) { m3 = s; i3 = i; }
    }
    if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
    else if (m3 < 0.1f * (float)m1) { i3 = -1; }
}

}  // namespace proj

extern "C" {

// SearchByProjection(CurrentFrame, LastFrame, th, bMono = true). Queries: the LastFrame entries
// with a non-outlier MapPoint, in index order (world position, MapPoint descriptor, last-frame
// keypoint octave and angle). claimed[k]: CurrentFrame.mvpMapPoints[k] already set (with
// observations) before the call. match[i] = current keypoint or -1. Returns nmatches.
int orc_search_by_projection_last(int n_cur, const void* cur_kps, const uint8_t* cur_desc, const uint8_t* claimed,
                                  float minx, float maxx, float miny, float maxy, const float* scale_factors,
                                  const float* q, const float* t, float fx, float fy, float cx, float cy, int n_last,
                                  const float* pts, const uint8_t* mp_desc, const int32_t* last_octave,
                                  const float* last_angle, float th, int check_orientation, int32_t* match) {
    proj::Frame F;
    F.n = n_cur; F.kps = (const proj::Kp*)cur_kps; F.desc = cur_desc;
    F.minx = minx; F.maxx = maxx; F.miny = miny; F.maxy = maxy;
    F.build();
    std::vector<uint8_t> taken(n_cur, 0);
    if (claimed) for (int k = 0; k < n_cur; k++) taken[k] = claimed[k];
    std::vector<int> cand, bin(n_last, -1);
    int hist[proj::HISTO_LENGTH] = {0};
    const float factor = 1.0f / proj::HISTO_LENGTH;
    int nmatches = 0;
    for (int i = 0; i < n_last; i++) {
        match[i] = -1;
        float Xc[3];
        proj::qrot(q, &pts[3 * i], Xc);
        Xc[0] += t[0]; Xc[1] += t[1]; Xc[2] += t[2];
        const float invzc = 1.0 / Xc[2];
        if (invzc < 0) continue;
        const float u = fx * Xc[0] / Xc[2] + cx, v = fy * Xc[1] / Xc[2] + cy;
        if (u < minx || u > maxx || v < miny || v > maxy) continue;
        const int lo = last_octave[i];
        const float radius = th * scale_factors[lo];
        F.features_in_area(u, v, radius, lo - 1, lo + 1, cand);
        if (cand.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int i2 : cand) {
            if (taken[i2]) continue;
            const int dist = proj::hamming(&mp_desc[32 * i], &cur_desc[32 * i2]);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        }
        if (bestDist <= proj::TH_HIGH) {
            taken[bestIdx2] = 1;
            match[i] = bestIdx2;
            nmatches++;
            if (check_orientation) {
                float rot = last_angle[i] - F.kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int b = (int)std::round(rot * factor);
                if (b == proj::HISTO_LENGTH) b = 0;
                bin[i] = b;
                hist[b]++;
            }
        }
    }
    if (check_orientation) {
        int i1, i2, i3;
        proj::three_maxima(hist, i1, i2, i3);
        for (int i = 0; i < n_last; i++)
            if (match[i] >= 0 && bin[i] != i1 && bin[i] != i2 && bin[i] != i3) { match[i] = -1; nmatches--; }
    }
    return nmatches;
}

// Frame::isInFrustum(pMP, view_cos_limit) for every local MapPoint not skipped, then
// SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints). Per point: world position,
// normal, mfMinDistance, mfMaxDistance, descriptor; skip[m] = already matched in this frame /
// bad (mbTrackInView stays false). Outputs in_view (mbTrackInView), level (mnTrackScaleLevel),
// match (frame keypoint or -1). Returns nmatches.
int orc_search_local_points(int n_cur, const void* cur_kps, const uint8_t* cur_desc, const uint8_t* claimed,
                            float minx, float maxx, float miny, float maxy, const float* scale_factors, int n_levels,
                            float log_scale_factor, const float* q, const float* t, float fx, float fy, float cx,
                            float cy, int n_mp, const float* pts, const float* normals, const float* min_dist,
                            const float* max_dist, const uint8_t* mp_desc, const uint8_t* skip, float view_cos_limit,
                            float th, float nnratio, int far_points, float th_far, uint8_t* in_view, int32_t* level,
                            int32_t* match) {
    proj::Frame F;
    F.n = n_cur; F.kps = (const proj::Kp*)cur_kps; F.desc = cur_desc;
    F.minx = minx; F.maxx = maxx; F.miny = miny; F.maxy = maxy;
    F.build();
    std::vector<uint8_t> taken(n_cur, 0);
    if (claimed) for (int k = 0; k < n_cur; k++) taken[k] = claimed[k];
    float R[9];
    proj::qtomat(q, R);
    const float qc[4] = {-q[0], -q[1], -q[2], q[3]};
    const float mt[3] = {t[0] * -1.0f, t[1] * -1.0f, t[2] * -1.0f};
    float Ow[3];
    proj::qrot(qc, mt, Ow);
    std::vector<float> projx(n_mp), projy(n_mp), vcos(n_mp), depth(n_mp);
    // ---- isInFrustum ----
    for (int m = 0; m < n_mp; m++) {
        in_view[m] = 0; level[m] = -1; match[m] = -1;
        if (skip && skip[m]) continue;
        const float* P = &pts[3 * m];
        const float Pc[3] = {R[0] * P[0] + R[1] * P[1] + R[2] * P[2] + t[0],
                             R[3] * P[0] + R[4] * P[1] + R[5] * P[2] + t[1],
                             R[6] * P[0] + R[7] * P[1] + R[8] * P[2] + t[2]};
        const float Pc_dist = std::sqrt(Pc[0] * Pc[0] + Pc[1] * Pc[1] + Pc[2] * Pc[2]);
        if (Pc[2] < 0.0f) continue;
        const float u = fx * Pc[0] / Pc[2] + cx, v = fy * Pc[1] / Pc[2] + cy;
        if (u < minx || u > maxx) continue;
        if (v < miny || v > maxy) continue;
        const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
        const float dist = std::sqrt(PO[0] * PO[0] + PO[1] * PO[1] + PO[2] * PO[2]);
        const float maxDistance = 1.2f * max_dist[m], minDistance = 0.8f * min_dist[m];
        if (dist < minDistance || dist > maxDistance) continue;
        const float* Pn = &normals[3 * m];
        const float viewCos = (PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2]) / dist;
        if (viewCos < view_cos_limit) continue;
        const float ratio = max_dist[m] / dist;
        int nScale = (int)std::ceil(std::log(ratio) / log_scale_factor);
        if (nScale < 0) nScale = 0;
        else if (nScale >= n_levels) nScale = n_levels - 1;
        in_view[m] = 1; level[m] = nScale;
        projx[m] = u; projy[m] = v; vcos[m] = viewCos; depth[m] = Pc_dist;
    }
    // ---- SearchByProjection ----
    const bool bFactor = th != 1.0;
    std::vector<int> cand;
    int nmatches = 0;
    for (int m = 0; m < n_mp; m++) {
        if (!in_view[m]) continue;
        if (far_points && depth[m] > th_far) continue;
        const int nPredictedLevel = level[m];
        float r = vcos[m] > 0.998 ? 2.5 : 4.0;   // RadiusByViewingCos
        if (bFactor) r *= th;
        F.features_in_area(projx[m], projy[m], r * scale_factors[nPredictedLevel], nPredictedLevel - 1,
                           nPredictedLevel, cand);
        if (cand.empty()) continue;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int idx : cand) {
            if (taken[idx]) continue;
            const int dist = proj::hamming(&mp_desc[32 * m], &cur_desc[32 * idx]);
            if (dist < bestDist) {
                bestDist2 = bestDist; bestDist = dist;
                bestLevel2 = bestLevel; bestLevel = F.kps[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = F.kps[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= proj::TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            if (bestLevel != bestLevel2 || bestDist <= nnratio * bestDist2) {
                taken[bestIdx] = 1;
                match[m] = bestIdx;
                nmatches++;
            }
        }
    }
    return nmatches;
}

// SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) with the matcher's
// mfNNratio / mbCheckOrientation. F2's grid uses its own image bounds. prev: n1 x 2, in/out.
int orc_search_for_initialization(int n1, const void* kps1, const uint8_t* desc1, int n2, const void* kps2,
                                  const uint8_t* desc2, float minx, float maxx, float miny, float maxy, float* prev,
                                  int window, float nnratio, int check_orientation, int32_t* matches12) {
    proj::Frame F2;
    F2.n = n2; F2.kps = (const proj::Kp*)kps2; F2.desc = desc2;
    F2.minx = minx; F2.maxx = maxx; F2.miny = miny; F2.maxy = maxy;
    F2.build();
    const proj::Kp* K1 = (const proj::Kp*)kps1;
    constexpr int TH_LOW = 50;
    int nmatches = 0;
    for (int i = 0; i < n1; i++) matches12[i] = -1;
    std::vector<int> rotHist[proj::HISTO_LENGTH];
    const float factor = 1.0f / proj::HISTO_LENGTH;
    std::vector<int> vMatchedDistance(n2, INT_MAX), vnMatches21(n2, -1), cand;
    for (int i1 = 0; i1 < n1; i1++) {
        const int level1 = K1[i1].octave;
        if (level1 > 0) continue;
        F2.features_in_area(prev[2 * i1], prev[2 * i1 + 1], (float)window, level1, level1, cand);
        if (cand.empty()) continue;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int i2 : cand) {
            const int dist = proj::hamming(&desc1[32 * i1], &desc2[32 * i2]);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) { bestDist2 = bestDist; bestDist = dist; bestIdx2 = i2; }
            else if (dist < bestDist2) bestDist2 = dist;
        }
        if (bestDist <= TH_LOW && bestDist < (float)bestDist2 * nnratio) {
            if (vnMatches21[bestIdx2] >= 0) { matches12[vnMatches21[bestIdx2]] = -1; nmatches--; }
            matches12[i1] = bestIdx2;
            vnMatches21[bestIdx2] = i1;
            vMatchedDistance[bestIdx2] = bestDist;
            nmatches++;
            if (check_orientation) {
                float rot = K1[i1].angle - F2.kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int b = (int)std::round(rot * factor);
                if (b == proj::HISTO_LENGTH) b = 0;
                rotHist[b].push_back(i1);
            }
        }
    }
    if (check_orientation) {
        int h[proj::HISTO_LENGTH];
        for (int b = 0; b < proj::HISTO_LENGTH; b++) h[b] = (int)rotHist[b].size();
        int ind1, ind2, ind3;
        proj::three_maxima(h, ind1, ind2, ind3);
        for (int b = 0; b < proj::HISTO_LENGTH; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int idx1 : rotHist[b])
                if (matches12[idx1] >= 0) { matches12[idx1] = -1; nmatches--; }
        }
    }
    for (int i1 = 0; i1 < n1; i1++)
        if (matches12[i1] >= 0) {
            prev[2 * i1] = F2.kps[matches12[i1]].x;
            prev[2 * i1 + 1] = F2.kps[matches12[i1]].y;
        }
    return nmatches;
}

// ---- distorted pinhole cameras (UndistortKeyPoints + image bounds) ----
// U:src/Frame.cc::Frame::UndistortKeyPoints: if mDistCoef.at<float>(0) == 0, mvKeysUn = mvKeys;
// else cv::undistortPoints(mat(N x 1, CV_32FC2), mat, K (float), mDistCoef (float k1 k2 p1 p2
// [k3]), cv::Mat(), mK). OCV 4.5.4 imgproc/src/undistort.dispatch.cpp: undistortPoints(src, dst,
// K, D, R, P) = the TermCriteria(MAX_ITER, 5, 0.01) overload -> cvUndistortPointsInternal, all in
// double: x = (u - cx) * (1 / fx), 5 fixed-point rounds of
//   r2 = x*x + y*y
//   icdist = (1 + ((k7*r2 + k6)*r2 + k5)*r2) / (1 + ((k4*r2 + k1)*r2 + k0)*r2)   (icdist < 0: restart, stop)
//   deltaX = 2*k2*x*y + k3*(r2 + 2*x*x) + k8*r2 + k9*r2*r2
//   deltaY = k2*(r2 + 2*y*y) + 2*k3*x*y + k10*r2 + k11*r2*r2
//   x = (x0 - deltaX) * icdist,  y = (y0 - deltaY) * icdist
// then RR = P * I = K: u' = (fx*x + 0*y) + cx, v' = (0*x + fy*y) + cy, w = 1 / ((0*x + 0*y) + 1),
// stored as float. The tilt matrices are the identity (k12 = k13 = 0) and drop out exactly.
// Frame::ComputeImageBounds: the 4 corners (0,0), (cols,0), (0,rows), (cols,rows) undistorted;
// mnMinX = min(x0, x2), mnMaxX = max(x1, x3), mnMinY = min(y0, y1), mnMaxY = max(y2, y3).
static void undistort_one(float u_f, float v_f, const float cam[4], const float dist[5], float& xo, float& yo) {
    double k[14] = {0};
    for (int i = 0; i < 5; i++) k[i == 4 ? 4 : i] = (double)dist[i];   // k1 k2 p1 p2 k3 -> k[0..4]
    const double fx = cam[0], fy = cam[1], cx = cam[2], cy = cam[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    const double u = u_f, v = v_f;
    double x = (u - cx) * ifx, y = (v - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        if (icdist < 0) {
            x = (u - cx) * ifx;
            y = (v - cy) * ify;
            break;
        }
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    const double xx = fx * x + 0.0 * y + cx;
    const double yy = 0.0 * x + fy * y + cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    xo = (float)(xx * ww);
    yo = (float)(yy * ww);
}

// cam = {fx, fy, cx, cy}; dist = {k1, k2, p1, p2, k3}. in/out: orbhip_kp records (out may alias in).
void orc_undistort_keypoints(const void* in_kps, int n, const float* cam, const float* dist, void* out_kps) {
    const proj::Kp* in = (const proj::Kp*)in_kps;
    proj::Kp* out = (proj::Kp*)out_kps;
    for (int i = 0; i < n; i++) {
        proj::Kp k = in[i];
        if (dist[0] != 0.0f) undistort_one(in[i].x, in[i].y, cam, dist, k.x, k.y);
        out[i] = k;
    }
}

void orc_image_bounds(int cols, int rows, const float* cam, const float* dist, float* bounds) {
    if (dist[0] == 0.0f) {
        bounds[0] = 0.0f; bounds[1] = (float)cols; bounds[2] = 0.0f; bounds[3] = (float)rows;
        return;
    }
    float x[4], y[4];
    const float cu[4] = {0.0f, (float)cols, 0.0f, (float)cols}, cv_[4] = {0.0f, 0.0f, (float)rows, (float)rows};
    for (int i = 0; i < 4; i++) undistort_one(cu[i], cv_[i], cam, dist, x[i], y[i]);
    bounds[0] = std::min(x[0], x[2]);
    bounds[1] = std::max(x[1], x[3]);
    bounds[2] = std::min(y[0], y[1]);
    bounds[3] = std::max(y[2], y[3]);
}

}  // extern "C"
