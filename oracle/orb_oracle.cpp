// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into liborbhip.so.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load liborb_oracle.so, and only as the checker / CPU baseline.
//
// CPU restatement of the reference ORB front-end hot path:
//   U:src/ORBextractor.cc  (ORB_SLAM3 v1.0 / gjcliff fork; submodule EMPTY here)
//   U:src/ORBmatcher.cc    (DescriptorDistance, ratio test, rotation histogram)
//   OCV 4.5.4 primitives it calls: resize INTER_LINEAR 8U, FAST_t<16> +
//   cornerScore<16>, GaussianBlur bit-exact fixed point, fastAtan2, cvRound.
//   glibc 2.35 cosf/sinf are called directly (the reference's std::cos(float)).
//
// PARITY UNPINNED by the reference itself: the ORB_SLAM3 submodule is an empty
// un-vendored git submodule (R:.gitmodules:1-3), OpenCV is absent, and upstream
// has no tests or fixtures. The restatement follows
// SURVEY.md Appendix A (recalled upstream semantics) and is pinned by
// definitional KATs (tests/test_oracle_kats.py) and the rBRIEF pattern md5.
//
// Build: oracle/Makefile  (g++ -O3 -march=native -ffp-contract=off).
// The octree below deliberately uses std::list exactly like the reference, so
// it checks the GPU's array-based emulation independently. Hazard C.3: the
// reference breaks size ties by ExtractorNode* address (allocator-dependent);
// this restatement (and the GPU) use the node creation serial instead.
// ============================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <vector>

#include "../include/orbhip_pattern.h"

namespace orc {

using std::vector;

// ---- OpenCV rounding helpers (OCV:core/include/opencv2/core/fast_math.hpp) ----
static inline int cvRound(float v) { return (int)std::nearbyintf(v); }   // SSE cvtss2si: half-even
static inline int cvRoundD(double v) { return (int)std::nearbyint(v); }
static inline int cvFloor(float v) { int i = (int)v; return i - (i > v); }
static inline int cvCeil(double v) { int i = (int)v; return i + (i < v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }
static inline short sat_s16(int v) { return (short)(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }

struct KP {               // cv::KeyPoint fields the path uses
    float x, y, size, angle, response;
    int octave;
};

struct Img {
    int w = 0, h = 0;
    vector<uint8_t> d;    // continuous, step == w
    const uint8_t* row(int y) const { return d.data() + (size_t)y * w; }
    uint8_t* row(int y) { return d.data() + (size_t)y * w; }
};

// ---------------------------------------------------------------------------
// a1  U:src/ORBextractor.cc::ORBextractor::ORBextractor(nfeatures, scaleFactor,
//     nlevels, iniThFAST, minThFAST) — scale tables, features per level, umax.
// ---------------------------------------------------------------------------
struct Extractor {
    int nfeatures, nlevels, iniThFAST, minThFAST;
    double scaleFactor;   // member is double holding the float ctor argument
    vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
    vector<int> mnFeaturesPerLevel, umax;
    vector<Img> pyr;

    Extractor(int nf, float sf, int nl, int ini, int mn)
        : nfeatures(nf), nlevels(nl), iniThFAST(ini), minThFAST(mn), scaleFactor(sf) {
        mvScaleFactor.resize(nlevels);
        mvLevelSigma2.resize(nlevels);
        mvScaleFactor[0] = 1.0f;
        mvLevelSigma2[0] = 1.0f;
        for (int i = 1; i < nlevels; i++) {
            mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);
            mvLevelSigma2[i] = mvScaleFactor[i] * mvScaleFactor[i];
        }
        mvInvScaleFactor.resize(nlevels);
        mvInvLevelSigma2.resize(nlevels);
        for (int i = 0; i < nlevels; i++) {
            mvInvScaleFactor[i] = 1.0f / mvScaleFactor[i];
            mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
        }
        pyr.resize(nlevels);
        mnFeaturesPerLevel.resize(nlevels);
        float factor = (float)(1.0f / scaleFactor);
        float nDesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
        int sumFeatures = 0;
        for (int level = 0; level < nlevels - 1; level++) {
            mnFeaturesPerLevel[level] = cvRound(nDesired);
            sumFeatures += mnFeaturesPerLevel[level];
            nDesired *= factor;
        }
        mnFeaturesPerLevel[nlevels - 1] = std::max(nfeatures - sumFeatures, 0);

        const int HALF_PATCH_SIZE = 15;
        umax.resize(HALF_PATCH_SIZE + 1);
        int v, v0, vmax = (int)std::floor(HALF_PATCH_SIZE * std::sqrt(2.f) / 2 + 1);
        int vmin = cvCeil(HALF_PATCH_SIZE * std::sqrt(2.f) / 2);
        const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
        for (v = 0; v <= vmax; ++v) umax[v] = cvRoundD(std::sqrt(hp2 - v * v));
        for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }
};

// ---------------------------------------------------------------------------
// a4  OCV:imgproc/src/resize.cpp hal::resize → resizeGeneric_<HResizeLinear<u8,int,
//     short,2048,HResizeLinearVec_8u32s>, VResizeLinear<u8,int,short,
//     FixedPtCast<int,u8,22>, VResizeLinearVec_32s8u>> for CV_8UC1, INTER_LINEAR.
//     Baseline 128-bit SIMD build: V pass lanes [0, vend) use the v_mul_hi form.
// ---------------------------------------------------------------------------
static int vresize_simd_end(int width) {
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    for (; x < width - 8; x += 8) {}
    return x;
}

static bool resize_linear_8u(const Img& src, Img& dst) {
    const int sw = src.w, sh = src.h, dw = dst.w, dh = dst.h;
    double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    int iscale_x = cvRoundD(scale_x), iscale_y = cvRoundD(scale_y);
    bool is_area_fast = std::abs(scale_x - iscale_x) < DBL_EPSILON && std::abs(scale_y - iscale_y) < DBL_EPSILON;
    if (is_area_fast && iscale_x == 2 && iscale_y == 2) return false;   // INTER_AREA path: unsupported
    vector<int> xofs(dw), yofs(dh);
    vector<short> ialpha(2 * dw), ibeta(2 * dh);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cvFloor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0, sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        float cb0 = 1.f - fx, cb1 = fx;
        ialpha[2 * dx] = sat_s16(cvRound(cb0 * 2048));
        ialpha[2 * dx + 1] = sat_s16(cvRound(cb1 * 2048));
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cvFloor(fy);
        fy -= sy;
        yofs[dy] = sy;
        float cb0 = 1.f - fy, cb1 = fy;
        ibeta[2 * dy] = sat_s16(cvRound(cb0 * 2048));
        ibeta[2 * dy + 1] = sat_s16(cvRound(cb1 * 2048));
    }
    auto clip = [](int x, int a, int b) { return x >= a ? (x < b ? x : b - 1) : a; };
    vector<int> r0(dw), r1(dw);
    const int vend = vresize_simd_end(dw);
    for (int dy = 0; dy < dh; dy++) {
        const uint8_t* S0 = src.row(clip(yofs[dy], 0, sh));
        const uint8_t* S1 = src.row(clip(yofs[dy] + 1, 0, sh));
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (dx < xmax) {
                int a0 = ialpha[2 * dx], a1 = ialpha[2 * dx + 1];
                r0[dx] = S0[sx] * a0 + S0[sx + 1] * a1;
                r1[dx] = S1[sx] * a0 + S1[sx + 1] * a1;
            } else {
                r0[dx] = S0[sx] * 2048;
                r1[dx] = S1[sx] * 2048;
            }
        }
        const int b0 = ibeta[2 * dy], b1 = ibeta[2 * dy + 1];
        uint8_t* D = dst.row(dy);
        for (int x = 0; x < dw; x++) {
            if (x < vend) {
                // v_pack(S>>4) (sat s16), v_mul_hi(.,b) = (a*b)>>16, saturating s16 add,
                // v_rshr_pack_u<2>: (v+2)>>2 saturated to u8
                int s0 = std::min(std::max(r0[x] >> 4, -32768), 32767);
                int s1 = std::min(std::max(r1[x] >> 4, -32768), 32767);
                int t = ((s0 * b0) >> 16) + ((s1 * b1) >> 16);
                t = std::min(std::max(t, -32768), 32767);
                D[x] = sat_u8((t + 2) >> 2);
            } else {
                D[x] = sat_u8((r0[x] * b0 + r1[x] * b1 + (1 << 21)) >> 22);
            }
        }
    }
    return true;
}

// a3  U:src/ORBextractor.cc::ORBextractor::ComputePyramid — cascade: level l is
//     resized from level l-1. The 19-px copyMakeBorder is never read by any output
//     (FAST windows lie in [16, w-16), IC_Angle / descriptors stay >=1 px inside),
//     so only the ROI images are kept.
static bool compute_pyramid(Extractor& E, const uint8_t* img, int w, int h, int stride) {
    for (int level = 0; level < E.nlevels; ++level) {
        float scale = E.mvInvScaleFactor[level];
        int sw = cvRound((float)w * scale), sh = cvRound((float)h * scale);
        Img& L = E.pyr[level];
        L.w = sw; L.h = sh; L.d.assign((size_t)sw * sh, 0);
        if (level == 0) {
            for (int y = 0; y < h; y++) std::memcpy(L.row(y), img + (size_t)y * stride, w);
        } else {
            if (sw == E.pyr[level - 1].w && sh == E.pyr[level - 1].h) { L.d = E.pyr[level - 1].d; continue; }
            if (!resize_linear_8u(E.pyr[level - 1], L)) return false;
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// a6  OCV:features2d/src/fast.cpp::FAST_t<16> (scalar path) + fast_score.cpp::
//     cornerScore<16>, run on a sub-window (ptr, step, rows, cols).
// ---------------------------------------------------------------------------
static void makeOffsets16(int pixel[25], int step) {
    static const int offsets16[][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                       {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    int k = 0;
    for (; k < 16; k++) pixel[k] = offsets16[k][0] + offsets16[k][1] * step;
    for (; k < 25; k++) pixel[k] = pixel[k - 16];
}

static int cornerScore16(const uint8_t* ptr, const int pixel[], int threshold) {
    const int K = 8, N = K * 3 + 1;
    int k, v = ptr[0];
    short d[N];
    for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

static void fast16(const uint8_t* base, int step, int rows, int cols, vector<KP>& kps, int threshold) {
    const int K = 8, N = 16 + K + 1;
    int i, j, k, pixel[25];
    makeOffsets16(pixel, step);
    kps.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t threshold_tab[512];
    for (i = -255; i <= 255; i++) threshold_tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (cols < 1 || rows < 1) return;
    vector<uint8_t> bufv((size_t)cols * 3, 0);
    vector<int> cpv((size_t)(cols + 1) * 3, 0);
    uint8_t* buf[3] = {bufv.data(), bufv.data() + cols, bufv.data() + 2 * cols};
    int* cpbuf[3] = {cpv.data() + 1, cpv.data() + 1 + (cols + 1), cpv.data() + 1 + 2 * (cols + 1)};
    for (i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = base + (size_t)i * step + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        std::memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (j = 3; j < cols - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t* tab = &threshold_tab[0] - v + 255;
                int d = tab[ptr[pixel[0]]] | tab[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[2]]] | tab[ptr[pixel[10]]];
                d &= tab[ptr[pixel[4]]] | tab[ptr[pixel[12]]];
                d &= tab[ptr[pixel[6]]] | tab[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[1]]] | tab[ptr[pixel[9]]];
                d &= tab[ptr[pixel[3]]] | tab[ptr[pixel[11]]];
                d &= tab[ptr[pixel[5]]] | tab[ptr[pixel[13]]];
                d &= tab[ptr[pixel[7]]] | tab[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)cornerScore16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)cornerScore16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
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
        for (k = 0; k < ncorners; k++) {
            j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] && score > pprev[j] &&
                score > pprev[j + 1] && score > curr[j - 1] && score > curr[j] && score > curr[j + 1]) {
                kps.push_back(KP{(float)j, (float)(i - 1), 7.f, -1.f, (float)score, 0});
            }
        }
    }
}

// ---------------------------------------------------------------------------
// a7  U:src/ORBextractor.cc::ExtractorNode::DivideNode + ORBextractor::DistributeOctTree
// ---------------------------------------------------------------------------
struct Node {
    int ulx, uly, urx, ury, blx, bly, brx, bry;   // UL, UR, BL, BR
    vector<KP> keys;
    bool bNoMore = false;
    long serial = 0;                              // creation order (replaces the pointer tie-break)
    std::list<Node>::iterator lit;
};

static void divide_node(const Node& p, Node& n1, Node& n2, Node& n3, Node& n4) {
    const int halfX = (int)std::ceil((float)(p.urx - p.ulx) / 2);
    const int halfY = (int)std::ceil((float)(p.bry - p.uly) / 2);
    n1.ulx = p.ulx;          n1.uly = p.uly;
    n1.urx = p.ulx + halfX;  n1.ury = p.uly;
    n1.blx = p.ulx;          n1.bly = p.uly + halfY;
    n1.brx = p.ulx + halfX;  n1.bry = p.uly + halfY;
    n2.ulx = n1.urx; n2.uly = n1.ury;
    n2.urx = p.urx;  n2.ury = p.ury;
    n2.blx = n1.brx; n2.bly = n1.bry;
    n2.brx = p.urx;  n2.bry = p.uly + halfY;
    n3.ulx = n1.blx; n3.uly = n1.bly;
    n3.urx = n1.brx; n3.ury = n1.bry;
    n3.blx = p.blx;  n3.bly = p.bly;
    n3.brx = n1.brx; n3.bry = p.bly;
    n4.ulx = n3.urx; n4.uly = n3.ury;
    n4.urx = n2.brx; n4.ury = n2.bry;
    n4.blx = n3.brx; n4.bly = n3.bry;
    n4.brx = p.brx;  n4.bry = p.bry;
    for (const KP& kp : p.keys) {
        if (kp.x < n1.urx) {
            if (kp.y < n1.bry) n1.keys.push_back(kp); else n3.keys.push_back(kp);
        } else if (kp.y < n1.bry)
            n2.keys.push_back(kp);
        else
            n4.keys.push_back(kp);
    }
    if (n1.keys.size() == 1) n1.bNoMore = true;
    if (n2.keys.size() == 1) n2.bNoMore = true;
    if (n3.keys.size() == 1) n3.bNoMore = true;
    if (n4.keys.size() == 1) n4.bNoMore = true;
}

struct SizeSerial {
    int size;
    long serial;
    Node* node;
    bool operator<(const SizeSerial& o) const { return size != o.size ? size < o.size : serial < o.serial; }
};

static vector<KP> distribute_octtree(const vector<KP>& keys, int minX, int maxX, int minY, int maxY, int N) {
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    std::list<Node> lNodes;
    vector<Node*> vpIni(nIni);
    long serial = 0;
    for (int i = 0; i < nIni; i++) {
        Node ni;
        ni.ulx = (int)(hX * (float)i);       ni.uly = 0;
        ni.urx = (int)(hX * (float)(i + 1)); ni.ury = 0;
        ni.blx = ni.ulx;                     ni.bly = maxY - minY;
        ni.brx = ni.urx;                     ni.bry = maxY - minY;
        ni.serial = serial++;
        lNodes.push_back(ni);
        vpIni[i] = &lNodes.back();
    }
    for (const KP& kp : keys) vpIni[(int)(kp.x / hX)]->keys.push_back(kp);
    for (auto lit = lNodes.begin(); lit != lNodes.end();) {
        if (lit->keys.size() == 1) { lit->bNoMore = true; ++lit; }
        else if (lit->keys.empty()) lit = lNodes.erase(lit);
        else ++lit;
    }
    bool bFinish = false;
    vector<SizeSerial> vSize;
    auto push_child = [&](Node& c, bool track, int* nToExpand) {
        c.serial = serial++;
        lNodes.push_front(c);
        if (c.keys.size() > 1) {
            if (nToExpand) (*nToExpand)++;
            if (track) {
                vSize.push_back(SizeSerial{(int)c.keys.size(), lNodes.front().serial, &lNodes.front()});
                lNodes.front().lit = lNodes.begin();
            }
        }
    };
    while (!bFinish) {
        int prevSize = (int)lNodes.size();
        auto lit = lNodes.begin();
        int nToExpand = 0;
        vSize.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) { ++lit; continue; }
            Node n1, n2, n3, n4;
            divide_node(*lit, n1, n2, n3, n4);
            if (!n1.keys.empty()) push_child(n1, true, &nToExpand);
            if (!n2.keys.empty()) push_child(n2, true, &nToExpand);
            if (!n3.keys.empty()) push_child(n3, true, &nToExpand);
            if (!n4.keys.empty()) push_child(n4, true, &nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if (((int)lNodes.size() + nToExpand * 3) > N) {
            while (!bFinish) {
                prevSize = (int)lNodes.size();
                vector<SizeSerial> vPrev = vSize;
                vSize.clear();
                std::sort(vPrev.begin(), vPrev.end());
                for (int j = (int)vPrev.size() - 1; j >= 0; j--) {
                    Node n1, n2, n3, n4;
                    divide_node(*vPrev[j].node, n1, n2, n3, n4);
                    if (!n1.keys.empty()) push_child(n1, true, nullptr);
                    if (!n2.keys.empty()) push_child(n2, true, nullptr);
                    if (!n3.keys.empty()) push_child(n3, true, nullptr);
                    if (!n4.keys.empty()) push_child(n4, true, nullptr);
                    lNodes.erase(vPrev[j].node->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }
    vector<KP> res;
    res.reserve(lNodes.size());
    for (auto& nd : lNodes) {
        const KP* p = &nd.keys[0];
        float maxResponse = p->response;
        for (size_t k = 1; k < nd.keys.size(); k++)
            if (nd.keys[k].response > maxResponse) { p = &nd.keys[k]; maxResponse = p->response; }
        res.push_back(*p);
    }
    return res;
}

// ---------------------------------------------------------------------------
// a8  OCV:core mathfuncs_core atan_f32 (cv::fastAtan2) and U:src/ORBextractor.cc::IC_Angle
// ---------------------------------------------------------------------------
static const float atan2_p1 = 0.9997878412794807f * (float)(180 / M_PI);
static const float atan2_p3 = -0.3258083974640975f * (float)(180 / M_PI);
static const float atan2_p5 = 0.1555786518463281f * (float)(180 / M_PI);
static const float atan2_p7 = -0.04432655554792128f * (float)(180 / M_PI);

float fastAtan2(float y, float x) {
    float ax = std::abs(x), ay = std::abs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

static float ic_angle(const Img& im, float px, float py, const vector<int>& u_max) {
    int m_01 = 0, m_10 = 0;
    const int HALF = 15;
    const uint8_t* center = im.row(cvRound(py)) + cvRound(px);
    for (int u = -HALF; u <= HALF; ++u) m_10 += u * center[u];
    const int step = im.w;
    for (int v = 1; v <= HALF; ++v) {
        int v_sum = 0;
        int d = u_max[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * step], val_minus = center[u - v * step];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return fastAtan2((float)m_01, (float)m_10);
}

// ---------------------------------------------------------------------------
// a9  OCV:imgproc/src/smooth.dispatch.cpp GaussianBlur(7x7, sigma 2, REFLECT_101),
//     bit-exact fixed-point path: getGaussianKernelBitExact + fixed-point ED.
// ---------------------------------------------------------------------------
void gaussian_kernel_fixed(int n, double sigma, int out[]) {
    // getGaussianKernelBitExact (softdouble) then getGaussianKernelFixedPoint_ED, 8 frac bits
    const int n2 = (n - 1) / 2;
    vector<double> values(n2 + 1);
    double scale2X = -0.125 / (sigma * sigma);
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        double t = std::exp((double)(x * x) * scale2X);
        values[i] = t;
        sum += t;
    }
    sum *= 2;
    sum += 1.0;
    double mul1 = 1.0 / sum;
    vector<double> k(n);
    for (int i = 0; i < n2; i++) k[i] = k[n - 1 - i] = values[i] * mul1;
    k[n2] = mul1;
    double err = 0;
    long s = 0;
    for (int i = 0; i < n2; i++) {
        double adj = k[i] * 256.0 + err;
        long v0 = cvRoundD(adj);
        err = adj - (double)v0;
        out[i] = out[n - 1 - i] = (int)v0;
        s += v0;
    }
    out[n2] = (int)(256 - 2 * s);
}

static inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

static void gaussian_blur_7x7(const Img& src, Img& dst) {
    int k[7];
    gaussian_kernel_fixed(7, 2.0, k);
    const int w = src.w, h = src.h;
    vector<uint32_t> hrow((size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint32_t s = 0;
            for (int i = 0; i < 7; i++) s += (uint32_t)k[i] * src.row(y)[reflect101(x + i - 3, w)];
            hrow[(size_t)y * w + x] = s;   // ufixedpoint16, 8 fractional bits (exact)
        }
    dst.w = w; dst.h = h; dst.d.assign((size_t)w * h, 0);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint32_t s = 0;
            for (int j = 0; j < 7; j++) s += (uint32_t)k[j] * hrow[(size_t)reflect101(y + j - 3, h) * w + x];
            dst.row(y)[x] = sat_u8((int)((s + (1u << 15)) >> 16));
        }
}

// U:src/ORBextractor.cc::computeOrbDescriptor — std::cos/std::sin(float) = glibc cosf/sinf
static void orb_descriptor(const KP& kp, const Img& img, uint8_t* desc) {
    const float factorPI = (float)(M_PI / 180.f);
    float angle = (float)kp.angle * factorPI;
    float a = (float)std::cos(angle), b = (float)std::sin(angle);
    const uint8_t* center = img.row(cvRound(kp.y)) + cvRound(kp.x);
    const int step = img.w;
    const signed char* pattern = ORBHIP_BIT_PATTERN_31;
    auto get = [&](int idx) {
        float px = pattern[2 * idx], py = pattern[2 * idx + 1];
        return (int)center[cvRound(px * b + py * a) * step + cvRound(px * a - py * b)];
    };
    for (int i = 0; i < 32; ++i, pattern += 32) {
        int val = 0;
        for (int bit = 0; bit < 8; bit++) {
            int t0 = get(2 * bit), t1 = get(2 * bit + 1);
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

// ---------------------------------------------------------------------------
// a5  U:src/ORBextractor.cc::ComputeKeyPointsOctTree
// ---------------------------------------------------------------------------
static void compute_keypoints_octtree(Extractor& E, vector<vector<KP>>& all, vector<vector<KP>>* cand_out) {
    all.assign(E.nlevels, {});
    if (cand_out) cand_out->assign(E.nlevels, {});
    const int EDGE_THRESHOLD = 19, PATCH_SIZE = 31;
    const float W = 35;
    for (int level = 0; level < E.nlevels; ++level) {
        const Img& L = E.pyr[level];
        const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
        const int maxBorderX = L.w - EDGE_THRESHOLD + 3, maxBorderY = L.h - EDGE_THRESHOLD + 3;
        vector<KP> toDistribute;
        const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
        const int nCols = (int)(width / W), nRows = (int)(height / W);
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(minBorderY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minBorderX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                vector<KP> cell;
                const uint8_t* base = L.row((int)iniY) + (int)iniX;
                fast16(base, L.w, (int)maxY - (int)iniY, (int)maxX - (int)iniX, cell, E.iniThFAST);
                if (cell.empty()) fast16(base, L.w, (int)maxY - (int)iniY, (int)maxX - (int)iniX, cell, E.minThFAST);
                for (KP& kp : cell) {
                    kp.x += j * wCell;
                    kp.y += i * hCell;
                    toDistribute.push_back(kp);
                }
            }
        }
        if (cand_out) (*cand_out)[level] = toDistribute;
        vector<KP>& kps = all[level];
        if (!toDistribute.empty())
            kps = distribute_octtree(toDistribute, minBorderX, maxBorderX, minBorderY, maxBorderY,
                                     E.mnFeaturesPerLevel[level]);
        const int scaledPatchSize = (int)(PATCH_SIZE * E.mvScaleFactor[level]);
        for (KP& kp : kps) {
            kp.x += minBorderX;
            kp.y += minBorderY;
            kp.octave = level;
            kp.size = (float)scaledPatchSize;
        }
    }
    for (int level = 0; level < E.nlevels; ++level)
        for (KP& kp : all[level]) kp.angle = ic_angle(E.pyr[level], kp.x, kp.y, E.umax);
}

// a2  U:src/ORBextractor.cc::ORBextractor::operator()
static int extract(Extractor& E, const uint8_t* img, int w, int h, int stride, int lap0, int lap1,
                   vector<KP>& out, vector<uint8_t>& desc, vector<vector<KP>>* cand_out,
                   vector<vector<KP>>* level_out) {
    out.clear();
    desc.clear();
    if (!img || w <= 0 || h <= 0) return -1;
    if (!compute_pyramid(E, img, w, h, stride)) return -2;
    vector<vector<KP>> all;
    compute_keypoints_octtree(E, all, cand_out);
    if (level_out) *level_out = all;
    int nk = 0;
    for (auto& v : all) nk += (int)v.size();
    out.resize(nk);
    desc.assign((size_t)nk * 32, 0);
    int monoIndex = 0, stereoIndex = nk - 1;
    for (int level = 0; level < E.nlevels; ++level) {
        vector<KP>& kps = all[level];
        if (kps.empty()) continue;
        Img blurred;
        gaussian_blur_7x7(E.pyr[level], blurred);
        vector<uint8_t> ld(kps.size() * 32);
        for (size_t i = 0; i < kps.size(); i++) orb_descriptor(kps[i], blurred, &ld[i * 32]);
        float scale = E.mvScaleFactor[level];
        for (size_t i = 0; i < kps.size(); i++) {
            KP kp = kps[i];
            if (level != 0) { kp.x *= scale; kp.y *= scale; }
            int slot = (kp.x >= lap0 && kp.x <= lap1) ? stereoIndex-- : monoIndex++;
            out[slot] = kp;
            std::memcpy(&desc[(size_t)slot * 32], &ld[i * 32], 32);
        }
    }
    return monoIndex;
}

// ---------------------------------------------------------------------------
// a11/a12  U:src/ORBmatcher.cc::DescriptorDistance and the best/second + ratio +
// TH_LOW + rotation-histogram rule (SearchByBoW / SearchForInitialization acceptance)
// applied order-free over the whole train set (no greedy vnMatches21 pass).
// ---------------------------------------------------------------------------
int descriptor_distance(const uint8_t* a, const uint8_t* b) {
    const uint32_t* pa = (const uint32_t*)a;
    const uint32_t* pb = (const uint32_t*)b;
    int dist = 0;
    for (int i = 0; i < 8; i++, pa++, pb++) {
        unsigned int v = *pa ^ *pb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

static void compute_three_maxima(const vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s; ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

static int match_bf(const uint8_t* q, const float* q_angle, int nq, const uint8_t* t, const float* t_angle, int nt,
                    int th_low, float ratio, int check_orientation, int32_t* match, int32_t* best_d,
                    int32_t* second_d) {
    const int HISTO_LENGTH = 30;
    vector<int> rotHist[HISTO_LENGTH];
    const float factor = 1.0f / HISTO_LENGTH;
    int nmatches = 0;
    for (int i = 0; i < nq; i++) {
        int best = 256, second = 256, bidx = -1;   // SearchByBoW initialisation (256 == "none")
        for (int j = 0; j < nt; j++) {
            int d = descriptor_distance(q + (size_t)i * 32, t + (size_t)j * 32);
            if (d < best) { second = best; best = d; bidx = j; }
            else if (d < second) second = d;
        }
        best_d[i] = best;
        second_d[i] = second;
        match[i] = -1;
        if (bidx >= 0 && best <= th_low && (float)best < ratio * (float)second) {
            match[i] = bidx;
            nmatches++;
            if (check_orientation) {
                float rot = q_angle[i] - t_angle[bidx];
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                rotHist[bin].push_back(i);
            }
        }
    }
    if (check_orientation) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        compute_three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int idx : rotHist[i]) {
                if (match[idx] >= 0) { match[idx] = -1; nmatches--; }
            }
        }
    }
    return nmatches;
}

}  // namespace orc

// ===========================================================================
// extern "C" surface for ctypes (tests / bench cpu_baseline only)
// KP records are 6 floats: x, y, size, angle, response, octave(as float).
// ===========================================================================
extern "C" {

int orc_level_info(int w, int h, int nfeatures, float scaleFactor, int nlevels, int* lw, int* lh, int* feats,
                   float* scales, int* umax16) {
    orc::Extractor E(nfeatures, scaleFactor, nlevels, 20, 7);
    for (int l = 0; l < nlevels; l++) {
        float s = E.mvInvScaleFactor[l];
        lw[l] = orc::cvRound((float)w * s);
        lh[l] = orc::cvRound((float)h * s);
        feats[l] = E.mnFeaturesPerLevel[l];
        scales[l] = E.mvScaleFactor[l];
    }
    for (int v = 0; v < 16; v++) umax16[v] = E.umax[v];
    return 0;
}

static void put_kps(const std::vector<orc::KP>& v, float* out) {
    for (size_t i = 0; i < v.size(); i++) {
        out[6 * i + 0] = v[i].x; out[6 * i + 1] = v[i].y; out[6 * i + 2] = v[i].size;
        out[6 * i + 3] = v[i].angle; out[6 * i + 4] = v[i].response; out[6 * i + 5] = (float)v[i].octave;
    }
}

// Full ORBextractor::operator(). Returns monoIndex (>=0), -1 empty image, -2 unsupported,
// -3 capacity. kps: cap x 6 floats; desc: cap x 32 bytes.
int orc_extract(const uint8_t* img, int w, int h, int stride, int nfeatures, float scaleFactor, int nlevels,
                int iniTh, int minTh, int lap0, int lap1, float* kps, uint8_t* desc, int cap, int* n_out) {
    orc::Extractor E(nfeatures, scaleFactor, nlevels, iniTh, minTh);
    std::vector<orc::KP> out;
    std::vector<uint8_t> d;
    int mono = orc::extract(E, img, w, h, stride, lap0, lap1, out, d, nullptr, nullptr);
    *n_out = (int)out.size();
    if (mono < 0) { *n_out = 0; return mono; }
    if ((int)out.size() > cap) return -3;
    put_kps(out, kps);
    std::memcpy(desc, d.data(), d.size());
    return mono;
}

// Debug: pyramid images packed level after level (sizes from orc_level_info).
int orc_pyramid(const uint8_t* img, int w, int h, int stride, float scaleFactor, int nlevels, uint8_t* out) {
    orc::Extractor E(1000, scaleFactor, nlevels, 20, 7);
    if (!orc::compute_pyramid(E, img, w, h, stride)) return -2;
    size_t off = 0;
    for (int l = 0; l < nlevels; l++) {
        std::memcpy(out + off, E.pyr[l].d.data(), E.pyr[l].d.size());
        off += E.pyr[l].d.size();
    }
    return 0;
}

// Debug: per-level FAST candidates (pre-octree, cell-major) and per-level octree output
// (post-orientation, level coordinates). counts[2*l] = #cand, counts[2*l+1] = #kept.
int orc_extract_levels(const uint8_t* img, int w, int h, int stride, int nfeatures, float scaleFactor,
                       int nlevels, int iniTh, int minTh, float* cand, int cand_cap, float* kept, int kept_cap,
                       int* counts) {
    orc::Extractor E(nfeatures, scaleFactor, nlevels, iniTh, minTh);
    std::vector<orc::KP> out;
    std::vector<uint8_t> d;
    std::vector<std::vector<orc::KP>> c, k;
    int mono = orc::extract(E, img, w, h, stride, 0, 1000, out, d, &c, &k);
    if (mono < 0) return mono;
    int oc = 0, ok = 0;
    for (int l = 0; l < nlevels; l++) {
        counts[2 * l] = (int)c[l].size();
        counts[2 * l + 1] = (int)k[l].size();
        if (oc + (int)c[l].size() > cand_cap || ok + (int)k[l].size() > kept_cap) return -3;
        put_kps(c[l], cand + 6 * oc);
        put_kps(k[l], kept + 6 * ok);
        oc += (int)c[l].size();
        ok += (int)k[l].size();
    }
    return 0;
}

int orc_blur(const uint8_t* img, int w, int h, uint8_t* out) {
    orc::Img a, b;
    a.w = w; a.h = h; a.d.assign(img, img + (size_t)w * h);
    orc::gaussian_blur_7x7(a, b);
    std::memcpy(out, b.d.data(), b.d.size());
    return 0;
}

int orc_gaussian_kernel(int n, double sigma, int* out) { orc::gaussian_kernel_fixed(n, sigma, out); return 0; }

float orc_fast_atan2(float y, float x) { return orc::fastAtan2(y, x); }

int orc_corner_score(const uint8_t* patch7x7, int threshold) {
    int pixel[25];
    orc::makeOffsets16(pixel, 7);
    return orc::cornerScore16(patch7x7 + 3 * 7 + 3, pixel, threshold);
}

int orc_fast_window(const uint8_t* img, int step, int rows, int cols, int threshold, float* kps, int cap) {
    std::vector<orc::KP> v;
    orc::fast16(img, step, rows, cols, v, threshold);
    if ((int)v.size() > cap) return -3;
    put_kps(v, kps);
    return (int)v.size();
}

int orc_descriptor_distance(const uint8_t* a, const uint8_t* b) { return orc::descriptor_distance(a, b); }

// OCV imgproc/src/color_rgb.simd.hpp RGB2Gray<uchar> as reached by cv_bridge::toCvShare(msg,
// MONO8) on a bgr8 message (R:src/imu_mono_realsense.cpp:298): yuv_shift = 14, coefficients
// R2Y 4899, G2Y 9617, B2Y 1868; Y = (B*1868 + G*9617 + R*4899 + (1 << 13)) >> 14. The SIMD
// path uses the same integer dot product, so every pixel has one exact value.
void orc_bgr2gray(const uint8_t* bgr, int w, int h, int src_stride, uint8_t* gray, int dst_stride) {
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const uint8_t* p = bgr + (size_t)y * src_stride + 3 * x;
            gray[(size_t)y * dst_stride + x] = (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14);
        }
}

int orc_match_bf(const uint8_t* q, const float* q_angle, int nq, const uint8_t* t, const float* t_angle, int nt,
                 int th_low, float ratio, int check_orientation, int32_t* match, int32_t* best_d, int32_t* second_d) {
    return orc::match_bf(q, q_angle, nq, t, t_angle, nt, th_low, ratio, check_orientation, match, best_d, second_d);
}

}  // extern "C"

extern "C" {
// glibc cosf/sinf over the float bit range [lo, hi] (reference values for the device
// restatement's exhaustive check).
int orc_glibc_sincosf_range(uint32_t lo, uint32_t hi, float* c, float* s) {
    for (uint64_t u = lo; u <= hi; u++) {
        uint32_t v = (uint32_t)u;
        float x;
        std::memcpy(&x, &v, 4);
        c[u - lo] = cosf(x);
        s[u - lo] = sinf(x);
    }
    return 0;
}
}
