// liborbhip.so host side: contexts, per-size extraction plans, the C-ABI of include/orbhip.h.
//
// Plan construction restates the table logic of the reference (it is the product's own
// code, not the oracle's):
//   U:src/ORBextractor.cc::ORBextractor::ORBextractor  scale / feature / umax tables
//   U:src/ORBextractor.cc::ComputePyramid               level sizes
//   OCV:imgproc/src/resize.cpp hal::resize              xofs/alpha/yofs/beta fixed-point tables
//   U:src/ORBextractor.cc::ComputeKeyPointsOctTree      35-px cell grid
//   U:src/ORBextractor.cc::DistributeOctTree            root count nIni, root width hX
//   OCV:imgproc smooth.dispatch.cpp getGaussianKernelBitExact + fixed-point ED  (7x7, sigma 2)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#include "../../include/orbhip.h"
#include "dev_attr.h"
#include "orbhip_ba.h"
#include "pose_opt.h"
#include "proj.h"
#include "kfdb.h"
#include "ba_chol_blocked.h"
#include "ba_chol_dag.h"
#include "ba_nd.h"
#include "orbhip_kernels.h"
#include "orbhip_plan.h"
#include "graph_cache.h"

using namespace orbhip;

#define HIPOK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "orbhip: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_),     \
                         __FILE__, __LINE__);                                                      \
            return ORBHIP_ERR_DEVICE;                                                              \
        }                                                                                          \
    } while (0)

namespace {

inline int round_even_f(float v) { return (int)std::nearbyintf(v); }
inline int round_even_d(double v) { return (int)std::nearbyint(v); }
inline int floor_f(float v) { int i = (int)v; return i - (i > v); }
inline short sat_s16(int v) { return (short)std::min(std::max(v, -32768), 32767); }

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t ensure(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; n = 0; }
        hipError_t e = hipMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
};

constexpr int kConeHiStart = 2;        // batches: k_resize for levels 1..2, one cone launch for the rest
// threads per batch-cone tile: ORBHIP_CONE_HI_THREADS (256 / 512 / 1024), else 256
static int cone_hi_threads() {
    static const int t = std::getenv("ORBHIP_CONE_HI_THREADS") ? std::atoi(std::getenv("ORBHIP_CONE_HI_THREADS")) : 256;
    return (t == 512 || t == 1024) ? t : 256;
}

constexpr int kBandStart = 2;   // batches: k_resize for levels 1..2, k_resize_bands for the rest
// row bands per frame of k_resize_bands: ORBHIP_RZ_BANDS (read per plan lookup), default 0 =
// every level by k_resize. Opt-in: at C3 the band launch measured 400-1200 us for 8-64 bands
// against the 95 us of the five k_resize launches it replaces (tools/c3_pyr_sweep.sh)
static int rz_bands() {
    const char* e = std::getenv("ORBHIP_RZ_BANDS");
    return e ? std::max(0, std::atoi(e)) : 0;
}

struct Plan {
    ExtractPlan h{};
    std::vector<CellGeom> cells;
    std::vector<int> xofs, xalpha, yofs, ybeta, disc;
    std::vector<ConeRect> cone;   // k_pyr_cone tables (empty: per-level k_resize cascade)
    std::vector<int> cone_tab;    // per tile: every level's resize tables in the kernel's LDS layout
    int cone_tab_stride = 0;
    int cone_tiles = 0;
    size_t cone_lds = 0;
    DevBuf<ConeRect> d_cone;
    DevBuf<int> d_cone_tab;
    // the same for batches: levels kConeHiStart+1..L-1 in one launch behind the first
    // kConeHiStart k_resize levels (empty: all levels by k_resize)
    std::vector<ConeRect> cone_hi;
    std::vector<int> cone_hi_tab;
    int cone_hi_tab_stride = 0, cone_hi_tiles = 0;
    size_t cone_hi_lds = 0;
    DevBuf<ConeRect> d_cone_hi;
    DevBuf<int> d_cone_hi_tab;
    // batches: levels kBandStart+1..L-1 by k_resize_bands, the output rows of each (band, level)
    std::vector<int> bands;   // [nbands][kMaxLevels] (r0, r1) pairs
    int nbands = 0;
    DevBuf<int> d_bands;
    // batches: k_pyr_flow's 16-row bands (level 1 first), the level l-1 bands each band's source
    // rows lie in
    int flow_boff[kMaxLevels + 1] = {0};
    int flow_nbt = 0;
    std::vector<int> flow_dep;   // (b0, b1) per band
    DevBuf<int> d_flow_dep;
    OctreeCfg oct{};
    int kp_cap_frame = 0;   // sum of level caps = max keypoints per frame
    DevBuf<ExtractPlan> d_plan;
    DevBuf<CellGeom> d_cells;
    DevBuf<int> d_xofs, d_xalpha, d_yofs, d_ybeta, d_disc;
    std::vector<uint16_t> otab;   // k_octree interval tables (LevelGeom::oct_tab_off)
    DevBuf<uint16_t> d_otab;
};

}  // namespace

// A plan depends only on the device, the frame size, the ORBextractor parameters, the cone tile
// and the test switches read while building it, never on a context's buffers: contexts with the
// same key (e.g. the 16 camera streams of the C2 bench) share one, so its tables (the cone's
// per-tile resize tables are ~0.5 MB at 640x480) stay L2-resident once instead of once per
// context. The cache holds weak references: a plan dies with the last context using it.
struct PlanKey {
    int device, w, h, nfeat, nlev, ini, mn, cone_tile, clist_cap, fast_nt, cone_hi_tile, rz_bands;
    float scale;
    bool operator<(const PlanKey& o) const {
        return std::memcmp(this, &o, sizeof(PlanKey)) < 0;
    }
};
struct orbhip_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    orbhip_orb_params prm{};
    // ORBextractor ctor tables
    std::vector<float> scale, inv_scale;
    std::vector<int> feat, umax;
    int blurk[7] = {0};
    std::map<PlanKey, std::shared_ptr<Plan>> plans;   // shared with other contexts (plan_cache)
    // per-batch scratch (grown on demand)
    DevBuf<uint8_t> d_in, d_pyr;
    DevBuf<uint32_t> d_cand, d_kscratch;
    DevBuf<uint32_t> d_cprim;   // FAST candidates' primary slots (kCandPrim per cell)
    DevBuf<uint16_t> d_nscratch;
    DevBuf<int> d_cand_cnt, d_lvl_cnt, d_lvl_nlap, d_err;
    DevBuf<int> d_cand_off, d_cand_fill;   // packed FAST candidates (batches, CandPack)
    DevBuf<int> d_flow;         // k_pyr_flow: kFlowCtl control words + B x nbt band flags, zeroed when (re)allocated
    DevBuf<uint64_t> d_mpart;   // matcher chunk partials (match_part_entries)
    DevBuf<int> d_msync;        // one-launch matcher counters (zeroed once, reset by every launch)
    DevBuf<double> d_bw;        // bag-of-words weights (host transform)
    DevBuf<uint8_t> d_bow_stage;   // SearchByBoW host-call staging
    DevBuf<LevelKp> d_lvl_kp;
    DevBuf<orbhip_kp> d_kps;
    DevBuf<uint8_t> d_desc;
    DevBuf<int32_t> d_n, d_mono;
    // matcher scratch
    DevBuf<uint8_t> d_mq, d_mt;
    DevBuf<float> d_mqa, d_mta;
    DevBuf<int32_t> d_mm, d_mb, d_ms, d_mn;
    BaWorkspace* ba = nullptr;
    PoseWorkspace* pose = nullptr;
    ProjWorkspace* proj = nullptr;
    StageTimer timer;
    GraphCache graphs;   // replays of repeated per-frame launch sequences (graph_cache.h)
    int cone_tile = 0;   // k_pyr_cone tile edge in last-level pixels (0: 10, the one-frame latency optimum)
    int fast_nt = 0;     // k_fast_cells threads per cell hint (0: by batch size; 128/256/512/1024)
};

// ---------------------------------------------------------------------------
// ORBextractor ctor tables
// ---------------------------------------------------------------------------
static void build_orb_tables(orbhip_ctx* c) {
    const int L = c->prm.n_levels;
    const double sf = (double)c->prm.scale_factor;
    c->scale.assign(L, 1.f);
    c->inv_scale.assign(L, 1.f);
    for (int i = 1; i < L; i++) c->scale[i] = (float)(c->scale[i - 1] * sf);
    for (int i = 0; i < L; i++) c->inv_scale[i] = 1.0f / c->scale[i];
    c->feat.assign(L, 0);
    const float factor = (float)(1.0f / sf);
    float nd = c->prm.n_features * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; l++) {
        c->feat[l] = round_even_f(nd);
        sum += c->feat[l];
        nd *= factor;
    }
    c->feat[L - 1] = std::max(c->prm.n_features - sum, 0);
    // umax (HALF_PATCH_SIZE 15)
    const int H = 15;
    c->umax.assign(H + 1, 0);
    int vmax = (int)std::floor(H * std::sqrt(2.f) / 2 + 1);
    int vmin = (int)std::ceil(H * std::sqrt(2.f) / 2);
    const double hp2 = H * H;
    for (int v = 0; v <= vmax; ++v) c->umax[v] = round_even_d(std::sqrt(hp2 - v * v));
    for (int v = H, v0 = 0; v >= vmin; --v) {
        while (c->umax[v0] == c->umax[v0 + 1]) ++v0;
        c->umax[v] = v0;
        ++v0;
    }
    // bit-exact 7-tap Gaussian, sigma 2, 8 fractional bits, error diffusion
    const int n = 7, n2 = 3;
    double vals[3], s = 0, scale2X = -0.125 / (2.0 * 2.0);
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) { vals[i] = std::exp((double)(x * x) * scale2X); s += vals[i]; }
    s = s * 2 + 1.0;
    const double mul1 = 1.0 / s;
    double err = 0;
    long tot = 0;
    for (int i = 0; i < n2; i++) {
        double adj = vals[i] * mul1 * 256.0 + err;
        long v0 = round_even_d(adj);
        err = adj - (double)v0;
        c->blurk[i] = c->blurk[n - 1 - i] = (int)v0;
        tot += v0;
    }
    c->blurk[n2] = (int)(256 - 2 * tot);
}

// ---------------------------------------------------------------------------
// per-size plan
// ---------------------------------------------------------------------------
static std::mutex g_plan_m;
static std::map<PlanKey, std::weak_ptr<Plan>>& plan_cache() {
    static auto* m = new std::map<PlanKey, std::weak_ptr<Plan>>();   // never destroyed (exit order)
    return *m;
}
static int build_plan_new(orbhip_ctx* c, int w, int h, std::shared_ptr<Plan>& out);

// k_pyr_cone tile edge of a plan: ORBHIP_CONE_TILE (read per plan lookup, A/B and tests), else
// the context's choice, else 10 (the one-frame latency optimum)
static int cone_tile_of(const orbhip_ctx* c) {
    const char* e = std::getenv("ORBHIP_CONE_TILE");
    const int ts_env = e ? std::atoi(e) : 0;
    return ts_env > 0 ? ts_env : (c->cone_tile > 0 ? c->cone_tile : 10);
}

// the batch cone's tile edge (last-level pixels): ORBHIP_CONE_HI_TILE (read per plan lookup), else 32
static int cone_hi_tile_of() {
    const char* e = std::getenv("ORBHIP_CONE_HI_TILE");
    return e ? std::max(4, std::atoi(e)) : 32;
}

// k_pyr_cone tables from source level s0 (0: the frame): tiles of ts x ts pixels of the last
// level, every level l > s0 cut into the same tile grid (an even partition, the tile's owned
// pixels) plus the halo its level l+1 need reads (the need), the source level's need staged.
// Returns the tile count; rects (kMaxLevels per tile), the per-tile resize tables in the kernel's
// LDS layout (row indices clamped to the source), their stride, and the LDS bytes of the largest.
static int cone_tables(const ExtractPlan& P, const Plan& pl, int s0, int ts, std::vector<ConeRect>& rects,
                       std::vector<int>& ctab, size_t& tab_stride, size_t& lds_max) {
    const int L = P.n_levels;
    const LevelGeom& T = P.lv[L - 1];
    const int ntx = (T.w + ts - 1) / ts, nty = (T.h + ts - 1) / ts;
    lds_max = 0;
    rects.assign((size_t)ntx * nty * kMaxLevels, ConeRect{});
    // the source rectangle of level l's need [nx0, nx1) x [ny0, ny1) on level l - 1
    auto source_of = [&](int l, int nx0, int nx1, int ny0, int ny1, int* a0, int* a1, int* b0, int* b1) {
        const LevelGeom& U = P.lv[l];
        const LevelGeom& G = P.lv[l - 1];
        *a0 = pl.xofs[U.xtab_off + nx0];
        *a1 = pl.xofs[U.xtab_off + nx1 - 1] + ((nx1 - 1) < U.xmax ? 1 : 0) + 1;
        auto clampr = [&](int r) { return r < 0 ? 0 : (r < G.h ? r : G.h - 1); };
        *b0 = clampr(pl.yofs[U.ytab_off + ny0]);
        *b1 = clampr(pl.yofs[U.ytab_off + ny1 - 1] + 1) + 1;
    };
    for (int ti = 0; ti < nty; ti++)
        for (int tj = 0; tj < ntx; tj++) {
            ConeRect* R = &rects[((size_t)ti * ntx + tj) * kMaxLevels];
            int nx0 = 0, nx1 = 0, ny0 = 0, ny1 = 0;   // need of the level above (l + 1)
            for (int l = L - 1; l > s0; l--) {
                const LevelGeom& G = P.lv[l];
                const int ox0 = (int)((int64_t)tj * G.w / ntx), ox1 = (int)((int64_t)(tj + 1) * G.w / ntx);
                const int oy0 = (int)((int64_t)ti * G.h / nty), oy1 = (int)((int64_t)(ti + 1) * G.h / nty);
                int a0 = ox0, a1 = ox1, b0 = oy0, b1 = oy1;
                if (l < L - 1 && nx1 > nx0 && ny1 > ny0) {   // inputs of the level-(l+1) need
                    int lo, hi, r0, r1;
                    source_of(l + 1, nx0, nx1, ny0, ny1, &lo, &hi, &r0, &r1);
                    a0 = std::min(a0, lo); a1 = std::max(a1, hi);
                    b0 = std::min(b0, r0); b1 = std::max(b1, r1);
                    if (ox1 <= ox0 || oy1 <= oy0) { a0 = lo; a1 = hi; b0 = r0; b1 = r1; }
                }
                R[l] = ConeRect{(int16_t)a0, (int16_t)a1, (int16_t)b0, (int16_t)b1,
                                (int16_t)ox0, (int16_t)ox1, (int16_t)oy0, (int16_t)oy1};
                nx0 = a0; nx1 = a1; ny0 = b0; ny1 = b1;
            }
            {   // source-level inputs of the level-(s0+1) need (staged in LDS)
                int lo, hi, r0, r1;
                source_of(s0 + 1, nx0, nx1, ny0, ny1, &lo, &hi, &r0, &r1);
                R[s0] = ConeRect{(int16_t)lo, (int16_t)hi, (int16_t)r0, (int16_t)r1, 0, 0, 0, 0};
            }
            size_t tot = 0, ttot = 0;
            for (int l = s0; l < L; l++) {   // source: rows of round_up(width + 3, 4) (dword staging)
                const size_t wl = l == s0 ? (size_t)((R[s0].nx1 - R[s0].nx0 + 6) & ~3) : (size_t)(R[l].nx1 - R[l].nx0);
                tot += (wl * (R[l].ny1 - R[l].ny0) + 15) & ~size_t(15);
            }
            for (int l = s0 + 1; l < L; l++)
                ttot += 4 * (2 * (size_t)(R[l].nx1 - R[l].nx0) + 3 * (size_t)(R[l].ny1 - R[l].ny0));
            lds_max = std::max(lds_max, tot + ttot);
        }
    tab_stride = 0;
    for (int t = 0; t < ntx * nty; t++) {
        size_t tt = 0;
        for (int l = s0 + 1; l < L; l++) {
            const ConeRect& r = rects[(size_t)t * kMaxLevels + l];
            tt += 2 * (size_t)(r.nx1 - r.nx0) + 3 * (size_t)(r.ny1 - r.ny0);
        }
        tab_stride = std::max(tab_stride, tt);
    }
    ctab.assign((size_t)ntx * nty * tab_stride, 0);
    for (int t = 0; t < ntx * nty; t++) {
        int* o = ctab.data() + (size_t)t * tab_stride;
        for (int l = s0 + 1; l < L; l++) {
            const LevelGeom& D = P.lv[l];
            const LevelGeom& S = P.lv[l - 1];
            const ConeRect r = rects[(size_t)t * kMaxLevels + l];
            const int nw = r.nx1 - r.nx0, nh = r.ny1 - r.ny0;
            for (int i = 0; i < nw; i++) {
                o[i] = pl.xofs[D.xtab_off + r.nx0 + i];
                o[nw + i] = pl.xalpha[D.xtab_off + r.nx0 + i];
            }
            auto clampr = [&](int v) { return v < 0 ? 0 : (v < S.h ? v : S.h - 1); };
            for (int j = 0; j < nh; j++) {
                const int sy = pl.yofs[D.ytab_off + r.ny0 + j];
                o[2 * nw + 3 * j] = clampr(sy);
                o[2 * nw + 3 * j + 1] = clampr(sy + 1);
                o[2 * nw + 3 * j + 2] = pl.ybeta[D.ytab_off + r.ny0 + j];
            }
            o += 2 * nw + 3 * nh;
        }
    }
    return ntx * nty;
}

static int build_plan(orbhip_ctx* c, int w, int h, Plan** out) {
    // the context's cache is keyed by the full PlanKey, so an env switch read here
    // (ORBHIP_CONE_TILE / ORBHIP_CONE_HI_TILE / ORBHIP_FAST_CLIST_CAP / ORBHIP_FAST_NT) takes
    // effect on an existing context too
    const char* cap_env = getenv("ORBHIP_FAST_CLIST_CAP");
    const char* nt_env = getenv("ORBHIP_FAST_NT");
    PlanKey k;
    std::memset(&k, 0, sizeof(k));
    k.device = c->device; k.w = w; k.h = h; k.nfeat = c->prm.n_features; k.nlev = c->prm.n_levels;
    k.ini = c->prm.ini_th_fast; k.mn = c->prm.min_th_fast; k.scale = c->prm.scale_factor;
    k.cone_tile = cone_tile_of(c);
    k.clist_cap = cap_env ? atoi(cap_env) : -1;
    k.fast_nt = nt_env ? atoi(nt_env) : -1;
    k.cone_hi_tile = cone_hi_tile_of();
    k.rz_bands = rz_bands();
    auto it = c->plans.find(k);
    if (it != c->plans.end()) { *out = it->second.get(); return ORBHIP_OK; }
    std::lock_guard<std::mutex> g(g_plan_m);
    std::shared_ptr<Plan> sp = plan_cache()[k].lock();
    if (!sp) {
        if (int rc = build_plan_new(c, w, h, sp)) return rc;
        plan_cache()[k] = sp;
    }
    *out = sp.get();
    c->plans[k] = sp;
    return ORBHIP_OK;
}

static int build_plan_new(orbhip_ctx* c, int w, int h, std::shared_ptr<Plan>& out) {
    std::unique_ptr<Plan> pl(new Plan());
    ExtractPlan& P = pl->h;
    const int L = c->prm.n_levels;
    P.w = w; P.h = h; P.n_levels = L;
    P.ini_th = std::min(std::max(c->prm.ini_th_fast, 0), 255);
    P.min_th = std::min(std::max(c->prm.min_th_fast, 0), 255);
    // ORBHIP_FAST_CLIST_CAP lowers the survivor list (tests force the dense FAST pass with 0)
    const char* cap_env = getenv("ORBHIP_FAST_CLIST_CAP");   // read per plan (once per ctx and size)
    P.clist_cap = cap_env ? std::min(std::max(atoi(cap_env), 0), kClistCap) : kClistCap;
    // ORBHIP_FAST_NT pins k_fast_cells' threads per cell (A/B and tests; read per plan like the cap):
    // 128, 256, 512 or 1024; any other value is rejected loudly and the batch-size choice stays
    P.fast_nt = 0;
    if (const char* nt_env = getenv("ORBHIP_FAST_NT")) {
        const int v = atoi(nt_env);
        if (v == 128 || v == 256 || v == 512 || v == 1024) P.fast_nt = v;
        else std::fprintf(stderr, "orbhip: ORBHIP_FAST_NT=%s ignored (128, 256, 512 or 1024)\n", nt_env);
    }
    for (int i = 0; i < 7; i++) P.blurk[i] = c->blurk[i];
    // k_desc hard-codes these taps (GaussianBlur 7x7 sigma 2 is fixed in ORBextractor)
    static const int kTaps[7] = {18, 34, 48, 56, 48, 34, 18};
    for (int i = 0; i < 7; i++)
        if (P.blurk[i] != kTaps[i]) return ORBHIP_ERR_UNSUPPORTED;
    int64_t pyr_off = 0;
    int cell_base = 0, slot_base = 0, kp_base = 0, max_cells = 0, hc_max = 7, wc_max = 7;
    for (int l = 0; l < L; l++) {
        LevelGeom& G = P.lv[l];
        G.w = round_even_f((float)w * c->inv_scale[l]);
        G.h = round_even_f((float)h * c->inv_scale[l]);
        if (G.w < 64 || G.h < 64) return ORBHIP_ERR_UNSUPPORTED;   // every level must host 43x43 patches
        G.pitch = l == 0 ? 0 : ((G.w + 63) / 64) * 64;
        G.pyr_off = l == 0 ? 0 : pyr_off;
        if (l > 0) pyr_off += (int64_t)G.pitch * G.h;
        G.scale = c->scale[l];
        G.n_feat = c->feat[l];
        G.patch_size = (int)(31 * c->scale[l]);
        // resize tables (level l from l-1); each level's column table starts 16-byte aligned and
        // is padded, so k_resize reads 4 consecutive entries as one int4
        while (pl->xofs.size() % 4) { pl->xofs.push_back(0); pl->xalpha.push_back(0); }
        G.xtab_off = (int)pl->xofs.size();
        G.ytab_off = (int)pl->yofs.size();
        G.xmax = G.w;
        G.vend = 0;
        G.rz_noclamp = 1;
        // |p| <= 255 and taps a0, a1, b0, b1 >= 0 with a0 + a1, b0 + b1 <= 2049 keep every
        // intermediate of the vertical pass in range: (255 * 2049) >> 4 < 32768, and the rounded
        // sum (t + 2) >> 2 <= 255
        auto taps_ok = [](int packed) {
            const int t0 = (int)(short)(packed & 0xFFFF), t1 = (int)(short)(packed >> 16);
            return t0 >= 0 && t1 >= 0 && t0 + t1 <= 2049;
        };
        if (l > 0) {
            const int sw = P.lv[l - 1].w, sh = P.lv[l - 1].h, dw = G.w, dh = G.h;
            double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
            double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
            int isx = round_even_d(scale_x), isy = round_even_d(scale_y);
            if (std::abs(scale_x - isx) < DBL_EPSILON && std::abs(scale_y - isy) < DBL_EPSILON && isx == 2 && isy == 2)
                return ORBHIP_ERR_UNSUPPORTED;   // OpenCV switches to INTER_AREA for exact 2x
            int xmax = dw;
            for (int dx = 0; dx < dw; dx++) {
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = floor_f(fx);
                fx -= sx;
                if (sx < 0) { fx = 0; sx = 0; }
                if (sx + 1 >= sw) {
                    xmax = std::min(xmax, dx);
                    if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
                }
                pl->xofs.push_back(sx);
                const short a0 = sat_s16(round_even_f((1.f - fx) * 2048)), a1 = sat_s16(round_even_f(fx * 2048));
                pl->xalpha.push_back((int)(uint16_t)a0 | ((int)(uint16_t)a1 << 16));
                if (!taps_ok(pl->xalpha.back())) G.rz_noclamp = 0;
            }
            for (int dy = 0; dy < dh; dy++) {
                float fy = (float)((dy + 0.5) * scale_y - 0.5);
                int sy = floor_f(fy);
                fy -= sy;
                pl->yofs.push_back(sy);
                const short b0 = sat_s16(round_even_f((1.f - fy) * 2048)), b1 = sat_s16(round_even_f(fy * 2048));
                pl->ybeta.push_back((int)(uint16_t)b0 | ((int)(uint16_t)b1 << 16));
                if (!taps_ok(pl->ybeta.back())) G.rz_noclamp = 0;
            }
            G.xmax = xmax;
            int x = 0;
            for (; x <= dw - 16; x += 16) {}
            for (; x < dw - 8; x += 8) {}
            G.vend = x;
        }
        // cells (ComputeKeyPointsOctTree)
        const int EDGE = 19;
        G.min_bx = EDGE - 3; G.min_by = EDGE - 3;
        G.max_bx = G.w - EDGE + 3; G.max_by = G.h - EDGE + 3;
        const float width = (float)(G.max_bx - G.min_bx), height = (float)(G.max_by - G.min_by);
        G.n_cols = (int)(width / 35.f);
        G.n_rows = (int)(height / 35.f);
        if (G.n_cols <= 0 || G.n_rows <= 0) return ORBHIP_ERR_UNSUPPORTED;
        G.w_cell = (int)std::ceil(width / G.n_cols);
        G.h_cell = (int)std::ceil(height / G.n_rows);
        G.cell_base = cell_base;
        G.slot_base = slot_base;
        int ncell = 0;
        for (int i = 0; i < G.n_rows; i++) {
            const float iniY = (float)(G.min_by + i * G.h_cell);
            float maxY = iniY + G.h_cell + 6;
            const bool skipY = iniY >= G.max_by - 3;
            if (maxY > G.max_by) maxY = (float)G.max_by;
            for (int j = 0; j < G.n_cols; j++) {
                const float iniX = (float)(G.min_bx + j * G.w_cell);
                float maxX = iniX + G.w_cell + 6;
                const bool skipX = iniX >= G.max_bx - 6;
                if (maxX > G.max_bx) maxX = (float)G.max_bx;
                CellGeom cg{};
                cg.level = (int16_t)l;
                cg.x0 = (int16_t)iniX; cg.y0 = (int16_t)iniY;
                cg.wc = (skipY || skipX) ? 0 : (int16_t)((int)maxX - (int)iniX);
                cg.hc = (skipY || skipX) ? 0 : (int16_t)((int)maxY - (int)iniY);
                if (cg.wc > 76 || cg.hc > 76) return ORBHIP_ERR_UNSUPPORTED;
                cg.slot_off = slot_base;
                const int dc = std::max(cg.wc - 6, 0), dr = std::max(cg.hc - 6, 0);
                slot_base += ((dc + 1) / 2) * ((dr + 1) / 2);   // max strict-NMS survivors
                if (cg.wc > 6 && cg.hc > 6) {   // cells k_fast_cells works on
                    hc_max = std::max(hc_max, (int)cg.hc);
                    wc_max = std::max(wc_max, (int)cg.wc);
                }
                pl->cells.push_back(cg);
                ncell++;
            }
        }
        G.n_cells = ncell;
        G.n_slots = slot_base - G.slot_base;
        cell_base += ncell;
        max_cells = std::max(max_cells, ncell);
        // DistributeOctTree roots
        G.n_ini = (int)std::round((float)(G.max_bx - G.min_bx) / (G.max_by - G.min_by));
        if (G.n_ini <= 0 || G.n_ini > 64) return ORBHIP_ERR_UNSUPPORTED;
        G.hX = (float)(G.max_bx - G.min_bx) / G.n_ini;
        G.kp_cap = G.n_feat + 3 + 4 * G.n_ini;
        G.kp_base = kp_base;
        kp_base += G.kp_cap;
        if ((G.max_bx - G.min_bx) >= 4096 || (G.max_by - G.min_by) >= 4096) return ORBHIP_ERR_UNSUPPORTED;
        // k_octree interval tables: the first 6 quadrant splits of DistributeOctTree's root
        // rectangles (DivideNode: halfX = ceil((UR.x - UL.x) / 2.f)) are fixed by geometry, so a
        // column's root and x-side choices (and a row's y-side choices) are tabulated once
        {
            auto bits6 = [](int v, int a0, int a1) {
                int b = 0;
                for (int d = 0; d < 6; d++) {
                    const int sv = a0 + (int)std::ceil((float)(a1 - a0) / 2);
                    const bool hi = v >= sv;
                    (hi ? a0 : a1) = sv;
                    b = 2 * b + (hi ? 1 : 0);
                }
                return b;
            };
            const int Wl = G.max_bx - G.min_bx, Hl = G.max_by - G.min_by;
            G.oct_tab_off = (int)pl->otab.size();
            for (int x = 0; x < Wl; x++) {
                int r = (int)((float)x / G.hX);
                r = r < 0 ? 0 : (r >= G.n_ini ? G.n_ini - 1 : r);
                pl->otab.push_back((uint16_t)((r << 8) | bits6(x, (int)(G.hX * (float)r), (int)(G.hX * (float)(r + 1)))));
            }
            for (int y = 0; y < Hl; y++) pl->otab.push_back((uint16_t)bits6(y, 0, Hl));
        }
    }
    P.n_cells_total = cell_base;
    P.n_slots_total = slot_base;
    P.kp_slots_total = kp_base;
    P.pyr_bytes = ((pyr_off + 255) / 256) * 256;
    P.max_cells_level = max_cells;
    pl->kp_cap_frame = kp_base;
    P.fast_win_rows = hc_max;   // k_fast_cells' LDS variant
    P.fast_win_cols = wc_max;
    // cone pyramid tables: tiles of ~10x10 on the last level (252 at 640x480: the per-tile cascade
    // is latency bound, so smaller cones finish sooner), an even partition of every level; for
    // batches a second set from level kConeHiStart with bigger tiles (the small levels' launches
    // are latency bound there, the big levels' k_resize launches stream)
    if (L > 1) {
        std::vector<ConeRect> rects;
        std::vector<int> ctab;
        size_t stride = 0, lds = 0;
        const int ts = cone_tile_of(c);
        int tiles = cone_tables(P, *pl, 0, ts, rects, ctab, stride, lds);
        if (lds <= 60 * 1024) {
            pl->cone_tab.swap(ctab);
            pl->cone_tab_stride = (int)stride;
            pl->cone.swap(rects);
            pl->cone_tiles = tiles;
            pl->cone_lds = lds;
        }
        if (L > kConeHiStart + 1) {
            tiles = cone_tables(P, *pl, kConeHiStart, cone_hi_tile_of(), rects, ctab, stride, lds);
            if (lds <= 60 * 1024) {
                pl->cone_hi_tab.swap(ctab);
                pl->cone_hi_tab_stride = (int)stride;
                pl->cone_hi.swap(rects);
                pl->cone_hi_tiles = tiles;
                pl->cone_hi_lds = lds;
            }
        }
    }
    // k_resize_bands rows: per band, from the last level down, its own rows of the level plus the
    // rows the next level's band rows read (the source rows of k_resize's row tables, clamped)
    {
        const int nb = std::min(rz_bands(), L > 0 ? P.lv[L - 1].h : 0);
        if (L > kBandStart + 1 && nb > 0) {
            pl->bands.assign((size_t)nb * kMaxLevels * 2, 0);
            for (int b = 0; b < nb; b++) {
                int n0 = 0, n1 = 0;   // the rows of level l + 1 this band computes
                for (int l = L - 1; l > kBandStart; l--) {
                    const LevelGeom& G = P.lv[l];
                    int r0 = (int)((int64_t)b * G.h / nb), r1 = (int)((int64_t)(b + 1) * G.h / nb);
                    if (l < L - 1 && n1 > n0) {
                        const LevelGeom& U = P.lv[l + 1];
                        auto clampr = [&](int r) { return r < 0 ? 0 : (r < G.h ? r : G.h - 1); };
                        const int s0r = clampr(pl->yofs[U.ytab_off + n0]);
                        const int s1r = clampr(pl->yofs[U.ytab_off + n1 - 1] + 1) + 1;
                        if (r1 > r0) { r0 = std::min(r0, s0r); r1 = std::max(r1, s1r); }
                        else { r0 = s0r; r1 = s1r; }
                    }
                    pl->bands[((size_t)b * kMaxLevels + l) * 2] = r0;
                    pl->bands[((size_t)b * kMaxLevels + l) * 2 + 1] = r1;
                    n0 = r0; n1 = r1;
                }
            }
            pl->nbands = nb;
        }
    }
    // k_pyr_flow bands: task (l, b) = output rows [16 b, 16 b + 16) of level l; its source rows are
    // what resize_tile reads for each 4-row group (the interior path loads kRzSrc = 6 rows from the
    // group's first clamped source row, the per-row path rows sy and sy + 1), clamped
    if (L > 1) {
        constexpr int kFR = 16, kGroup = 4, kSrcRows = 6;
        int nbt = 0;
        for (int l = 1; l < L; l++) {
            pl->flow_boff[l] = nbt;
            nbt += (P.lv[l].h + kFR - 1) / kFR;
        }
        for (int l = L; l <= kMaxLevels; l++) pl->flow_boff[l] = nbt;
        pl->flow_nbt = nbt;
        pl->flow_dep.assign((size_t)nbt * 2, 0);
        for (int l = 2; l < L; l++) {
            const LevelGeom& G = P.lv[l];
            const int Sh = P.lv[l - 1].h;
            auto clampr = [&](int r) { return r < 0 ? 0 : (r < Sh ? r : Sh - 1); };
            for (int b = 0; b * kFR < G.h; b++) {
                const int r0 = b * kFR, r1 = std::min(r0 + kFR, G.h);
                int lo = Sh, hi = 0;
                for (int g = r0; g < r1; g += kGroup) {
                    const int rb = clampr(pl->yofs[G.ytab_off + g]);
                    lo = std::min(lo, rb);
                    hi = std::max(hi, std::min(rb + kSrcRows - 1, Sh - 1));
                    for (int dy = g; dy < std::min(g + kGroup, r1); dy++) {
                        lo = std::min(lo, clampr(pl->yofs[G.ytab_off + dy]));
                        hi = std::max(hi, clampr(pl->yofs[G.ytab_off + dy] + 1));
                    }
                }
                pl->flow_dep[(size_t)(pl->flow_boff[l] + b) * 2] = lo / kFR;
                pl->flow_dep[(size_t)(pl->flow_boff[l] + b) * 2 + 1] = hi / kFR;
            }
        }
    }
    // IC_Angle disc offsets (u, v) packed as int16 pairs
    for (int v = -15; v <= 15; v++) {
        const int d = c->umax[std::abs(v)];
        for (int u = -d; u <= d; u++) pl->disc.push_back((int)(uint16_t)(int16_t)u | ((int)(int16_t)v << 16));
    }
    P.n_disc = (int)pl->disc.size();   // <= 31 x 31 (k_desc_kp holds 4 entries per thread)
    if (P.n_disc > 1024) return ORBHIP_ERR_UNSUPPORTED;
    pl->disc.resize(1024, 0);   // zero-padded: k_desc_kp loads 4 x 256 entries without a bound (a (0, 0) entry adds nothing)
    // octree LDS configuration
    int max_kp_cap = 0;
    for (int l = 0; l < L; l++) max_kp_cap = std::max(max_kp_cap, P.lv[l].kp_cap);
    OctreeCfg& oc = pl->oct;
    oc.node_cap = ((max_kp_cap + 63) / 64) * 64;
    oc.sort_cap = 1;
    while (oc.sort_cap < oc.node_cap) oc.sort_cap <<= 1;
    oc.key_cap = 0;
    const size_t budget = 160 * 1024;
    const size_t base = octree_lds_bytes(P, oc);
    if (base + 1024 > budget) return ORBHIP_ERR_UNSUPPORTED;
    oc.key_cap = (int)std::min<size_t>(16384, ((budget - base - 64) / 6) & ~size_t(15));
    while (octree_lds_bytes(P, oc) > budget) oc.key_cap -= 16;
    // upload
    HIPOK(pl->d_plan.ensure(1));
    HIPOK(hipMemcpy(pl->d_plan.p, &P, sizeof(ExtractPlan), hipMemcpyHostToDevice));
    HIPOK(pl->d_cells.ensure(pl->cells.size()));
    HIPOK(hipMemcpy(pl->d_cells.p, pl->cells.data(), pl->cells.size() * sizeof(CellGeom), hipMemcpyHostToDevice));
    auto up = [](DevBuf<int>& d, const std::vector<int>& v) -> hipError_t {
        hipError_t e = d.ensure(v.size());
        if (e != hipSuccess) return e;
        if (v.empty()) return hipSuccess;
        return hipMemcpy(d.p, v.data(), v.size() * sizeof(int), hipMemcpyHostToDevice);
    };
    for (int i = 0; i < 4; i++) { pl->xofs.push_back(0); pl->xalpha.push_back(0); }   // int4 tail reads
    HIPOK(up(pl->d_xofs, pl->xofs));
    HIPOK(up(pl->d_xalpha, pl->xalpha));
    HIPOK(up(pl->d_yofs, pl->yofs));
    HIPOK(up(pl->d_ybeta, pl->ybeta));
    HIPOK(up(pl->d_disc, pl->disc));
    HIPOK(pl->d_otab.ensure(pl->otab.size()));
    HIPOK(hipMemcpy(pl->d_otab.p, pl->otab.data(), pl->otab.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    if (pl->nbands) HIPOK(up(pl->d_bands, pl->bands));
    if (pl->flow_nbt) HIPOK(up(pl->d_flow_dep, pl->flow_dep));
    if (!pl->cone_hi.empty()) {
        HIPOK(pl->d_cone_hi.ensure(pl->cone_hi.size()));
        HIPOK(hipMemcpy(pl->d_cone_hi.p, pl->cone_hi.data(), pl->cone_hi.size() * sizeof(ConeRect),
                        hipMemcpyHostToDevice));
        HIPOK(up(pl->d_cone_hi_tab, pl->cone_hi_tab));
    }
    if (!pl->cone.empty()) {
        HIPOK(pl->d_cone.ensure(pl->cone.size()));
        HIPOK(hipMemcpy(pl->d_cone.p, pl->cone.data(), pl->cone.size() * sizeof(ConeRect), hipMemcpyHostToDevice));
        HIPOK(up(pl->d_cone_tab, pl->cone_tab));
    }
    out = std::shared_ptr<Plan>(pl.release());
    return ORBHIP_OK;
}

static int ensure_batch(orbhip_ctx* c, const Plan* pl, int B) {
    const ExtractPlan& P = pl->h;
    HIPOK(c->d_pyr.ensure((size_t)B * P.pyr_bytes));
    HIPOK(c->d_cand.ensure((size_t)B * P.n_slots_total));
    HIPOK(c->d_cprim.ensure((size_t)B * P.n_cells_total * kCandPrim));
    HIPOK(c->d_kscratch.ensure((size_t)B * P.n_slots_total));
    HIPOK(c->d_nscratch.ensure((size_t)B * P.n_slots_total));
    HIPOK(c->d_cand_cnt.ensure((size_t)B * P.n_cells_total));
    HIPOK(c->d_cand_off.ensure((size_t)B * P.n_cells_total));
    HIPOK(c->d_cand_fill.ensure((size_t)B * kMaxLevels));
    if (pl->flow_nbt) {
        int* const was = c->d_flow.p;
        HIPOK(c->d_flow.ensure(kFlowCtl + (size_t)B * pl->flow_nbt));
        if (c->d_flow.p != was) HIPOK(hipMemset(c->d_flow.p, 0, c->d_flow.n * sizeof(int)));
    }
    HIPOK(c->d_lvl_kp.ensure((size_t)B * P.kp_slots_total));
    HIPOK(c->d_lvl_cnt.ensure((size_t)B * P.n_levels));
    HIPOK(c->d_lvl_nlap.ensure((size_t)B * P.n_levels));
    HIPOK(c->d_err.ensure(4));
    return ORBHIP_OK;
}

static int run_extract(orbhip_ctx* c, Plan* pl, const uint8_t* d_imgs, int B, int stride, int64_t fstride, int lap0,
                       int lap1, orbhip_kp* d_kps, uint8_t* d_desc, int cap, int32_t* d_n, int32_t* d_mono,
                       hipStream_t st) {
    const ExtractPlan& P = pl->h;
    (void)hipGetLastError();   // clear a sticky error of an earlier, already-reported call
    int rc = ensure_batch(c, pl, B);
    if (rc) return rc;
    // octree division engine (read per call so that tests can switch it): ORBHIP_OCTREE_SWEEP=1 runs
    // the sweep path only, ORBHIP_OCTREE_DH=d caps the pyramid depth (a shallow cap forces the
    // pyramid path's fallback to the sweep path)
    const char* e_sw = std::getenv("ORBHIP_OCTREE_SWEEP");
    const char* e_dh = std::getenv("ORBHIP_OCTREE_DH");
    const int oct_fast = (e_sw && e_sw[0] == '1') ? 0 : 1;
    const int oct_max_dh = e_dh ? std::max(1, std::min(6, std::atoi(e_dh))) : 6;
    // pyramid engine, also per call: ORBHIP_NO_CONE=1 forces the k_resize cascade
    const bool no_cone = std::getenv("ORBHIP_NO_CONE") != nullptr;
    // ORBHIP_CONE_HI=1: batches run levels 3.. as one cone launch behind two k_resize levels.
    // Off by default: at C3 (B = 64, 1280x720) that launch took 255-320 us against the 89 us of
    // the five k_resize launches it replaces (tools/c3_pyr_sweep.sh, tiles 16-48)
    const char* e_hi = std::getenv("ORBHIP_CONE_HI");
    const bool cone_hi_on = e_hi && e_hi[0] == '1';
    // ORBHIP_CAND_PACK=1 (read per call): packed FAST candidates, the octree then reads whole
    // lines. Off: at C3 it cut k_octree's traffic 21.8 -> 6.4 MB per launch (PMC), but the atomic
    // each FAST cell waits on held its work-group slot ~1 us longer: k_fast_cells 525 -> 568 us
    const char* e_pk = std::getenv("ORBHIP_CAND_PACK");
    const bool pack = e_pk && e_pk[0] == '1';
    // ORBHIP_RZ_FLOW=1 (read per call): batches build levels 1..L-1 in one k_pyr_flow launch
    const char* e_fl = std::getenv("ORBHIP_RZ_FLOW");
    const bool flow_on = e_fl && e_fl[0] == '1' && pl->flow_nbt > 0 && (int64_t)B * P.pyr_bytes < (1ll << 31);
    GraphKey key;
    key.add(1).add((uint64_t)oct_fast).add((uint64_t)oct_max_dh).add((uint64_t)no_cone).add((uint64_t)cone_hi_on).add((uint64_t)flow_on).add((uint64_t)pack).add((uint64_t)c->fast_nt).ptr(pl).ptr(d_imgs).add((uint64_t)B).add((uint64_t)stride).add((uint64_t)fstride).add((uint64_t)lap0)
        .add((uint64_t)lap1).ptr(d_kps).ptr(d_desc).add((uint64_t)cap).ptr(d_n).ptr(d_mono).ptr(st).ptr(c->d_pyr.p)
        .ptr(c->d_cand.p).ptr(c->d_kscratch.p).ptr(c->d_nscratch.p).ptr(c->d_cand_cnt.p).ptr(c->d_lvl_kp.p)
        .ptr(c->d_lvl_cnt.p).ptr(c->d_lvl_nlap.p).ptr(c->d_err.p).ptr(c->d_cand_off.p).ptr(c->d_cand_fill.p).ptr(c->d_cprim.p);
    return c->graphs.run(key, st, c->timer.stage != 0, [&](hipStream_t st) -> int {
        FrameBufs fb;
        fb.in = d_imgs; fb.in_stride = stride; fb.in_fstride = fstride; fb.pyr = c->d_pyr.p;
        StageTimer& tm = c->timer;
        const StageScope scope(tm);
        tm.begin(1, st);
        // the cone recomputes each tile's halo on every level: it pays only while the per-level
        // cascade is launch-latency bound (a few work-groups per CU); big batches keep the cascade
        static const size_t cone_max = std::getenv("ORBHIP_CONE_MAX_WG")
                                           ? (size_t)std::atol(std::getenv("ORBHIP_CONE_MAX_WG"))
                                           : (size_t)1024;
        const bool cone_path = pl->cone_tiles && !no_cone && (size_t)B * pl->cone_tiles <= cone_max;
        const bool cone_hi = !cone_path && pl->cone_hi_tiles && cone_hi_on;
        // the one-launch pyramid stamps its own execution span for the stage timer
        fb.stamp = (cone_path && tm.stage == 1 && tm.dstamp && tm.n < StageTimer::kCap) ? tm.dstamp + tm.n : nullptr;
        if (cone_path) {
            static const int cone_nt = [] {   // threads per tile (A/B: ORBHIP_CONE_NT = 256 / 512)
                const char* e = std::getenv("ORBHIP_CONE_NT");
                const int v = e ? std::atoi(e) : 1024;
                return (v == 256 || v == 512) ? v : 1024;
            }();
            launch_pyr_cone(pl->d_plan.p, pl->cone_tiles, pl->cone_lds, fb, B, pl->d_cone.p, pl->d_cone_tab.p,
                            pl->cone_tab_stride, st, 0, cone_nt, pl->d_xofs.p, pl->d_xalpha.p, pl->d_yofs.p,
                            pl->d_ybeta.p);
        } else if (flow_on) {
            PyrFlow fa{};
            fa.ctl = c->d_flow.p;
            fa.flags = c->d_flow.p + kFlowCtl;
            fa.dep = (const int2*)pl->d_flow_dep.p;
            for (int l = 0; l <= kMaxLevels; l++) fa.boff[l] = pl->flow_boff[l];
            fa.B = B;
            fa.nbt = pl->flow_nbt;
            fa.pyr_limit = (int)((int64_t)B * P.pyr_bytes);
            launch_pyr_flow(pl->d_plan.p, fb, pl->d_xofs.p, pl->d_xalpha.p, pl->d_yofs.p, pl->d_ybeta.p, fa, st);
        } else {
            const bool bands = !cone_hi && pl->nbands > 0;
            const int lr = cone_hi ? kConeHiStart + 1 : (bands ? kBandStart + 1 : P.n_levels);
            for (int l = 1; l < lr; l++)
                launch_resize(pl->d_plan.p, P, fb, B, l, pl->d_xofs.p, pl->d_xalpha.p, pl->d_yofs.p, pl->d_ybeta.p,
                              st);
            if (cone_hi)
                launch_pyr_cone(pl->d_plan.p, pl->cone_hi_tiles, pl->cone_hi_lds, fb, B, pl->d_cone_hi.p,
                                pl->d_cone_hi_tab.p, pl->cone_hi_tab_stride, st, kConeHiStart, cone_hi_threads(),
                                pl->d_xofs.p, pl->d_xalpha.p, pl->d_yofs.p, pl->d_ybeta.p);
            if (bands)
                launch_resize_bands(pl->d_plan.p, pl->nbands, fb, B, kBandStart, (const int2*)pl->d_bands.p,
                                    pl->d_xofs.p, pl->d_xalpha.p, pl->d_yofs.p, pl->d_ybeta.p, st);
        }
        tm.end(1, st);
        tm.begin(2, st);
        CandPack cp;
        cp.prim = c->d_cprim.p;
        if (pack) {
            HIPOK(hipMemsetAsync(c->d_cand_fill.p, 0, sizeof(int) * (size_t)B * kMaxLevels, st));
            cp.fill = c->d_cand_fill.p;
            cp.off = c->d_cand_off.p;
        }
        launch_fast(pl->d_plan.p, P, pl->d_cells.p, fb, B, c->d_cand.p, c->d_cand_cnt.p, c->d_err.p, st, c->fast_nt,
                    cp);
        tm.end(2, st);
        OctreeCfg oc = pl->oct;
        oc.lap0 = lap0; oc.lap1 = lap1;
        oc.fast = oct_fast;
        oc.max_dh = oct_max_dh;
        tm.begin(3, st);
        launch_octree(pl->d_plan.p, P, pl->d_cells.p, pl->d_otab.p, c->d_cand.p, cp.off ? nullptr : cp.prim,
                      c->d_cand_cnt.p, cp.off,
                      c->d_kscratch.p, c->d_nscratch.p, c->d_lvl_kp.p, c->d_lvl_cnt.p, c->d_lvl_nlap.p, oc, c->d_err.p, B,
                      st, (tm.stage == 3 && tm.dstamp && tm.n < StageTimer::kCap) ? tm.dstamp + tm.n : nullptr);
        tm.end(3, st);
        tm.begin(4, st);
        launch_desc(pl->d_plan.p, P, fb, c->d_lvl_kp.p, c->d_lvl_cnt.p, c->d_lvl_nlap.p, pl->d_disc.p, d_kps, d_desc,
                    cap, d_n, d_mono, B, st);
        tm.end(4, st);
        HIPOK(hipGetLastError());
        return ORBHIP_OK;
    });
}

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int orbhip_abi_version(void) { return ORBHIP_ABI_VERSION; }

int orbhip_bgr_to_gray_device(orbhip_ctx* c, const uint8_t* d_bgr, int B, int w, int h, int src_stride,
                              int64_t src_fstride, uint8_t* d_gray, int dst_stride, int64_t dst_fstride, void* stream) {
    if (!c || !d_bgr || !d_gray || B < 0 || w <= 0 || h <= 0 || src_stride < 3 * w || dst_stride < w ||
        (B > 1 && (src_fstride < (int64_t)src_stride * h || dst_fstride < (int64_t)dst_stride * h)))
        return ORBHIP_ERR_ARG;
    if (B == 0) return ORBHIP_OK;
    HIPOK(hipSetDevice(c->device));
    (void)hipGetLastError();
    hipStream_t st = (hipStream_t)stream;   // NULL = the HIP null stream (HIP convention)
    launch_bgr2gray(d_bgr, B, w, h, src_stride, src_fstride, d_gray, dst_stride, dst_fstride, st);
    HIPOK(hipGetLastError());
    return ORBHIP_OK;
}

static bool valid_cam(const orbhip_pinhole* c) {
    return c && c->fx != 0.0f && c->fy != 0.0f && std::isfinite(c->fx) && std::isfinite(c->fy);
}

int orbhip_undistort_keypoints(orbhip_ctx* c, const orbhip_pinhole* cam, const orbhip_kp* kps, int n, orbhip_kp* out) {
    if (!c || !valid_cam(cam) || n < 0 || (n > 0 && (!kps || !out))) return ORBHIP_ERR_ARG;
    if (n == 0) return ORBHIP_OK;
    if (cam->k1 == 0.0f) {   // mvKeysUn = mvKeys
        if (out != kps) std::memmove(out, kps, sizeof(orbhip_kp) * (size_t)n);
        return ORBHIP_OK;
    }
    HIPOK(hipSetDevice(c->device));
    HIPOK(c->d_kps.ensure((size_t)n));
    hipStream_t st = c->stream;
    HIPOK(hipMemcpyAsync(c->d_kps.p, kps, sizeof(orbhip_kp) * (size_t)n, hipMemcpyHostToDevice, st));
    (void)hipGetLastError();
    launch_undistort_kps(c->d_kps.p, nullptr, n, 1, n, *cam, c->d_kps.p, st);
    HIPOK(hipGetLastError());
    HIPOK(hipMemcpyAsync(out, c->d_kps.p, sizeof(orbhip_kp) * (size_t)n, hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    return ORBHIP_OK;
}

int orbhip_undistort_keypoints_device(orbhip_ctx* c, const orbhip_pinhole* cam, const orbhip_kp* d_kps,
                                      const int32_t* d_n, int B, int cap, orbhip_kp* d_out, void* stream) {
    if (!c || !valid_cam(cam) || B < 0 || cap < 0 || (B > 0 && (!d_kps || !d_n || !d_out))) return ORBHIP_ERR_ARG;
    if (B == 0 || cap == 0) return ORBHIP_OK;
    HIPOK(hipSetDevice(c->device));
    (void)hipGetLastError();
    launch_undistort_kps(d_kps, d_n, 0, B, cap, *cam, d_out, (hipStream_t)stream);   // k1 == 0: a copy
    HIPOK(hipGetLastError());
    return ORBHIP_OK;
}

int orbhip_image_bounds(orbhip_ctx* c, const orbhip_pinhole* cam, int cols, int rows, float bounds[4]) {
    if (!c || !valid_cam(cam) || cols <= 0 || rows <= 0 || !bounds) return ORBHIP_ERR_ARG;
    if (cam->k1 == 0.0f) {
        bounds[0] = 0.0f; bounds[1] = (float)cols; bounds[2] = 0.0f; bounds[3] = (float)rows;
        return ORBHIP_OK;
    }
    HIPOK(hipSetDevice(c->device));
    HIPOK(c->d_kps.ensure(4));   // 4 floats of scratch
    hipStream_t st = c->stream;
    (void)hipGetLastError();
    launch_image_bounds(cols, rows, *cam, (float*)c->d_kps.p, st);
    HIPOK(hipGetLastError());
    HIPOK(hipMemcpyAsync(bounds, c->d_kps.p, 4 * sizeof(float), hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    return ORBHIP_OK;
}

int orbhip_create(orbhip_ctx** out, int device, const orbhip_orb_params* params) {
    if (!out) return ORBHIP_ERR_ARG;
    *out = nullptr;
    orbhip_orb_params p = {1000, 1.2f, 8, 20, 7};
    if (params) p = *params;
    if (p.n_features < 0 || p.n_levels < 1 || p.n_levels > kMaxLevels || !(p.scale_factor >= 1.0f))
        return ORBHIP_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ORBHIP_ERR_DEVICE;
    // device < 0: the calling thread's current HIP device (the rank's GPU after torch.cuda.set_device
    // / hipSetDevice in a one-process-per-GPU job)
    if (device < 0 && hipGetDevice(&device) != hipSuccess) return ORBHIP_ERR_DEVICE;
    if (device < 0 || device >= ndev) return ORBHIP_ERR_DEVICE;
    std::unique_ptr<orbhip_ctx> c(new orbhip_ctx());
    c->device = device;
    c->prm = p;
    HIPOK(hipSetDevice(device));
    HIPOK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (!octree_set_lds_limit(160 * 1024)) return ORBHIP_ERR_DEVICE;
    build_orb_tables(c.get());
    *out = c.release();
    return ORBHIP_OK;
}

int orbhip_destroy(orbhip_ctx* c) {
    if (!c) return ORBHIP_ERR_ARG;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->graphs.graphs()) (void)hipDeviceSynchronize();   // replays may run on caller streams
    c->graphs.clear();
    if (c->timer.created) {
        for (int i = 0; i < 2 * StageTimer::kCap; i++) (void)hipEventDestroy(c->timer.ev[i]);
        if (c->timer.dstamp) (void)hipFree(c->timer.dstamp);
    }
    ba_destroy(c->ba);
    if (c->stream) dag_stream_retired(c->stream);   // before the stream goes: no solve may wait on it
    pose_ws_destroy(c->pose);
    proj_ws_destroy(c->proj);
    c->plans.clear();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return ORBHIP_OK;
}

int orbhip_level_info(orbhip_ctx* c, int w, int h, int32_t* lw, int32_t* lh, int32_t* nf, float* sc) {
    if (!c || w <= 0 || h <= 0) return ORBHIP_ERR_ARG;
    for (int l = 0; l < c->prm.n_levels; l++) {
        if (lw) lw[l] = round_even_f((float)w * c->inv_scale[l]);
        if (lh) lh[l] = round_even_f((float)h * c->inv_scale[l]);
        if (nf) nf[l] = c->feat[l];
        if (sc) sc[l] = c->scale[l];
    }
    return ORBHIP_OK;
}

int orbhip_max_keypoints(orbhip_ctx* c, int w, int h) {
    if (!c || w <= 0 || h <= 0) return ORBHIP_ERR_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return ORBHIP_ERR_DEVICE;
    Plan* pl = nullptr;
    int rc = build_plan(c, w, h, &pl);
    return rc ? rc : pl->kp_cap_frame;
}

int orbhip_extract_batch_device(orbhip_ctx* c, const uint8_t* d_imgs, int B, int w, int h, int stride,
                                int64_t frame_stride, int lap0, int lap1, orbhip_kp* d_kps, uint8_t* d_desc, int cap,
                                int32_t* d_n, int32_t* d_mono, void* stream) {
    if (!c || !d_imgs || B <= 0 || w <= 0 || h <= 0 || stride < w || !d_kps || !d_desc || !d_n || !d_mono || cap <= 0)
        return ORBHIP_ERR_ARG;
    if (B > 1 && frame_stride < (int64_t)stride * h) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    Plan* pl = nullptr;
    int rc = build_plan(c, w, h, &pl);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;   // NULL = the HIP null stream (HIP convention)
    return run_extract(c, pl, d_imgs, B, stride, frame_stride, lap0, lap1, d_kps, d_desc, cap, d_n, d_mono, st);
}

int orbhip_extract(orbhip_ctx* c, const uint8_t* img, int w, int h, int stride, int lap0, int lap1, orbhip_kp* kps,
                   uint8_t* desc32, int cap, int* n_out, int* mono_index) {
    if (!c || !n_out) return ORBHIP_ERR_ARG;
    *n_out = 0;
    if (mono_index) *mono_index = -1;
    if (!img || w <= 0 || h <= 0) return ORBHIP_ERR_EMPTY;   // operator(): _image.empty() -> -1
    if (stride < w || (cap > 0 && (!kps || !desc32))) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    Plan* pl = nullptr;
    int rc = build_plan(c, w, h, &pl);
    if (rc) return rc;
    const int kcap = pl->kp_cap_frame;
    HIPOK(c->d_in.ensure((size_t)w * h));
    HIPOK(c->d_kps.ensure(kcap));
    HIPOK(c->d_desc.ensure((size_t)kcap * 32));
    HIPOK(c->d_n.ensure(1));
    HIPOK(c->d_mono.ensure(1));
    hipStream_t st = c->stream;
    HIPOK(hipMemcpy2DAsync(c->d_in.p, w, img, stride, w, h, hipMemcpyHostToDevice, st));
    rc = run_extract(c, pl, c->d_in.p, 1, w, (int64_t)w * h, lap0, lap1, c->d_kps.p, c->d_desc.p, kcap, c->d_n.p,
                     c->d_mono.p, st);
    if (rc) return rc;
    int n = 0, mono = 0, err[4] = {0, 0, 0, 0};
    HIPOK(hipMemcpyAsync(&n, c->d_n.p, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(&mono, c->d_mono.p, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(err, c->d_err.p, sizeof(err), hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    if (err[0]) return ORBHIP_ERR_DEVICE;
    *n_out = n;
    if (mono_index) *mono_index = mono;
    if (n > cap) return ORBHIP_ERR_CAPACITY;
    if (n > 0) {
        HIPOK(hipMemcpyAsync(kps, c->d_kps.p, (size_t)n * sizeof(orbhip_kp), hipMemcpyDeviceToHost, st));
        HIPOK(hipMemcpyAsync(desc32, c->d_desc.p, (size_t)n * 32, hipMemcpyDeviceToHost, st));
        HIPOK(hipStreamSynchronize(st));
    }
    return ORBHIP_OK;
}

int orbhip_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    if (!a || !b) return ORBHIP_ERR_ARG;
    int d = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        std::memcpy(&x, a + 4 * i, 4);
        std::memcpy(&y, b + 4 * i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

// the one-launch matcher's counters: zeroed on the call's stream before their first use
static int ensure_msync(orbhip_ctx* c, hipStream_t st) {
    if (c->d_msync.p) return ORBHIP_OK;
    HIPOK(c->d_msync.ensure(kMatchSyncInts));
    HIPOK(hipMemsetAsync(c->d_msync.p, 0, sizeof(int) * kMatchSyncInts, st));
    return ORBHIP_OK;
}

int orbhip_match_bf(orbhip_ctx* c, const uint8_t* q, const float* qa, int nq, const uint8_t* t, const float* ta,
                    int nt, int th_low, float ratio, int check_orientation, int32_t* match, int32_t* best_d,
                    int32_t* second_d) {
    if (!c || nq < 0 || nt < 0 || (nq > 0 && (!q || !qa || !match || !best_d || !second_d)) || (nt > 0 && (!t || !ta)))
        return ORBHIP_ERR_ARG;
    if (nq == 0) return 0;
    HIPOK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    HIPOK(c->d_mq.ensure((size_t)nq * 32));
    HIPOK(c->d_mt.ensure((size_t)std::max(nt, 1) * 32));
    HIPOK(c->d_mqa.ensure(nq));
    HIPOK(c->d_mta.ensure(std::max(nt, 1)));
    HIPOK(c->d_mm.ensure(nq));
    HIPOK(c->d_mb.ensure(nq));
    HIPOK(c->d_ms.ensure(nq));
    HIPOK(c->d_mn.ensure(1));
    HIPOK(hipMemcpyAsync(c->d_mq.p, q, (size_t)nq * 32, hipMemcpyHostToDevice, st));
    HIPOK(hipMemcpyAsync(c->d_mqa.p, qa, (size_t)nq * 4, hipMemcpyHostToDevice, st));
    if (nt > 0) {
        HIPOK(hipMemcpyAsync(c->d_mt.p, t, (size_t)nt * 32, hipMemcpyHostToDevice, st));
        HIPOK(hipMemcpyAsync(c->d_mta.p, ta, (size_t)nt * 4, hipMemcpyHostToDevice, st));
    } else {
        // no train descriptors: every query keeps best = second = 256 (no match)
        HIPOK(hipMemsetAsync(c->d_mm.p, 0xFF, (size_t)nq * 4, st));
    }
    HIPOK(c->d_mpart.ensure(match_part_entries(1, nq, nt)));
    if (int rc = ensure_msync(c, st)) return rc;
    (void)hipGetLastError();
    launch_match_bf(c->d_mq.p, c->d_mqa.p, nq, c->d_mt.p, c->d_mta.p, nt, th_low, ratio, check_orientation, c->d_mm.p,
                    c->d_mb.p, c->d_ms.p, c->d_mn.p, c->d_mpart.p, st, c->d_msync.p);
    HIPOK(hipGetLastError());
    int nm = 0;
    HIPOK(hipMemcpyAsync(match, c->d_mm.p, (size_t)nq * 4, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(best_d, c->d_mb.p, (size_t)nq * 4, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(second_d, c->d_ms.p, (size_t)nq * 4, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(&nm, c->d_mn.p, 4, hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    return nm;
}

int orbhip_match_pairs_device(orbhip_ctx* c, const orbhip_kp* d_kps, const uint8_t* d_desc, const int32_t* d_n, int B,
                              int cap, int th_low, float ratio, int check_orientation, int32_t* d_match,
                              int32_t* d_best, int32_t* d_second, int32_t* d_nmatch, void* stream) {
    if (!c || !d_kps || !d_desc || !d_n || B < 2 || cap <= 0 || !d_match || !d_best || !d_second || !d_nmatch)
        return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;   // NULL = the HIP null stream (HIP convention)
    HIPOK(c->d_mpart.ensure(match_part_entries(B - 1, cap, cap)));
    if (int rc = ensure_msync(c, st)) return rc;
    (void)hipGetLastError();
    GraphKey key;
    key.add(3).ptr(d_kps).ptr(d_desc).ptr(d_n).add((uint64_t)B).add((uint64_t)cap).add((uint64_t)th_low).f32(ratio)
        .add((uint64_t)check_orientation).ptr(d_match).ptr(d_best).ptr(d_second).ptr(d_nmatch).ptr(st)
        .ptr(c->d_mpart.p).ptr(c->d_msync.p);
    return c->graphs.run(key, st, c->timer.stage != 0, [&](hipStream_t st) -> int {
        launch_match_pairs(d_kps, d_desc, d_n, B - 1, cap, th_low, ratio, check_orientation, d_match, d_best,
                           d_second, d_nmatch, c->d_mpart.p, st, &c->timer, c->d_msync.p);
        HIPOK(hipGetLastError());
        return ORBHIP_OK;
    });
}

int orbhip_match_frames_device(orbhip_ctx* c, const orbhip_kp* d_q_kps, const uint8_t* d_q_desc, const int32_t* d_nq,
                               const orbhip_kp* d_t_kps, const uint8_t* d_t_desc, const int32_t* d_nt, int cap,
                               int th_low, float ratio, int check_orientation, int32_t* d_match, int32_t* d_best,
                               int32_t* d_second, int32_t* d_nmatch, void* stream) {
    if (!c || !d_q_kps || !d_q_desc || !d_nq || !d_t_kps || !d_t_desc || !d_nt || cap <= 0 || !d_match || !d_best ||
        !d_second || !d_nmatch)
        return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;   // NULL = the HIP null stream (HIP convention)
    HIPOK(c->d_mpart.ensure(match_part_entries(1, cap, cap)));
    if (int rc = ensure_msync(c, st)) return rc;
    (void)hipGetLastError();
    GraphKey key;
    key.add(2).ptr(d_q_kps).ptr(d_q_desc).ptr(d_nq).ptr(d_t_kps).ptr(d_t_desc).ptr(d_nt).add((uint64_t)cap)
        .add((uint64_t)th_low).f32(ratio).add((uint64_t)check_orientation).ptr(d_match).ptr(d_best).ptr(d_second)
        .ptr(d_nmatch).ptr(st).ptr(c->d_mpart.p).ptr(c->d_msync.p);
    return c->graphs.run(key, st, c->timer.stage != 0, [&](hipStream_t st) -> int {
        launch_match_frames(d_q_kps, d_q_desc, d_nq, d_t_kps, d_t_desc, d_nt, cap, th_low, ratio, check_orientation,
                            d_match, d_best, d_second, d_nmatch, c->d_mpart.p, st, &c->timer, c->d_msync.p);
        HIPOK(hipGetLastError());
        return ORBHIP_OK;
    });
}

int orbhip_launch_graphs(orbhip_ctx* c) {
    if (!c) return ORBHIP_ERR_ARG;
    return c->graphs.graphs();
}

int orbhip_profile_stage(orbhip_ctx* c, int stage) {
    if (!c || stage < 0 || stage > 6) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    StageTimer& t = c->timer;
    if (!t.created) {
        for (int i = 0; i < 2 * StageTimer::kCap; i++) HIPOK(hipEventCreate(&t.ev[i]));
        HIPOK(hipMalloc((void**)&t.dstamp, 2 * StageTimer::kCap * sizeof(unsigned long long)));
        t.created = true;
    }
    HIPOK(hipDeviceSynchronize());
    HIPOK(hipMemset(t.dstamp, 0xFF, StageTimer::kCap * sizeof(unsigned long long)));   // minima: ~0
    HIPOK(hipMemset(t.dstamp + StageTimer::kCap, 0, StageTimer::kCap * sizeof(unsigned long long)));
    t.stage = stage;
    t.n = 0;
    return ORBHIP_OK;
}

int orbhip_profile_collect(orbhip_ctx* c, double* total_ms, int32_t* count) {
    if (!c || !total_ms || !count) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    StageTimer& t = c->timer;
    double s = 0;
    for (int i = 0; i < t.n; i++) {
        HIPOK(hipEventSynchronize(t.ev[2 * i + 1]));
        float ms = 0;
        HIPOK(hipEventElapsedTime(&ms, t.ev[2 * i], t.ev[2 * i + 1]));
        s += ms;
    }
    // the pyramid's k_pyr_cone and k_octree also stamp their execution span from the device (first
    // workgroup start -> last workgroup end, as rocprofv3's kernel trace counts it): used when every
    // timed launch stamped (the k_resize cascade of batches does not)
    if ((t.stage == 1 || t.stage == 3) && t.n > 0 && t.dstamp) {
        std::vector<unsigned long long> h(2 * (size_t)t.n);
        HIPOK(hipMemcpy(h.data(), t.dstamp, t.n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        HIPOK(hipMemcpy(h.data() + t.n, t.dstamp + StageTimer::kCap, t.n * sizeof(unsigned long long),
                        hipMemcpyDeviceToHost));
        int rate_khz = 0;
        HIPOK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c->device));
        bool all = rate_khz > 0;
        double d = 0;
        for (int i = 0; i < t.n && all; i++) {
            all = h[t.n + i] != 0 && h[i] != ~0ull && h[t.n + i] >= h[i];
            d += (double)(h[t.n + i] - h[i]);
        }
        if (all) s = d / rate_khz;   // ticks / kHz = ms
        HIPOK(hipMemset(t.dstamp, 0xFF, t.n * sizeof(unsigned long long)));
        HIPOK(hipMemset(t.dstamp + StageTimer::kCap, 0, t.n * sizeof(unsigned long long)));
    }
    *total_ms = s;
    *count = t.n;
    t.n = 0;
    return ORBHIP_OK;
}

int orbhip_ba_solve(orbhip_ctx* c, const orbhip_ba_problem* prob, orbhip_ba_result* res, const volatile int* stop) {
    if (!c || !prob || !res) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    if (!c->ba) c->ba = ba_create();
    if (!c->ba) return ORBHIP_ERR_DEVICE;
    return ba_solve(c->ba, prob, res, stop, c->stream);
}

int orbhip_ba_stats(orbhip_ctx* c, int64_t out[4]) {
    if (!c || !out) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    long long l = 0, h = 0, t = 0, r = 0;
    dag_device_stats(&l, &h);
    ba_stats(c->ba, &t, &r);
    out[0] = l; out[1] = h; out[2] = t; out[3] = r;
    return ORBHIP_OK;
}

int orbhip_ba_solve_batch(orbhip_ctx* c, const orbhip_ba_problem* probs, int B, orbhip_ba_result* res,
                          const volatile int* stop) {
    if (!c || !probs || !res || B <= 0) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    if (!c->ba) c->ba = ba_create();
    if (!c->ba) return ORBHIP_ERR_DEVICE;
    std::vector<const orbhip_ba_problem*> pp(B);
    std::vector<orbhip_ba_result*> rr(B);
    for (int b = 0; b < B; b++) { pp[b] = probs + b; rr[b] = res + b; }
    return ba_solve_batch(c->ba, pp.data(), B, rr.data(), stop, c->stream, kShardNone);
}

int orbhip_pose_optimization_batch(orbhip_ctx* c, const orbhip_pose_problem* probs, int B,
                                   orbhip_pose_result* res) {
    if (!c || !probs || !res || B <= 0) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    if (!c->pose) c->pose = pose_ws_create();
    if (!c->pose) return ORBHIP_ERR_DEVICE;
    return pose_opt_batch(c->pose, probs, B, res, c->stream);
}

int orbhip_pose_optimization(orbhip_ctx* c, const orbhip_pose_problem* prob, orbhip_pose_result* res) {
    const int rc = orbhip_pose_optimization_batch(c, prob, 1, res);
    return rc < 0 ? rc : res->n_inliers;
}

int orbhip_search_by_projection_last(orbhip_ctx* c, const orbhip_frame* cur, const orbhip_proj_last* last,
                                     float th, int check_orientation, int32_t* match) {
    if (!c) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    if (!c->proj) c->proj = proj_ws_create();
    return proj_search_last(c->proj, cur, last, th, check_orientation, match, nullptr, c->stream);
}

int orbhip_search_local_points(orbhip_ctx* c, const orbhip_frame* frame, const orbhip_local_points* mps,
                               float view_cos_limit, float th, float nnratio, int far_points, float th_far,
                               uint8_t* in_view, int32_t* level, int32_t* match) {
    if (!c) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    if (!c->proj) c->proj = proj_ws_create();
    return proj_search_local(c->proj, frame, mps, view_cos_limit, th, nnratio, far_points, th_far, in_view, level,
                             match, nullptr, c->stream);
}

int orbhip_search_for_initialization(orbhip_ctx* c, const orbhip_init_frame* f1, const orbhip_init_frame* f2,
                                     float* prev_matched, int window_size, float nnratio, int check_orientation,
                                     int32_t* matches12) {
    if (!c) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    if (!c->proj) c->proj = proj_ws_create();
    return init_search(c->proj, f1, f2, prev_matched, window_size, nnratio, check_orientation, matches12, c->stream);
}

struct orbhip_kfdb {
    orbhip::KfDb* d = nullptr;
    int device = 0;
};

int orbhip_kfdb_create(orbhip_ctx* c, int max_kf, orbhip_kfdb** out) {
    if (!c || !out) return ORBHIP_ERR_ARG;
    *out = nullptr;
    HIPOK(hipSetDevice(c->device));
    int rc = ORBHIP_OK;
    KfDb* d = kfdb_create(max_kf, c->stream, &rc);
    if (!d) return rc;
    *out = new orbhip_kfdb{d, c->device};
    return ORBHIP_OK;
}

int orbhip_kfdb_destroy(orbhip_kfdb* db) {
    if (!db) return ORBHIP_ERR_ARG;
    (void)hipSetDevice(db->device);
    kfdb_destroy(db->d);
    delete db;
    return ORBHIP_OK;
}

int orbhip_kfdb_add(orbhip_kfdb* db, int kf, const int32_t* words, const double* values, int n) {
    if (!db) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(db->device));
    return kfdb_add(db->d, kf, words, values, n);
}

int orbhip_kfdb_erase(orbhip_kfdb* db, int kf) {
    if (!db) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(db->device));
    return kfdb_erase(db->d, kf);
}

int orbhip_kfdb_detect_relocalization(orbhip_kfdb* db, const orbhip_kfdb_query* q, int32_t* out, int cap) {
    if (!db) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(db->device));
    return kfdb_detect_relocalization(db->d, q, out, cap);
}

int orbhip_kfdb_detect_nbest(orbhip_kfdb* db, const orbhip_kfdb_query* q, const uint8_t* connected, int n,
                             int32_t* loop_out, int32_t* n_loop, int32_t* merge_out, int32_t* n_merge) {
    if (!db) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(db->device));
    return kfdb_detect_nbest(db->d, q, connected, n, loop_out, n_loop, merge_out, n_merge);
}

int orbhip_comm_unique_id(uint8_t* id) {
    if (!id) return ORBHIP_ERR_ARG;
    return ba_comm_unique_id(id);
}

int orbhip_comm_init(orbhip_ctx* c, int nranks, int rank, const uint8_t* id) {
    if (!c || !id) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    if (!c->ba) c->ba = ba_create();
    if (!c->ba) return ORBHIP_ERR_DEVICE;
    return ba_comm_init(c->ba, nranks, rank, id);
}

int orbhip_ba_solve_sharded(orbhip_ctx* c, const orbhip_ba_problem* shard, orbhip_ba_result* res,
                            const volatile int* stop) {
    if (!c || !shard || !res || !c->ba) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    const orbhip_ba_problem* pp[1] = {shard};
    orbhip_ba_result* rr[1] = {res};
    return ba_solve_batch(c->ba, pp, 1, rr, stop, c->stream, kShardRccl);
}

int orbhip_ba_solve_sharded_segments(orbhip_ctx* c, const orbhip_ba_problem* shards, int nlocal, orbhip_ba_result* res,
                                     const volatile int* stop) {
    if (!c || !shards || !res || nlocal <= 0 || !c->ba) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    std::vector<const orbhip_ba_problem*> pp(nlocal);
    std::vector<orbhip_ba_result*> rr(nlocal);
    for (int b = 0; b < nlocal; b++) { pp[b] = shards + b; rr[b] = res + b; }
    return ba_solve_batch(c->ba, pp.data(), nlocal, rr.data(), stop, c->stream, kShardRccl);
}

int orbhip_ba_solve_shards_local(orbhip_ctx* c, const orbhip_ba_problem* shards, int nshards, orbhip_ba_result* res,
                                 const volatile int* stop) {
    if (!c || !shards || !res || nshards <= 0) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    if (!c->ba) c->ba = ba_create();
    if (!c->ba) return ORBHIP_ERR_DEVICE;
    std::vector<const orbhip_ba_problem*> pp(nshards);
    std::vector<orbhip_ba_result*> rr(nshards);
    for (int b = 0; b < nshards; b++) { pp[b] = shards + b; rr[b] = res + b; }
    return ba_solve_batch(c->ba, pp.data(), nshards, rr.data(), stop, c->stream, kShardLocal);
}

// ---- bag of words (a13/a14) ----
}  // extern "C"

struct orbhip_vocab {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0;
    DevBuf<uint8_t> desc;
    DevBuf<int> first_child, n_child, children, word_id;
    DevBuf<double> weight;
    VocabView view() const {
        VocabView v;
        v.desc = (const uint4*)desc.p;
        v.first_child = first_child.p; v.n_child = n_child.p; v.children = children.p;
        v.word_id = word_id.p; v.weight = weight.p; v.L = L;
        return v;
    }
};

static int vocab_build(orbhip_ctx* c, int k, int L, int scoring, int weighting, int N, const int32_t* parent,
                       const uint8_t* is_leaf, const uint8_t* desc32, const double* weight, orbhip_vocab** out) {
    if (!c || !out || N < 2 || !parent || !is_leaf || !desc32 || !weight || L < 1) return ORBHIP_ERR_ARG;
    for (int i = 1; i < N; i++)
        if (parent[i] < 0 || parent[i] >= i) return ORBHIP_ERR_ARG;   // file order: parents precede children
    std::vector<int> nch(N, 0), first(N, 0), children(N > 1 ? N - 1 : 1), fill(N), word(N, -1);
    for (int i = 1; i < N; i++) nch[parent[i]]++;
    for (int i = 1; i < N; i++) first[i] = first[i - 1] + nch[i - 1];
    fill = first;
    for (int i = 1; i < N; i++) children[fill[parent[i]]++] = i;   // file order within a parent
    int nw = 0;
    for (int i = 1; i < N; i++) {
        if (is_leaf[i] && nch[i] > 0) return ORBHIP_ERR_ARG;
        if (!is_leaf[i] && nch[i] == 0) return ORBHIP_ERR_ARG;
        if (is_leaf[i]) word[i] = nw++;
    }
    if (nch[0] == 0) return ORBHIP_ERR_ARG;
    std::unique_ptr<orbhip_vocab> v(new orbhip_vocab());
    v->device = c->device; v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting; v->n_nodes = N;
    HIPOK(hipSetDevice(c->device));
    HIPOK(v->desc.ensure((size_t)N * 32));
    HIPOK(v->first_child.ensure(N)); HIPOK(v->n_child.ensure(N)); HIPOK(v->children.ensure(children.size()));
    HIPOK(v->word_id.ensure(N)); HIPOK(v->weight.ensure(N));
    HIPOK(hipMemcpy(v->desc.p, desc32, (size_t)N * 32, hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(v->first_child.p, first.data(), N * sizeof(int), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(v->n_child.p, nch.data(), N * sizeof(int), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(v->children.p, children.data(), children.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(v->word_id.p, word.data(), N * sizeof(int), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(v->weight.p, weight, N * sizeof(double), hipMemcpyHostToDevice));
    *out = v.release();
    return ORBHIP_OK;
}

extern "C" {

int orbhip_vocab_create(orbhip_ctx* c, int k, int L, int scoring, int weighting, int n_nodes, const int32_t* parent,
                        const uint8_t* is_leaf, const uint8_t* desc32, const double* weight, orbhip_vocab** out) {
    return vocab_build(c, k, L, scoring, weighting, n_nodes, parent, is_leaf, desc32, weight, out);
}

int orbhip_vocab_load_text(orbhip_ctx* c, const char* path, orbhip_vocab** out) {
    if (!c || !path || !out) return ORBHIP_ERR_ARG;
    FILE* f = std::fopen(path, "r");
    if (!f) return ORBHIP_ERR_ARG;
    int k = 0, L = 0, sc = 0, wt = 0;
    if (std::fscanf(f, "%d %d %d %d", &k, &L, &sc, &wt) != 4) { std::fclose(f); return ORBHIP_ERR_ARG; }
    std::vector<int32_t> parent(1, -1);
    std::vector<uint8_t> leaf(1, 0), desc(32, 0);
    std::vector<double> weight(1, 0.0);
    int p, il;
    while (std::fscanf(f, "%d %d", &p, &il) == 2) {
        unsigned char d[32];
        for (int j = 0; j < 32; j++) {
            int v;
            if (std::fscanf(f, "%d", &v) != 1) { std::fclose(f); return ORBHIP_ERR_ARG; }
            d[j] = (unsigned char)v;
        }
        double w;
        if (std::fscanf(f, "%lf", &w) != 1) { std::fclose(f); return ORBHIP_ERR_ARG; }
        parent.push_back(p); leaf.push_back((uint8_t)il); weight.push_back(w);
        desc.insert(desc.end(), d, d + 32);
    }
    std::fclose(f);
    return vocab_build(c, k, L, sc, wt, (int)parent.size(), parent.data(), leaf.data(), desc.data(), weight.data(), out);
}

int orbhip_vocab_destroy(orbhip_vocab* v) {
    if (!v) return ORBHIP_ERR_ARG;
    (void)hipSetDevice(v->device);
    delete v;
    return ORBHIP_OK;
}

int orbhip_vocab_info(const orbhip_vocab* v, int32_t* k, int32_t* L, int32_t* n_nodes, int32_t* n_words) {
    if (!v) return ORBHIP_ERR_ARG;
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (n_nodes) *n_nodes = v->n_nodes;
    if (n_words) {
        int nw = 0;
        std::vector<int> w(v->n_nodes);
        if (hipMemcpy(w.data(), v->word_id.p, v->n_nodes * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
            return ORBHIP_ERR_DEVICE;
        for (int x : w) nw += x >= 0;
        *n_words = nw;
    }
    return ORBHIP_OK;
}

int orbhip_bow_transform(orbhip_ctx* c, const orbhip_vocab* v, const uint8_t* desc, int n, int levelsup,
                         int32_t* word, int32_t* node, double* weight) {
    if (!c || !v || n < 0 || (n && (!desc || !word || !node || !weight))) return ORBHIP_ERR_ARG;
    if (n == 0) return ORBHIP_OK;
    HIPOK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    HIPOK(c->d_mq.ensure((size_t)n * 32));
    HIPOK(c->d_mm.ensure(n)); HIPOK(c->d_mb.ensure(n)); HIPOK(c->d_bw.ensure(n));
    HIPOK(hipMemcpyAsync(c->d_mq.p, desc, (size_t)n * 32, hipMemcpyHostToDevice, st));
    (void)hipGetLastError();
    launch_bow_transform(v->view(), c->d_mq.p, nullptr, n, 1, n, levelsup, c->d_mm.p, c->d_mb.p, c->d_bw.p, st);
    HIPOK(hipGetLastError());
    HIPOK(hipMemcpyAsync(word, c->d_mm.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(node, c->d_mb.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(weight, c->d_bw.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    return ORBHIP_OK;
}

int orbhip_bow_transform_device(orbhip_ctx* c, const orbhip_vocab* v, const uint8_t* d_desc, const int32_t* d_n,
                                int B, int cap, int levelsup, int32_t* d_word, int32_t* d_node, double* d_weight,
                                void* stream) {
    if (!c || !v || !d_desc || !d_n || B <= 0 || cap <= 0 || !d_word || !d_node || !d_weight) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    (void)hipGetLastError();
    launch_bow_transform(v->view(), d_desc, d_n, 0, B, cap, levelsup, d_word, d_node, d_weight, (hipStream_t)stream);
    HIPOK(hipGetLastError());
    return ORBHIP_OK;
}

int orbhip_search_bow(orbhip_ctx* c, const uint8_t* kf_desc, const float* kf_angle, const int32_t* kf_node,
                      const double* kf_weight, const uint8_t* kf_valid, int nkf, const uint8_t* f_desc,
                      const float* f_angle, const int32_t* f_node, const double* f_weight, int nf, float ratio,
                      int check_orientation, int th_low, int32_t* match) {
    if (!c || nkf < 0 || nf < 0 || (nf && !match)) return ORBHIP_ERR_ARG;
    if (nkf > kBowMax || nf > kBowMax) return ORBHIP_ERR_UNSUPPORTED;
    if (nf == 0) return 0;
    for (int i = 0; i < nf; i++) match[i] = -1;
    if (nkf == 0) return 0;
    if (!kf_desc || !kf_angle || !kf_node || !kf_weight || !kf_valid || !f_desc || !f_angle || !f_node || !f_weight)
        return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    if (!search_bow_set_lds_limit()) return ORBHIP_ERR_DEVICE;   // once per device (dev_attr.h)
    // one staging block: [kf desc | f desc | kf angle | f angle | kf node | f node | kf w | f w | valid | match, n]
    const size_t bytes = (size_t)(nkf + nf) * 32 + (size_t)(nkf + nf) * (4 + 4 + 8) + nkf + (size_t)nf * 4 + 64;
    HIPOK(c->d_bow_stage.ensure(bytes + 64));
    uint8_t* base = c->d_bow_stage.p;
    size_t off = 0;
    auto place = [&](const void* src, size_t n_) -> uint8_t* {
        off = (off + 15) & ~size_t(15);
        uint8_t* d = base + off;
        if (src && n_) (void)hipMemcpyAsync(d, src, n_, hipMemcpyHostToDevice, st);
        off += n_;
        return d;
    };
    BowSide K, F;
    K.desc = place(kf_desc, (size_t)nkf * 32); F.desc = place(f_desc, (size_t)nf * 32);
    K.angle = (const float*)place(kf_angle, (size_t)nkf * 4); F.angle = (const float*)place(f_angle, (size_t)nf * 4);
    K.angle_stride = F.angle_stride = 1;
    K.node = (const int32_t*)place(kf_node, (size_t)nkf * 4); F.node = (const int32_t*)place(f_node, (size_t)nf * 4);
    K.weight = (const double*)place(kf_weight, (size_t)nkf * 8); F.weight = (const double*)place(f_weight, (size_t)nf * 8);
    K.valid = place(kf_valid, nkf); F.valid = nullptr;
    K.n = nkf; F.n = nf;
    int32_t* d_match = (int32_t*)place(nullptr, (size_t)nf * 4);
    int32_t* d_nm = (int32_t*)place(nullptr, 4);
    (void)hipGetLastError();
    launch_search_bow(K, F, ratio, check_orientation, th_low, d_match, d_nm, st);
    HIPOK(hipGetLastError());
    int nm = 0;
    HIPOK(hipMemcpyAsync(match, d_match, (size_t)nf * 4, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(&nm, d_nm, 4, hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    return nm;
}

// ---- test hooks (not part of the reference surface) ----
int orbhip_test_cholesky(const double* A, const double* b, double* x, int n, unsigned long long* phases5,
                         float* ms) {
    if (!A || !b || !x || n <= 0 || n > 480) return ORBHIP_ERR_ARG;
    return ba_test_cholesky(A, b, x, n, phases5, ms);
}
int orbhip_test_cholesky_reg(const double* A, const double* b, double* x, int n, int reps, float* ms,
                             unsigned long long* phases5) {
    if (!A || !b || !x || !ms) return ORBHIP_ERR_ARG;
    return ba_test_cholesky_reg(A, b, x, n, reps, ms, phases5);
}
int orbhip_test_cholesky_blocked(const double* A, const double* b, double* x, int n, float* ms) {
    if (!A || !b || !x || n <= 0 || !ms) return ORBHIP_ERR_ARG;
    return chol_blocked_test(A, b, x, n, ms);
}
int orbhip_test_cholesky_dag(const double* A, const double* b, double* x, int n, int reps, int max_helpers, float* ms,
                             unsigned long long* dbg) {
    if (!A || !b || !x || n <= 0 || reps < 1) return ORBHIP_ERR_ARG;
    return chol_dag_test(A, b, x, n, reps, max_helpers, ms, dbg);
}
// host only (no device): the BA preparation serial vs on host threads (identical lists -> 0)
int orbhip_test_ba_prepare(const orbhip_ba_problem* prob, int threads, double* out4) {
    if (!prob || threads < 1) return ORBHIP_ERR_ARG;
    return ba_test_prepare(prob, threads, out4);
}
// nested-dissection solve of a pose-structured SPD system (ba_nd.hip): K segments (0 = planned)
int orbhip_test_nd_solve(const double* A, const double* b, double* x, int np, const int* bi, const int* bj, int nblk,
                         int K, int reps, float* ms, int* K_used) {
    if (!A || !b || !x || np <= 0 || !bi || !bj || nblk <= 0 || reps < 1) return ORBHIP_ERR_ARG;
    return nd_test(A, b, x, np, bi, bj, nblk, K, reps, ms, K_used);
}
// the same, with the two halves timed alone (stage_ms[0]: interior factorizations + separator
// assembly, stage_ms[1]: separator solve + interior back-substitution) and the plan's segment
// starts (seg_out: the plan's K + 1 pose indices, then the band's half-width; capacity 65)
int orbhip_test_nd_stages(const double* A, const double* b, double* x, int np, const int* bi, const int* bj, int nblk,
                          int K, int reps, float* ms, int* K_used, float* stage_ms, int* seg_out) {
    if (!A || !b || !x || np <= 0 || !bi || !bj || nblk <= 0 || reps < 1 || !stage_ms || !seg_out) return ORBHIP_ERR_ARG;
    return nd_test(A, b, x, np, bi, bj, nblk, K, reps, ms, K_used, stage_ms, seg_out);
}

int orbhip_test_sincosf(const float* x, float* cs, float* sn, int64_t n) {
    if (!x || !cs || !sn || n <= 0) return ORBHIP_ERR_ARG;
    float *dx = nullptr, *dc = nullptr, *ds = nullptr;
    HIPOK(hipMalloc((void**)&dx, n * 4));
    HIPOK(hipMalloc((void**)&dc, n * 4));
    HIPOK(hipMalloc((void**)&ds, n * 4));
    HIPOK(hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice));
    launch_sincos_probe(dx, dc, ds, n, nullptr);
    HIPOK(hipDeviceSynchronize());
    HIPOK(hipMemcpy(cs, dc, n * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(sn, ds, n * 4, hipMemcpyDeviceToHost));
    (void)hipFree(dx); (void)hipFree(dc); (void)hipFree(ds);
    return ORBHIP_OK;
}

// Compare device sinf/cosf with host reference values over float bit range [lo, hi].
int64_t orbhip_test_sincosf_sweep(uint32_t lo, uint32_t hi, const float* ref_c, const float* ref_s) {
    if (hi < lo || !ref_c || !ref_s) return ORBHIP_ERR_ARG;
    const size_t n = (size_t)hi - lo + 1;
    float *dc = nullptr, *ds = nullptr;
    unsigned long long* dm = nullptr;
    unsigned long long hm = 0;
    if (hipMalloc((void**)&dc, n * 4) != hipSuccess) return ORBHIP_ERR_DEVICE;
    if (hipMalloc((void**)&ds, n * 4) != hipSuccess) return ORBHIP_ERR_DEVICE;
    if (hipMalloc((void**)&dm, 8) != hipSuccess) return ORBHIP_ERR_DEVICE;
    (void)hipMemset(dm, 0, 8);
    (void)hipMemcpy(dc, ref_c, n * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(ds, ref_s, n * 4, hipMemcpyHostToDevice);
    launch_sincos_sweep(lo, hi, dc, ds, dm, nullptr);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(&hm, dm, 8, hipMemcpyDeviceToHost);
    (void)hipFree(dc); (void)hipFree(ds); (void)hipFree(dm);
    return (int64_t)hm;
}

// Debug hook: run one frame and return the intermediates (pyramid levels 1.., candidates
// per cell, octree output per level) so a mismatch can be localised offline.
// pyr: sum_{l>=1} w_l*h_l bytes (packed, no pitch); cand: n_slots_total u32; cand_cnt:
// n_cells_total; lvl: kp_slots_total LevelKp (8 B each); lvl_cnt/lvl_nlap: n_levels.
int orbhip_test_extract_debug(orbhip_ctx* c, const uint8_t* img, int w, int h, int lap0, int lap1, uint8_t* pyr,
                              uint32_t* cand, int32_t* cand_cnt, void* lvl, int32_t* lvl_cnt, int32_t* lvl_nlap,
                              int32_t* sizes /* n_slots_total, n_cells_total, kp_slots_total, err */) {
    if (!c || !img) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    Plan* pl = nullptr;
    int rc = build_plan(c, w, h, &pl);
    if (rc) return rc;
    const ExtractPlan& P = pl->h;
    sizes[0] = P.n_slots_total; sizes[1] = P.n_cells_total; sizes[2] = P.kp_slots_total;
    if (!pyr) return ORBHIP_OK;   // size query
    const int kcap = pl->kp_cap_frame;
    HIPOK(c->d_in.ensure((size_t)w * h));
    HIPOK(c->d_kps.ensure(kcap));
    HIPOK(c->d_desc.ensure((size_t)kcap * 32));
    HIPOK(c->d_n.ensure(1));
    HIPOK(c->d_mono.ensure(1));
    hipStream_t st = c->stream;
    HIPOK(hipMemcpy2DAsync(c->d_in.p, w, img, w, w, h, hipMemcpyHostToDevice, st));
    rc = run_extract(c, pl, c->d_in.p, 1, w, (int64_t)w * h, lap0, lap1, c->d_kps.p, c->d_desc.p, kcap, c->d_n.p,
                     c->d_mono.p, st);
    if (rc) return rc;
    HIPOK(hipStreamSynchronize(st));
    size_t off = 0;
    for (int l = 1; l < P.n_levels; l++) {
        const LevelGeom& G = P.lv[l];
        HIPOK(hipMemcpy2D(pyr + off, G.w, c->d_pyr.p + G.pyr_off, G.pitch, G.w, G.h, hipMemcpyDeviceToHost));
        off += (size_t)G.w * G.h;
    }
    HIPOK(hipMemcpy(cand, c->d_cand.p, (size_t)P.n_slots_total * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(cand_cnt, c->d_cand_cnt.p, (size_t)P.n_cells_total * 4, hipMemcpyDeviceToHost));
    {   // each cell's first kCandPrim candidates sit in its primary slots: back into its slot range
        std::vector<uint32_t> prim((size_t)P.n_cells_total * kCandPrim);
        HIPOK(hipMemcpy(prim.data(), c->d_cprim.p, prim.size() * 4, hipMemcpyDeviceToHost));
        for (int ci = 0; ci < P.n_cells_total; ci++)
            for (int j = 0; j < std::min(cand_cnt[ci], kCandPrim); j++)
                cand[pl->cells[ci].slot_off + j] = prim[(size_t)ci * kCandPrim + j];
    }
    HIPOK(hipMemcpy(lvl, c->d_lvl_kp.p, (size_t)P.kp_slots_total * sizeof(LevelKp), hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(lvl_cnt, c->d_lvl_cnt.p, (size_t)P.n_levels * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(lvl_nlap, c->d_lvl_nlap.p, (size_t)P.n_levels * 4, hipMemcpyDeviceToHost));
    int err[4];
    HIPOK(hipMemcpy(err, c->d_err.p, sizeof(err), hipMemcpyDeviceToHost));
    sizes[3] = err[0];
    return ORBHIP_OK;
}

// Cell table of a plan (level, x0, y0, wc, hc, slot_off per cell) for offline checks.
// Device timing trace (diagnostics; see orbhip_device.h TR_*): on != 0 allocates a zeroed
// buffer of kTraceKernels x kTraceStride u64 and points every kernel unit at it; on == 0 copies
// it to `out` (if non-null, kTraceKernels * kTraceStride entries) and detaches it.
int orbhip_test_trace(int on, unsigned long long* out) {
    static unsigned long long* buf = nullptr;
    const size_t n = (size_t)kTraceKernels * kTraceStride;
    if (on) {
        if (!buf) HIPOK(hipMalloc((void**)&buf, n * sizeof(unsigned long long)));
        HIPOK(hipMemset(buf, 0, n * sizeof(unsigned long long)));
        trace_set_extract(buf);
        trace_set_match(buf);
        trace_set_proj(buf);
        return ORBHIP_OK;
    }
    HIPOK(hipDeviceSynchronize());
    if (buf && out) HIPOK(hipMemcpy(out, buf, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    trace_set_extract(nullptr);
    trace_set_match(nullptr);
    trace_set_proj(nullptr);
    return ORBHIP_OK;
}

// FAST candidates of frame `frame` of the context's last extraction at w x h (sum over its cells):
// the octree's input size, for the bench's algorithmic bytes of k_octree
int orbhip_test_candidates(orbhip_ctx* c, int w, int h, int frame, int64_t* n) {
    if (!c || !n || frame < 0) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    Plan* pl = nullptr;
    const int rc = build_plan(c, w, h, &pl);
    if (rc) return rc;
    const size_t nc = (size_t)pl->h.n_cells_total;
    if (!c->d_cand_cnt.p || c->d_cand_cnt.n < (frame + 1) * nc) return ORBHIP_ERR_ARG;
    std::vector<int> cnt(nc);
    HIPOK(hipStreamSynchronize(c->stream));
    HIPOK(hipDeviceSynchronize());
    HIPOK(hipMemcpy(cnt.data(), c->d_cand_cnt.p + frame * nc, nc * sizeof(int), hipMemcpyDeviceToHost));
    int64_t s = 0;
    for (int v : cnt) s += v;
    *n = s;
    return ORBHIP_OK;
}

int orbhip_test_cells(orbhip_ctx* c, int w, int h, int32_t* out6, int cap) {
    if (!c) return ORBHIP_ERR_ARG;
    Plan* pl = nullptr;
    int rc = build_plan(c, w, h, &pl);
    if (rc) return rc;
    const int n = (int)pl->cells.size();
    if (n > cap) return n;
    for (int i = 0; i < n; i++) {
        const CellGeom& g = pl->cells[i];
        out6[6 * i + 0] = g.level; out6[6 * i + 1] = g.x0; out6[6 * i + 2] = g.y0;
        out6[6 * i + 3] = g.wc; out6[6 * i + 4] = g.hc; out6[6 * i + 5] = g.slot_off;
    }
    return n;
}

}  // extern "C"

// ===========================================================================
// Camera front-end stream (orbhip_frontend_*): one camera's frames, each extracted at batch 1
// and matched to the previous frame, pipelined over S contexts (the contexts' own HIP streams,
// created back to back so they land on distinct hardware queues). Frame k runs on context
// k % S into output slot k % ns (ns = 2S; 2 for S = 1). Per frame the host issues: a wait for
// the slot's last cross-stream reader only if it has not finished (hipEventQuery; it is 2S - 1
// frames back, so normally done), the extraction, the extraction event, a wait on the previous
// frame's extraction event, the match (previous frame = queries, this frame = train, as the C2
// bench) and one event that also marks the frame complete. Same kernels and results as the
// one-frame calls; the host work per frame is one C call instead of the caller's bookkeeping.
// ===========================================================================
// Cone tile of the front-end's frames by the number of live front-ends (camera streams) in the
// process: one stream is latency-bound (10-pixel tiles, 252 work-groups at 640x480: 15.7k
// frames/s one frame at a time against 15.0k at 14), many streams share the chip and want less
// halo recompute per frame (16 cameras: 39.6k frames/s at 16-pixel tiles against 38.3k at 14;
// tools/gpu_cone_tile.sh). Both tilings give the same pyramid (every tile writes what it owns).
// Counted per device: a process driving one camera per GPU keeps every GPU at the one-camera choice.
constexpr int kMaxDevices = 64;
static std::atomic<int> g_live_frontends[kMaxDevices];
static std::atomic<int>& live_frontends(int device) { return g_live_frontends[device & (kMaxDevices - 1)]; }
static int frontend_cone_tile(int device) {
    const int n = live_frontends(device).load(std::memory_order_relaxed);
    return n >= 8 ? 16 : (n >= 2 ? 14 : 10);
}
// FAST threads per cell the same way: one camera keeps the one-frame rule (512 at 640x480, 15.8k
// frames/s against 15.4k at 256); 8+ cameras take 256 (16 cameras: 40.5k against 39.6k at 512,
// 35.6k at 1024; tools/gpu_c2_fastnt.sh)
static int frontend_fast_nt(int device) {
    return live_frontends(device).load(std::memory_order_relaxed) >= 8 ? 256 : 0;
}

struct orbhip_frontend {
    int device = 0, w = 0, h = 0, S = 0, ns = 0, cap = 0;
    int th_low = 50, check_orientation = 1;
    float ratio = 0.9f;
    int64_t k = 0;   // frames pushed
    std::vector<orbhip_ctx*> ctx;
    orbhip_kp* kps = nullptr;
    uint8_t* desc = nullptr;
    int32_t *n = nullptr, *mono = nullptr, *mm = nullptr, *nm = nullptr;
    std::vector<hipEvent_t> ev_x, ev_m;   // slot's extraction done / the match that read the slot as prev done
    std::vector<int64_t> frame_of;        // frame number held by each slot (-1 none)
    // one frame in flight (S = 1): completion is recorded on demand by wait (ev_done covers the
    // frames up to done_upto), not per push (an event per frame costs ~3% of the 16-camera rate)
    hipEvent_t ev_done = nullptr;
    int64_t done_upto = -1;
    bool live = false;   // counted in live_frontends(device)
};

static void frontend_free(orbhip_frontend* f) {
    if (!f) return;
    for (orbhip_ctx* c : f->ctx)
        if (c) (void)hipStreamSynchronize(c->stream);
    for (hipEvent_t e : f->ev_x)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : f->ev_m)
        if (e) (void)hipEventDestroy(e);
    if (f->ev_done) (void)hipEventDestroy(f->ev_done);
    if (f->kps) (void)hipFree(f->kps);
    if (f->desc) (void)hipFree(f->desc);
    if (f->n) (void)hipFree(f->n);
    if (f->mono) (void)hipFree(f->mono);
    if (f->mm) (void)hipFree(f->mm);
    if (f->nm) (void)hipFree(f->nm);
    for (orbhip_ctx* c : f->ctx)
        if (c) (void)orbhip_destroy(c);
    if (f->live) live_frontends(f->device).fetch_sub(1, std::memory_order_relaxed);
    delete f;
}

extern "C" {

int orbhip_frontend_create(orbhip_frontend** out, int device, const orbhip_orb_params* params, int w, int h,
                           int frames_in_flight, int th_low, float ratio, int check_orientation) {
    if (!out || w <= 0 || h <= 0 || frames_in_flight < 1 || frames_in_flight > 32) return ORBHIP_ERR_ARG;
    *out = nullptr;
    if (device < 0 && hipGetDevice(&device) != hipSuccess) return ORBHIP_ERR_DEVICE;   // as orbhip_create
    std::unique_ptr<orbhip_frontend, void (*)(orbhip_frontend*)> f(new orbhip_frontend(), frontend_free);
    f->device = device; f->w = w; f->h = h;
    f->S = frames_in_flight;
    f->ns = frames_in_flight == 1 ? 2 : 2 * frames_in_flight;
    f->th_low = th_low; f->ratio = ratio; f->check_orientation = check_orientation;
    f->ctx.assign(f->S, nullptr);
    for (int j = 0; j < f->S; j++) {
        if (int rc = orbhip_create(&f->ctx[j], device, params)) return rc;
        f->ctx[j]->cone_tile = 10;   // set per push (frontend_cone_tile)
    }
    live_frontends(device).fetch_add(1, std::memory_order_relaxed);
    f->live = true;
    const int cap = orbhip_max_keypoints(f->ctx[0], w, h);
    if (cap <= 0) return cap < 0 ? cap : ORBHIP_ERR_UNSUPPORTED;
    f->cap = cap;
    const size_t ns = (size_t)f->ns;
    HIPOK(hipMalloc((void**)&f->kps, sizeof(orbhip_kp) * cap * ns));
    HIPOK(hipMalloc((void**)&f->desc, 32 * (size_t)cap * ns));
    HIPOK(hipMalloc((void**)&f->n, 4 * ns));
    HIPOK(hipMalloc((void**)&f->mono, 4 * ns));
    HIPOK(hipMalloc((void**)&f->mm, 12 * (size_t)cap * ns));
    HIPOK(hipMalloc((void**)&f->nm, 4 * ns));
    f->ev_x.assign(ns, nullptr);
    f->ev_m.assign(ns, nullptr);
    f->frame_of.assign(ns, -1);
    for (size_t i = 0; i < ns; i++) {
        HIPOK(hipEventCreateWithFlags(&f->ev_x[i], hipEventDisableTiming));
        HIPOK(hipEventCreateWithFlags(&f->ev_m[i], hipEventDisableTiming));
    }
    HIPOK(hipEventCreateWithFlags(&f->ev_done, hipEventDisableTiming));
    *out = f.release();
    return ORBHIP_OK;
}

int orbhip_frontend_destroy(orbhip_frontend* f) {
    if (!f) return ORBHIP_ERR_ARG;
    (void)hipSetDevice(f->device);
    frontend_free(f);
    return ORBHIP_OK;
}

int orbhip_frontend_push(orbhip_frontend* f, const uint8_t* d_img, int stride, int lap0, int lap1) {
    if (!f || !d_img || stride < f->w) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(f->device));
    const int64_t k = f->k;
    const int S = f->S, ns = f->ns, cap = f->cap;
    const int j = (int)(k % S), cur = (int)(k % ns), prev = (int)((k + ns - 1) % ns);
    orbhip_ctx* c = f->ctx[j];
    c->cone_tile = frontend_cone_tile(f->device);
    c->fast_nt = frontend_fast_nt(f->device);
    hipStream_t st = c->stream;
    // slot `cur` was last read as `prev` by the match of frame k - ns + 1 (on another stream when
    // S > 1); its reader as `cur`, frame k - ns, ran on this stream
    if (S > 1 && k >= ns && hipEventQuery(f->ev_m[cur]) != hipSuccess) HIPOK(hipStreamWaitEvent(st, f->ev_m[cur], 0));
    orbhip_kp* kc = f->kps + (size_t)cur * cap;
    uint8_t* dc = f->desc + (size_t)cur * cap * 32;
    if (int rc = orbhip_extract_batch_device(c, d_img, 1, f->w, f->h, stride, (int64_t)stride * f->h, lap0, lap1, kc,
                                             dc, cap, f->n + cur, f->mono + cur, st))
        return rc;
    if (S > 1) HIPOK(hipEventRecord(f->ev_x[cur], st));   // the next frame's match (another stream) waits on it
    int32_t* m = f->mm + (size_t)cur * 3 * cap;
    if (k == 0) {
        HIPOK(hipMemsetAsync(f->nm + cur, 0xFF, 4, st));   // no previous frame: nmatch = -1
    } else {
        if (S > 1) HIPOK(hipStreamWaitEvent(st, f->ev_x[prev], 0));
        if (int rc = orbhip_match_frames_device(c, f->kps + (size_t)prev * cap, f->desc + (size_t)prev * cap * 32,
                                                f->n + prev, kc, dc, f->n + cur, cap, f->th_low, f->ratio,
                                                f->check_orientation, m, m + cap, m + 2 * cap, f->nm + cur, st))
            return rc;
    }
    // the match read `prev`, and frame k is complete (S = 1: recorded on demand by wait)
    if (S > 1) HIPOK(hipEventRecord(f->ev_m[prev], st));
    f->frame_of[cur] = k;
    f->k = k + 1;
    return cur;
}

int orbhip_frontend_view(orbhip_frontend* f, int slot, orbhip_frontend_slot* v) {
    if (!f || !v || slot < 0 || slot >= f->ns) return ORBHIP_ERR_ARG;
    const size_t cap = (size_t)f->cap;
    v->frame = f->frame_of[slot];
    v->cap = f->cap;
    v->slots = f->ns;
    v->kps = f->kps + slot * cap;
    v->desc = f->desc + slot * cap * 32;
    v->n = f->n + slot;
    v->mono = f->mono + slot;
    v->match = f->mm + (size_t)slot * 3 * cap;
    v->best = v->match + cap;
    v->second = v->match + 2 * cap;
    v->nmatch = f->nm + slot;
    return ORBHIP_OK;
}

int orbhip_frontend_wait(orbhip_frontend* f, int slot, void* stream) {
    if (!f || slot < 0 || slot >= f->ns || f->frame_of[slot] < 0) return ORBHIP_ERR_ARG;
    HIPOK(hipSetDevice(f->device));
    // frame k completes with the event its push recorded on ev_m[(k - 1) mod ns]; with S = 1
    // every frame runs on context 0's stream in order: record ev_done there if no record covers
    // this frame yet
    hipEvent_t e = f->ev_m[(slot + f->ns - 1) % f->ns];
    if (f->S == 1) {
        if (f->done_upto < f->frame_of[slot]) {
            HIPOK(hipEventRecord(f->ev_done, f->ctx[0]->stream));
            f->done_upto = f->k - 1;
        }
        e = f->ev_done;
    }
    if (stream) HIPOK(hipStreamWaitEvent((hipStream_t)stream, e, 0));
    else HIPOK(hipEventSynchronize(e));
    return ORBHIP_OK;
}

int orbhip_frontend_context(orbhip_frontend* f, int j, orbhip_ctx** out) {
    if (!f || !out || j < 0 || j >= f->S) return ORBHIP_ERR_ARG;
    *out = f->ctx[j];
    return ORBHIP_OK;
}

}  // extern "C"
