// Host-visible launchers of the gfx950 kernels (one TU per kernel family, no RDC).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/orbhip.h"
#include "orbhip_plan.h"

namespace orbhip {

struct FrameBufs {
    const uint8_t* in;     // level 0: caller frames
    int in_stride;
    int64_t in_fstride;
    uint8_t* pyr;          // levels >= 1
    // live timing of the launch (stage timer, pyramid stage): the earliest workgroup start is
    // atomic-min'ed into stamp[0], the latest end (after its stores drained) max'ed into
    // stamp[kStampStride], both s_memrealtime; null: not timed
    unsigned long long* stamp = nullptr;
};
constexpr int kStampStride = 8192;   // == StageTimer::kCap

struct OctreeCfg {
    int node_cap;          // LDS node capacity (>= max list size of any level)
    int sort_cap;          // power of two >= node_cap
    int key_cap;           // keys kept in LDS when a level has <= key_cap candidates
    int lap0, lap1;        // vLappingArea
    int fast;              // 1: pyramid division first (sweep path as its fallback); 0: sweep path only
    int max_dh;            // deepest pyramid level allowed (<= 6; tests lower it to force the fallback)
};

// Live timing of one pipeline stage. The kernels launched between begin() and end() carry the
// timer's event pair (hipExtLaunchKernelGGL: the first launch the start event, every launch the
// stop event), so a pair spans the first kernel's start to the last kernel's end on the device:
// the execution-only duration rocprofv3's kernel trace reports, without the dispatch latency an
// event pair recorded on the stream around the launches would add.
struct StageTimer;
inline thread_local StageTimer* g_stage_timer = nullptr;   // the timer whose stage is open on this thread
struct StageTimer {
    int stage = 0;                    // selected stage id (0 = off)
    int n = 0;                        // recorded pairs
    static constexpr int kCap = 8192;
    hipEvent_t ev[2 * kCap];
    bool created = false;
    bool used = false;                // a kernel of the open stage carries this pair
    unsigned long long* dstamp = nullptr;   // device: kCap start minima, then kCap end maxima (FrameBufs::stamp)
    void begin(int s, hipStream_t) {
        if (s == stage && n < kCap) { used = false; g_stage_timer = this; }
    }
    void end(int s, hipStream_t) {
        if (s == stage && g_stage_timer == this) { g_stage_timer = nullptr; if (used) n++; }
    }
};
// closes whatever stage of `t` is still open when the scope ends (an early error return between
// begin() and end() must not leave g_stage_timer pointing at a timer that may be destroyed later)
struct StageScope {
    StageTimer& t;
    explicit StageScope(StageTimer& tm) : t(tm) {}
    ~StageScope() {
        if (g_stage_timer == &t) g_stage_timer = nullptr;
    }
};

// every pipeline-stage kernel launches through this (the stage timer's events when one is open)
#define ORBHIP_LAUNCH(kern, grid, block, shm, st, ...)                                                          \
    do {                                                                                                      \
        ::orbhip::StageTimer* t_ = ::orbhip::g_stage_timer;                                                   \
        if (t_) {                                                                                             \
            hipExtLaunchKernelGGL(kern, grid, block, (uint32_t)(shm), st, t_->used ? nullptr : t_->ev[2 * t_->n], \
                                  t_->ev[2 * t_->n + 1], 0u, __VA_ARGS__);                                    \
            t_->used = true;                                                                                  \
        } else {                                                                                              \
            hipLaunchKernelGGL(kern, grid, block, shm, st, __VA_ARGS__);                                      \
        }                                                                                                     \
    } while (0)

// ---- extraction ----
// s0 = 0: levels 1..L-1 from the frame (1024 threads per tile); s0 >= 1: levels s0+1..L-1 from
// pyramid level s0 (written by k_resize before), `nthreads` per tile
void launch_pyr_cone(const ExtractPlan* dP, int ntiles, size_t lds, const FrameBufs& fb, int B, const ConeRect* rects,
                     const int* ctab, int tab_stride, hipStream_t st, int s0 = 0, int nthreads = 1024,
                     const int* xofs = nullptr, const int* xalpha = nullptr, const int* yofs = nullptr,
                     const int* ybeta = nullptr);
// levels s0+1..L-1 in one launch, nbands row bands per frame (rows: [nbands][kMaxLevels] int2)
void launch_resize_bands(const ExtractPlan* dP, int nbands, const FrameBufs& fb, int B, int s0, const int2* rows,
                         const int* xofs, const int* xalpha, const int* yofs, const int* ybeta, hipStream_t st);
void launch_resize(const ExtractPlan* dP, const ExtractPlan& hP, const FrameBufs& fb, int B, int l,
                   const int* xofs, const int* xalpha, const int* yofs, const int* ybeta, hipStream_t st);
// k_pyr_flow (batches): levels 1..L-1 of every frame in one launch, a dataflow over 16-row bands
constexpr int kFlowQ = 8;         // task queues (frame f in queue f mod kFlowQ)
constexpr int kFlowChunk = 1;     // tickets taken per counter add
constexpr int kFlowCtl = 16;      // control ints ahead of the flags
struct PyrFlow {
    int* ctl;                     // [0, Q) queue tickets, [Q] work-groups out, [Q+1] generation, [Q+2] timed-out waits
    int* flags;                   // B x nbt band flags (zeroed once with ctl)
    const int2* dep;              // per (level >= 2, band): the level l-1 bands its source rows lie in
    int boff[kMaxLevels + 1];     // first band of each level (level 1 at 0), boff[l >= L] = nbt
    int B;
    int nbt;
    int pyr_limit;                // bytes of the batch's pyramid block (buffer resource range)
};
void launch_pyr_flow(const ExtractPlan* dP, const FrameBufs& fb, const int* xofs, const int* xalpha, const int* yofs,
                     const int* ybeta, const PyrFlow& a, hipStream_t st);
// Packed FAST candidates (batches): per (frame, level) fill counters, zeroed before the launch, and
// each cell's run offset (per frame); off == nullptr keeps each cell's fixed slot range
struct CandPack {
    int* fill = nullptr;   // B x kMaxLevels
    int* off = nullptr;    // B x n_cells_total
    // fixed slot ranges (off == nullptr): a cell's first kCandPrim candidates go to its primary
    // slots prim[(f n_cells_total + cell) kCandPrim ..], the rest to its slot range at the same
    // index; null: everything in the slot range
    uint32_t* prim = nullptr;
};
constexpr int kCandPrim = 16;
void launch_fast(const ExtractPlan* dP, const ExtractPlan& hP, const CellGeom* cells, const FrameBufs& fb, int B,
                 uint32_t* cand, int* cand_cnt, int* err, hipStream_t st, int nt_hint = 0, CandPack cp = {});
size_t octree_lds_bytes(const ExtractPlan& hP, const OctreeCfg& cfg);
bool octree_set_lds_limit(size_t bytes);
void launch_octree(const ExtractPlan* dP, const ExtractPlan& hP, const CellGeom* cells, const uint16_t* otab,
                   const uint32_t* cand, const uint32_t* cprim,
                   const int* cand_cnt, const int* cand_off, uint32_t* kscratch, uint16_t* nscratch, LevelKp* lvl_kp,
                   int* lvl_cnt, int* lvl_nlap, const OctreeCfg& cfg, int* err, int B, hipStream_t st,
                   unsigned long long* stamp = nullptr);
void launch_desc(const ExtractPlan* dP, const ExtractPlan& hP, const FrameBufs& fb, const LevelKp* lvl_kp,
                 const int* lvl_cnt, const int* lvl_nlap, const int* disc, orbhip_kp* out_kps, uint8_t* out_desc,
                 int cap, int* n_out, int* mono_out, int B, hipStream_t st);

// ---- matching ----
// `part`: scratch of match_part_entries(npairs, max queries, max train) x 8 bytes (chunk partials)
// `sync`: kMatchSyncInts zero-initialised ints kept by the caller across launches (the one-launch
// matcher's counters, reset by each launch); null = the two-kernel path
constexpr int kMatchSyncInts = 64 * 4;
size_t match_part_entries(int npairs, int max_q, int max_t);
void launch_match_pairs(const orbhip_kp* kps, const uint8_t* desc, const int32_t* n, int npairs, int cap,
                        int th_low, float ratio, int check_orientation, int32_t* match, int32_t* best,
                        int32_t* second, int32_t* nmatch, void* part, hipStream_t st, StageTimer* timer,
                        int* sync);
void launch_match_frames(const orbhip_kp* q_kps, const uint8_t* q_desc, const int32_t* nq, const orbhip_kp* t_kps,
                         const uint8_t* t_desc, const int32_t* nt, int cap, int th_low, float ratio,
                         int check_orientation, int32_t* match, int32_t* best, int32_t* second, int32_t* nmatch,
                         void* part, hipStream_t st, StageTimer* timer, int* sync);
void launch_match_bf(const uint8_t* q, const float* qa, int nq, const uint8_t* t, const float* ta, int nt,
                     int th_low, float ratio, int check_orientation, int32_t* match, int32_t* best,
                     int32_t* second, int32_t* nmatch, void* part, hipStream_t st,
                     int* sync);

// ---- bag of words ----
constexpr int kBowMax = 2048;   // features per frame in SearchByBoW (LDS-resident FeatureVectors)
struct VocabView {
    const uint4* desc;          // n_nodes x 2 uint4
    const int* first_child;     // CSR, children in file order
    const int* n_child;
    const int* children;
    const int* word_id;         // -1 for internal nodes
    const double* weight;
    int L;
};
struct BowSide {
    const uint8_t* desc;        // n x 32
    const float* angle;         // keypoint angles, angle_stride floats apart
    int angle_stride;
    const int32_t* node;        // FeatureVector node (transform output)
    const double* weight;       // word weight (FeatureVector holds weight > 0 only)
    const uint8_t* valid;       // KF side: feature has a good map point (null on the frame side)
    int n;
};
void launch_bow_transform(const VocabView& V, const uint8_t* desc, const int32_t* n_arr, int n_fixed, int B, int cap,
                          int levelsup, int32_t* word, int32_t* node, double* weight, hipStream_t st);
size_t search_bow_lds_bytes();
bool search_bow_set_lds_limit();
void launch_search_bow(const BowSide& K, const BowSide& F, float ratio, int check_orientation, int th_low,
                       int32_t* match, int32_t* nmatch, hipStream_t st);

// ---- ingest ----
void launch_bgr2gray(const uint8_t* src, int B, int w, int h, int sstride, int64_t sfstride, uint8_t* dst, int dstride,
                     int64_t dfstride, hipStream_t st);

// ---- distorted pinhole camera (Frame::UndistortKeyPoints / ComputeImageBounds) ----
void launch_undistort_kps(const orbhip_kp* kps, const int32_t* n_arr, int n_fixed, int B, int cap,
                          const orbhip_pinhole& cam, orbhip_kp* out, hipStream_t st);
void launch_image_bounds(int cols, int rows, const orbhip_pinhole& cam, float* bounds, hipStream_t st);

// ---- test hooks ----
constexpr int kTraceStride = 16384;   // u64 per kernel id in the timing trace (orbhip_device.h)
constexpr int kTraceKernels = 8;
void trace_set_extract(unsigned long long* p);
void trace_set_match(unsigned long long* p);
void trace_set_proj(unsigned long long* p);
void launch_sincos_probe(const float* x, float* c, float* s, int64_t n, hipStream_t st);
void launch_sincos_sweep(uint32_t lo_bits, uint32_t hi_bits, const float* ref_c, const float* ref_s,
                         unsigned long long* mismatches, hipStream_t st);

}  // namespace orbhip
