// Nested dissection of the reduced camera system (ba_nd.h): the plan, the separator assembly and
// the interiors' back-substitution; the factorizations themselves are the persistent tiled-DAG
// Cholesky (ba_chol_dag.hip) in its multi-problem partial form and its plain form.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ba_args.h"
#include "ba_chol_dag.h"
#include "ba_nd.h"
#include "dev_attr.h"
#include "wave_f64.h"

namespace orbhip {

namespace {

constexpr int kT = kDagTile;

// element (r, c) of a 32x32 tile in the DAG buffer's quadrant layout (ba_chol_dag.hip qidx)
__device__ __forceinline__ int tq(int r, int c) {
    return (((r >> 4) * 2 + (c >> 4)) * 256) + (((r & 15) + 16 * (c & 3)) * 4) + ((c & 15) >> 2);
}

struct NdSegDev {
    const double* buf;   // the segment's DAG buffer (L, Linv, y, the trailing block's contributions)
    const int* rf;       // its tile envelope
    const int* flag;     // [0]: its interior factored
    const int* perm;     // local row -> S row (-1 padding)
    const int* zmap;     // local row nip + j -> separator index
    int n, NT, nti, nip;
    int own0, own1;      // local rows of the segment's own separator (written back by this segment)
};

struct NdDev {
    const double* S;
    const double* bs;
    double* x;
    int* flag;
    const int* gate;
    int ld, K, nZ;
    const NdSegDev* segs;
    const int* zg;       // separator index -> S row
    const int* zsa;      // separator index -> first segment holding it (-1 none), local row zla
    const int* zla;
    const int* zsb;      // -> second segment (-1 none), local row zlb
    const int* zlb;
    const int* rfZ;
    double* SZ;
    double* bZ;
    const double* xZ;
    const int* flagZ;
    double* x_loc;       // shard of a distributed solve: its interior + own separator, [n] failure
    const double* xg;    // the shards' sum of x_loc
    int n;
};

// a segment's trailing-block contribution at local rows (li, lj) (symmetric; zero outside its envelope)
__device__ __forceinline__ double seg_contrib(const NdSegDev& s, int li, int lj) {
    if (li < lj) { const int t = li; li = lj; lj = t; }
    const int R = li / kT, C = lj / kT;
    if (C < s.rf[R]) return 0.0;
    return s.buf[dag_off_L(s.NT, R, C) + tq(li % kT, lj % kT)];
}

// S_Z row i (lower triangle inside its envelope) and bZ[i]: S's entries plus the contributions of
// the (at most two) segments whose trailing block holds both separator variables
__global__ __launch_bounds__(256) void k_nd_assemble(NdDev d) {
    if (d.gate && *d.gate != kPhTrial) return;
    const int i = blockIdx.x;
    const int gi = d.zg[i];
    const int sa = d.zsa[i], sb = d.zsb[i], la = d.zla[i], lb = d.zlb[i];
    const int c0 = kT * d.rfZ[i / kT];
    for (int j = c0 + (int)threadIdx.x; j <= i; j += blockDim.x) {
        const int gj = d.zg[j];
        double v = gi >= gj ? d.S[(size_t)gi * d.ld + gj] : d.S[(size_t)gj * d.ld + gi];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int sg = h ? sb : sa, li = h ? lb : la;
            if (sg < 0) continue;
            const int lj = d.zsa[j] == sg ? d.zla[j] : (d.zsb[j] == sg ? d.zlb[j] : -1);
            if (lj >= 0) v += seg_contrib(d.segs[sg], li, lj);
        }
        d.SZ[(size_t)i * d.nZ + j] = v;
    }
    if (threadIdx.x == 0) {
        double b = d.bs[gi];
        if (sa >= 0) b += d.segs[sa].buf[dag_off_R(d.segs[sa].NT, la / kT) + la % kT];
        if (sb >= 0) b += d.segs[sb].buf[dag_off_R(d.segs[sb].NT, lb / kT) + lb % kT];
        d.bZ[i] = b;
    }
}

// workgroup barrier ordering LDS only (__syncthreads() on gfx950 also drains vmcnt, i.e. would
// wait for the next step's prefetched tile loads)
__device__ __forceinline__ void lds_only_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// one workgroup per segment (4 waves): x of its separator rows from x_Z, then
// L_II^T x_I = y_I - L_ZI^T x_Z in two phases.
//   1. the separator rows' part of every interior column at once: y_R -= sum over separator tile
//      rows R' of L(R', R)^T x_R' (no dependency between columns: a stream of tile loads);
//   2. the banded back-substitution over the interior tiles only: at step R each wave adds the
//      products of its tiles of column R (rows R + 1 + w, + 4, ...) lane-locally, ONE set of
//      16-lane reductions per wave, then wave 0 forms x_R = Linv_R^T (y_R - sum) (one more).
// Tiles are read in their quadrant layout, 16 doubles per lane in four 32-byte loads (coalesced),
// one step ahead in two register sets. r04's form walked every tile of column R (separator rows
// included) with 16 scattered 8-byte loads per thread and tile and four barriers per step.
// A failed factorization anywhere (a segment or the separator system) zeroes x and flag.
// the segment buffers are reached through pointers loaded from memory (NdSegDev), which the
// compiler cannot place in an address space: without these casts every load is a flat load,
// counted in lgkmcnt too, so each LDS wait of a step would also wait for the prefetched tiles
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gp(const T* p) {
    return (const __attribute__((address_space(1))) T*)p;
}
typedef double dv4 __attribute__((ext_vector_type(4)));
// this lane's 16 values of a tile: quadrant qd, component q = element
// (16 (qd >> 1) + (l & 15), 16 (qd & 1) + (l >> 4) + 4 q)
__device__ __forceinline__ void tile_ld(const double* t, dv4 (&v)[4]) {
    const auto p = gp((const dv4*)t) + (threadIdx.x & 63);
#pragma unroll
    for (int qd = 0; qd < 4; qd++) v[qd] = p[64 * qd];
}
// p[b][q] += this lane's part of (tile^T x) for column 16 b + (l >> 4) + 4 q (its two rows)
__device__ __forceinline__ void tile_acc(const dv4 (&v)[4], const double* x, double (&p)[2][4]) {
    const int r = threadIdx.x & 15;
    const double x0 = x[r], x1 = x[16 + r];
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
        for (int q = 0; q < 4; q++) p[b][q] = fma(v[2 + b][q], x1, fma(v[b][q], x0, p[b][q]));
}
// the 16-lane sums: lanes with (l & 15) == 0 store column 16 b + (l >> 4) + 4 q to out
__device__ __forceinline__ void tile_red_store(double (&p)[2][4], double* out) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
        for (int q = 0; q < 4; q++) p[b][q] = row16_sum(p[b][q]);
    if ((lane & 15) == 0)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int q = 0; q < 4; q++) out[16 * b + (lane >> 4) + 4 * q] = p[b][q];
}

constexpr int kBsM = 2;   // tiles per wave and step held in registers (more are loaded in the step)
constexpr size_t kBsMaxLds = 128 * 1024;   // (below the 160 KB of a CU: the kernel has static LDS too)
// dynamic LDS of k_nd_backsolve for segments of at most maxNT tiles (the layout below): the
// planner keeps every segment within kBsMaxLds (84 tiles), nd_setup checks it again
constexpr size_t bs_lds_bytes(int maxNT) {
    return sizeof(double) * ((size_t)6 * maxNT * kDagTile + 5 * kDagTile) + sizeof(int) * (size_t)maxNT;
}

__global__ __launch_bounds__(256) void k_nd_backsolve(NdDev d) {
    if (d.gate && *d.gate != kPhTrial) return;
    // LDS: xs (NT x 32), ys (NT x 32), part1 (4 x NT x 32), part (4 x 32), sv (32), then NT ints
    extern __shared__ double xs[];
    const NdSegDev s = d.segs[blockIdx.x];
    const int NT = s.NT, nti = s.nti;
    double* ys = xs + NT * kT;
    double* part1 = ys + NT * kT;
    double* part = part1 + 4 * NT * kT;
    double* sv = part + 4 * kT;
    int* rfs = (int*)(sv + kT);
    __shared__ int okw;
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    double* xo = d.x_loc ? d.x_loc : d.x;
    if (tid == 0) okw = d.flagZ[0] != 0;
    for (int i = tid; i < NT; i += blockDim.x) rfs[i] = gp(s.rf)[i];
    for (int i = tid; i < NT * kT; i += blockDim.x) {
        double v = 0.0;
        if (i >= s.nip && i < s.n) v = gp(d.xZ)[gp(s.zmap)[i - s.nip]];
        xs[i] = v;
        ys[i] = i < nti * kT ? gp(s.buf)[dag_off_y(NT, i / kT) + i % kT] : 0.0;
    }
    __syncthreads();
    if (tid < d.K && gp(d.segs[tid].flag)[0] == 0) okw = 0;   // every segment factored (all in parallel)
    __syncthreads();
    const bool ok = okw != 0;
    if (blockIdx.x == 0 && tid == 0) {
        if (d.x_loc) d.x_loc[d.n] = ok ? 0.0 : 1.0;
        else d.flag[0] = ok;
    }
    if (ok && nti > 0) {
        // ---- phase 1: wave w takes separator tile rows nti + w, + 4, ... of every interior column,
        // the next column's first kBsM tiles loaded while this one's are summed ----
        {
            dv4 tv[2][kBsM][4];
            int rp[2][kBsM];
            auto load1 = [&](auto setc, int R) {
                constexpr int S = decltype(setc)::value;
                int Rp = nti + wid;
#pragma unroll
                for (int m = 0; m < kBsM; m++) {
                    while (Rp < NT && rfs[Rp] > R) Rp += 4;
                    rp[S][m] = Rp < NT && R < nti ? Rp : -1;
                    if (rp[S][m] >= 0) {
                        tile_ld(s.buf + dag_off_L(NT, Rp, R), tv[S][m]);
                        Rp += 4;
                    }
                }
            };
            auto col1 = [&](auto setc, int R) {
                constexpr int S = decltype(setc)::value;
                double p[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
                int last = -1;
#pragma unroll
                for (int m = 0; m < kBsM; m++)
                    if (rp[S][m] >= 0) { tile_acc(tv[S][m], xs + rp[S][m] * kT, p); last = rp[S][m]; }
                if (rp[S][kBsM - 1] >= 0)   // more separator tiles in this column: loaded here
                    for (int Rp = last + 4; Rp < NT; Rp += 4)
                        if (rfs[Rp] <= R) {
                            dv4 w4[4];
                            tile_ld(s.buf + dag_off_L(NT, Rp, R), w4);
                            tile_acc(w4, xs + Rp * kT, p);
                        }
                load1(setc, R + 2);
                tile_red_store(p, part1 + (wid * NT + R) * kT);
            };
            load1(std::integral_constant<int, 0>{}, 0);
            load1(std::integral_constant<int, 1>{}, 1);
            for (int R = 0; R < nti; R += 2) {
                col1(std::integral_constant<int, 0>{}, R);
                if (R + 1 < nti) col1(std::integral_constant<int, 1>{}, R + 1);
            }
        }
        __syncthreads();
        for (int i = tid; i < nti * kT; i += blockDim.x) {
            const int R = i / kT, c = i % kT;
            double t = 0.0;
#pragma unroll
            for (int w = 0; w < 4; w++) t += part1[(w * NT + R) * kT + c];
            ys[i] -= t;
        }
        __syncthreads();
        // ---- phase 2: the banded back-substitution over the interior tiles ----
        dv4 tv[2][kBsM][4], li[2][4];
        int rp[2][kBsM];
        auto load2 = [&](auto setc, int R) {
            constexpr int S = decltype(setc)::value;
            int Rp = R + 1 + wid;
#pragma unroll
            for (int m = 0; m < kBsM; m++) {
                while (Rp < nti && rfs[Rp] > R) Rp += 4;
                rp[S][m] = Rp < nti && R >= 0 ? Rp : -1;
                if (rp[S][m] >= 0) {
                    tile_ld(s.buf + dag_off_L(NT, Rp, R), tv[S][m]);
                    Rp += 4;
                }
            }
            if (wid == 0 && R >= 0) tile_ld(s.buf + dag_off_Linv(NT, R), li[S]);
        };
        auto step = [&](auto setc, int R) {
            constexpr int S = decltype(setc)::value;
            double p[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
            int last = -1;
#pragma unroll
            for (int m = 0; m < kBsM; m++)
                if (rp[S][m] >= 0) { tile_acc(tv[S][m], xs + rp[S][m] * kT, p); last = rp[S][m]; }
            if (rp[S][kBsM - 1] >= 0)
                for (int Rp = last + 4; Rp < nti; Rp += 4)
                    if (rfs[Rp] <= R) {
                        dv4 w4[4];
                        tile_ld(s.buf + dag_off_L(NT, Rp, R), w4);
                        tile_acc(w4, xs + Rp * kT, p);
                    }
            tile_red_store(p, part + wid * kT);
            lds_only_barrier();
            if (wid == 0) {
                if (lane < kT)
                    sv[lane] = ys[R * kT + lane] - ((part[lane] + part[kT + lane]) + (part[2 * kT + lane] + part[3 * kT + lane]));
                wave_lds_sync();
                double q[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
                tile_acc(li[S], sv, q);
                tile_red_store(q, xs + R * kT);
            }
            load2(setc, R - 2);
            lds_only_barrier();
        };
        load2(std::integral_constant<int, 0>{}, nti - 1);
        load2(std::integral_constant<int, 1>{}, nti - 2);
        for (int R = nti - 1; R >= 0; R -= 2) {
            step(std::integral_constant<int, 0>{}, R);
            if (R - 1 >= 0) step(std::integral_constant<int, 1>{}, R - 1);
        }
    }
    __syncthreads();
    for (int i = tid; i < s.nip; i += blockDim.x) {
        const int p = gp(s.perm)[i];
        if (p >= 0) xo[p] = ok ? xs[i] : 0.0;
    }
    for (int i = s.own0 + tid; i < s.own1; i += blockDim.x) xo[gp(s.perm)[i]] = ok ? xs[i] : 0.0;
}

// a shard's last step: the summed x, and the solve's flag (every shard's factorization and the
// separator system's)
__global__ __launch_bounds__(256) void k_nd_finish(NdDev d) {
    if (d.gate && *d.gate != kPhTrial) return;
    const bool ok = d.xg[d.n] == 0.0 && d.flagZ[0] != 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < d.n; i += gridDim.x * blockDim.x) d.x[i] = ok ? d.xg[i] : 0.0;
    if (blockIdx.x == 0 && threadIdx.x == 0) d.flag[0] = ok ? 1 : 0;
}

// the separator system's lower envelope <-> a packed buffer (tile row R: columns [32 rf[R], 32R + 32))
__global__ __launch_bounds__(256) void k_nd_env_pack(NdDev d, const long long* __restrict__ toff, double* __restrict__ buf,
                                                     int dir) {
    if (d.gate && *d.gate != kPhTrial) return;
    const int R = blockIdx.y, n = d.nZ;
    const int c0 = kT * d.rfZ[R], c1 = min(kT * R + kT, n), w = c1 - c0;
    const int rows = min(kT, n - kT * R);
    double* tb = buf + toff[R];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < rows * w; i += gridDim.x * blockDim.x) {
        const int r = i / w, c = i - r * w;
        double* e = d.SZ + (size_t)(kT * R + r) * n + c0 + c;
        if (dir == 0) tb[i] = *e;
        else *e = tb[i];
    }
}

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t ensure(size_t c) {
        if (p && c <= n) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; n = 0; }
        const hipError_t e = hipMalloc((void**)&p, std::max<size_t>(c, 1) * sizeof(T));
        if (e == hipSuccess) n = c;
        return e;
    }
};
template <typename T>
struct PinBuf {
    T* p = nullptr;
    size_t n = 0;
    ~PinBuf() { if (p) (void)hipHostFree(p); }
    hipError_t ensure(size_t c) {
        if (p && c <= n) return hipSuccess;
        if (p) { (void)hipHostFree(p); p = nullptr; n = 0; }
        c = std::max<size_t>(c + c / 4, 64);
        const hipError_t e = hipHostMalloc((void**)&p, c * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = c;
        return e;
    }
};

}  // namespace

struct NdWorkspace {
    DevBuf<double> dbl;
    DevBuf<int> ints;
    DevBuf<unsigned char> rec;
    PinBuf<int> hint;
    PinBuf<unsigned char> hrec;
    // launch state of the last nd_setup
    int K = 0, grid = 0;
    size_t lds = 0, bs_lds = 0;
    const void* d_ks = nullptr;
    const int* d_wgoff = nullptr;
    NdDev dev{};
    DagDev dZ{};
    int* rfZ = nullptr;
    int* flagZ = nullptr;
    std::vector<const int*> tw;
    DevBuf<long long> envoff;   // packed separator envelope: per tile row offsets
    DevBuf<double> pack, xl;    // the packed envelope; x_loc and xg (n + 1 each)
    size_t pack_n = 0;
    int nZt = 0;                // tile rows of the separator system
    NdWorkspace* inner = nullptr;   // the separator system's own dissection (second level), or none
    bool use_inner = false;
    ~NdWorkspace();
};

NdWorkspace* nd_create() { return new NdWorkspace(); }
void nd_destroy(NdWorkspace* w) { delete w; }
NdWorkspace::~NdWorkspace() { delete inner; }

void nd_timeout_words(const NdWorkspace* w, std::vector<const int*>& out) {
    out.insert(out.end(), w->tw.begin(), w->tw.end());
}

void nd_bandwidth(int np, const int* bi, const int* bj, int nblk, int& wl, int& wc) {
    wl = 0;
    wc = 0;
    for (int b = 0; b < nblk; b++) {
        const int d = std::abs(bj[b] - bi[b]);
        wl = std::max(wl, d);
        wc = std::max(wc, std::min(d, np - d));
    }
}

namespace {
// levels of the dissection: ORBHIP_ND_LEVELS=1 solves the separator system densely; 2 (default)
// dissects a cyclic separator system of >= 6 separators once more (nd_inner_plan)
int nd_levels() {
    const char* e = std::getenv("ORBHIP_ND_LEVELS");
    return e ? std::max(1, std::atoi(e)) : 2;
}

// the second level: the K separators of a cyclic dissection, w poses each, as a cyclic chain of
// K2 = K / 2 segments of two separators (the last one takes a third when K is odd): the even
// separators become interiors, the odd ones the separators of the separator system
bool nd_inner_plan(int nsep, int w, NdPlan& p) {
    if (nsep < 6 || 6 * w <= kT) return false;   // (interiors of one separator: more than one tile)
    // its longest segment (three separators' interior when nsep is odd, plus two separators) must
    // fit the back-substitution's LDS; otherwise the separator system is solved densely
    if (bs_lds_bytes((kT * ((6 * w * (nsep % 2 ? 2 : 1) + kT - 1) / kT) + 12 * w + kT - 1) / kT) > kBsMaxLds)
        return false;
    const int K2 = nsep / 2;
    p = NdPlan{};
    p.np = nsep * w; p.K = K2; p.w = w; p.cyclic = true;
    p.seg.assign(K2 + 1, 0);
    for (int r = 0; r < K2; r++) p.seg[r] = 2 * r * w;
    p.seg[K2] = nsep * w;
    return true;
}

int plan_cost(int np, int w, bool cyc, int k, std::vector<int>& seg) {
    auto tiles = [](int vars) { return (vars + kT - 1) / kT; };
    seg.assign(k + 1, 0);
    for (int r = 0; r <= k; r++) seg[r] = (int)((long long)r * np / k);
    const int nsep = cyc ? k : k - 1;
    int mi = 0;
    for (int r = 0; r < k; r++) {
        const bool own = cyc || r < k - 1;
        const int ni = seg[r + 1] - seg[r] - (own ? w : 0);
        // interiors at least as wide as the band (a block-tridiagonal separator system) and longer
        // than one tile (the partial DAG solve's chain forms two tile rows past its last interval)
        if (ni < w || 6 * ni <= kT) return -1;
        mi = std::max(mi, tiles(6 * ni));
        // the segment's matrix (interior padded to tiles + its two separators) must fit the
        // back-substitution's LDS (nd_setup: segment tiles NT)
        const int nseg = kT * tiles(6 * ni) + 6 * w * ((cyc || r > 0 ? 1 : 0) + (own ? 1 : 0));
        if (bs_lds_bytes(tiles(nseg)) > kBsMaxLds) return -1;
    }
    if (6 * w * nsep > kDagMaxN) return -1;   // the separator system on one DAG solve (nd_setup)
    int sep = tiles(6 * w * nsep);
    if (cyc && nd_levels() > 1 && nsep >= 6 && 6 * w > kT)   // the separator system dissected once more
        sep = std::min(sep, tiles(6 * w * (nsep % 2 ? 2 : 1)) + tiles(6 * w * (nsep / 2)) + 3);
    return mi + sep + 3;   // + the assembly / back-substitution / launches
}
}  // namespace

bool nd_plan_band(int np, int wl, int wc, int K, NdPlan& p) {
    p = NdPlan{};
    const bool cyc = wl > wc;
    const int w = std::max(1, cyc ? wc : wl);
    std::vector<int> seg;
    const int c = K >= 2 ? plan_cost(np, w, cyc, K, seg) : -1;
    if (c < 0) return false;
    p.np = np; p.K = K; p.w = w; p.cyclic = cyc; p.seg = seg; p.est_intervals = c;
    p.full_intervals = (6 * np + kT - 1) / kT;
    return true;
}

bool nd_plan(int np, const int* bi, const int* bj, int nblk, int K, NdPlan& p) {
    p = NdPlan{};
    if (np < 8) return false;
    int wl = 0, wc = 0;
    nd_bandwidth(np, bi, bj, nblk, wl, wc);
    const bool cyc = wl > wc;
    const int w = std::max(1, cyc ? wc : wl);
    std::vector<int> seg;
    int best = -1, bestK = 0;
    // every segment's factorization needs two workgroups (chain + a helper) resident together: K
    // is capped by the device's persistent grid (a partitioned or smaller device holds fewer)
    const int kcap = (dag_max_helpers() + 1) / 2;
    if (K > kcap) return false;
    const int k0 = K > 0 ? K : 2, k1 = K > 0 ? K : std::min(std::min(32, kcap), np / std::max(1, 2 * w));
    for (int k = k0; k <= k1; k++) {
        const int c = plan_cost(np, w, cyc, k, seg);
        if (c > 0 && (best < 0 || c < best)) { best = c; bestK = k; }
    }
    if (best < 0 || !nd_plan_band(np, wl, wc, bestK, p)) return false;
    // a forced K always plans; the automatic choice only when it pays
    return K > 0 || best * 10 <= p.full_intervals * 7;
}

bool nd_blocks_fit(const NdPlan& p, int r, const int* bi, const int* bj, int nblk) {
    const int K = p.K, w = p.w;
    const bool own = p.cyclic || r < K - 1, prev = p.cyclic || r > 0;
    auto in = [&](int q) {
        if (q >= p.seg[r] && q < p.seg[r + 1]) return true;   // the interior and the own separator
        if (!prev) return false;
        const int t = (r - 1 + K) % K, z0 = p.seg[t + 1] - w;
        return q >= z0 && q < z0 + w;
    };
    (void)own;
    for (int b = 0; b < nblk; b++)   // a pose's own block may be empty here (the solver lists every diagonal)
        if (bi[b] != bj[b] && (!in(bi[b]) || !in(bj[b]))) return false;
    return true;
}

int nd_setup(NdWorkspace* W, const NdPlan& P, const int* bi, const int* bj, int nblk, const double* S,
             const double* bs, double* x, int* flag, const int* gate, hipStream_t st, int seg_sel) {
    const int np = P.np, K = P.K, w = P.w, n = 6 * np;
    const bool cyc = P.cyclic;
    const int nsep = cyc ? K : K - 1;
    const int nZ = 6 * w * nsep;
    if (K < 2 || nZ <= 0 || nZ > kDagMaxN) return -5;
    // pose adjacency (both directions, itself included)
    std::vector<std::vector<int>> adj(np);
    for (int i = 0; i < np; i++) adj[i].push_back(i);
    for (int b = 0; b < nblk; b++)
        if (bi[b] != bj[b]) { adj[bi[b]].push_back(bj[b]); adj[bj[b]].push_back(bi[b]); }
    // separators: Z_t = poses [seg[t+1] - w, seg[t+1]), separator index 6 w t + ...
    auto sep_first = [&](int t) { return P.seg[t + 1] - w; };
    struct Seg {
        int prev, own, i0, i1, nip, n, NT, nti;
        std::vector<int> perm, rf, zmap;
        DagPlan plan;
    };
    std::vector<Seg> sg(K);
    const int helpers = dag_max_helpers();
    const int KL = seg_sel >= 0 ? 1 : K;   // segments factored here
    const int share = std::max(2, (helpers + 1) / KL);   // workgroups per segment (chain + helpers)
    for (int r = 0; r < K; r++) {
        Seg& s = sg[r];
        s.own = (cyc || r < K - 1) ? r : -1;
        s.prev = (cyc || r > 0) ? (r - 1 + K) % K : -1;
        s.i0 = P.seg[r];
        s.i1 = s.own >= 0 ? P.seg[r + 1] - w : P.seg[r + 1];
        const int ni = 6 * (s.i1 - s.i0);
        s.nip = (ni + kT - 1) / kT * kT;
        s.nti = s.nip / kT;
        s.n = s.nip + (s.prev >= 0 ? 6 * w : 0) + (s.own >= 0 ? 6 * w : 0);
        s.NT = (s.n + kT - 1) / kT;
        s.perm.assign(s.n, -1);
        std::vector<int> pos(np, -1);   // pose -> local row of its first variable
        for (int q = s.i0; q < s.i1; q++) {
            pos[q] = 6 * (q - s.i0);
            for (int c = 0; c < 6; c++) s.perm[6 * (q - s.i0) + c] = 6 * q + c;
        }
        int at = s.nip;
        for (int t : {s.prev, s.own}) {
            if (t < 0) continue;
            for (int q = sep_first(t); q < sep_first(t) + w; q++) {
                pos[q] = at;
                for (int c = 0; c < 6; c++) {
                    s.perm[at + c] = 6 * q + c;
                    s.zmap.push_back(6 * w * t + 6 * (q - sep_first(t)) + c);
                }
                at += 6;
            }
        }
        // tile envelope: first coupled local column of every row (padding rows: themselves)
        s.rf.assign(s.NT, 0);
        for (int R = 0; R < s.NT; R++) {
            int f = R;
            for (int i = kT * R; i < std::min(s.n, kT * R + kT); i++) {
                int first = i;
                const int pi = s.perm[i];
                if (pi >= 0)
                    for (int q : adj[pi / 6])
                        if (pos[q] >= 0) first = std::min(first, pos[q]);
                f = std::min(f, first / kT);
            }
            s.rf[R] = f;
        }
        if (seg_sel < 0 || seg_sel == r) dag_plan(s.rf.data(), s.n, share - 1, s.plan, s.nti);
    }
    std::vector<int> loc(K, -1);   // segment -> its index among the ones factored here
    for (int r = 0, i = 0; r < K; r++)
        if (seg_sel < 0 || seg_sel == r) loc[r] = i++;
    // separator system: envelope from direct couplings and the fill of each segment's elimination
    std::vector<int> rfZ((nZ + kT - 1) / kT);
    {
        std::vector<int> firstZ(nsep);   // first separator index coupled to separator t
        for (int t = 0; t < nsep; t++) firstZ[t] = 6 * w * t;
        for (int r = 0; r < K; r++)
            if (sg[r].prev >= 0 && sg[r].own >= 0) {
                const int a = sg[r].prev, b = sg[r].own;
                firstZ[a] = std::min(firstZ[a], 6 * w * b);
                firstZ[b] = std::min(firstZ[b], 6 * w * a);
            }
        // (no direct coupling between two separators: the interior between them is >= w poses wide, so
        // the envelope is the same on every shard of a distributed solve)
        for (size_t R = 0; R < rfZ.size(); R++) {
            int f = (int)R;
            for (int i = kT * (int)R; i < std::min(nZ, kT * (int)R + kT); i++) f = std::min(f, firstZ[i / (6 * w)] / kT);
            rfZ[R] = f;
        }
    }
    DagPlan pZ;
    dag_plan(rfZ.data(), nZ, helpers, pZ);
    // separator index -> (segment, local row), twice
    std::vector<int> zg(nZ), zsa(nZ, -1), zla(nZ, -1), zsb(nZ, -1), zlb(nZ, -1);
    for (int t = 0; t < nsep; t++)
        for (int j = 0; j < 6 * w; j++) zg[6 * w * t + j] = 6 * sep_first(t) + j;
    for (int r = 0; r < K; r++) {
        const Seg& s = sg[r];
        if (loc[r] < 0) continue;   // another shard's segment: its contributions are summed in there
        for (size_t j = 0; j < s.zmap.size(); j++) {
            const int z = s.zmap[j], l = s.nip + (int)j;
            if (zsa[z] < 0) { zsa[z] = loc[r]; zla[z] = l; }
            else { zsb[z] = loc[r]; zlb[z] = l; }
        }
    }
    // ---- sizes: doubles (128-byte aligned DAG buffers), ints, records ----
    auto al16 = [](size_t v) { return (v + 15) & ~size_t(15); };
    size_t nd = 0;
    std::vector<size_t> o_buf(K);
    for (int r = 0; r < K; r++)
        if (loc[r] >= 0) { o_buf[r] = nd; nd = al16(nd + dag_doubles(sg[r].n)); }
    const size_t o_bufZ = nd; nd = al16(nd + dag_doubles(nZ));
    const size_t o_SZ = nd; nd = al16(nd + (size_t)nZ * nZ);
    const size_t o_bZ = nd; nd = al16(nd + nZ);
    const size_t o_xZ = nd; nd = al16(nd + nZ);
    size_t ni = 0;
    auto ai4 = [](size_t v) { return (v + 3) & ~size_t(3); };
    struct SegOff { size_t perm, rf, ints, toff, tasks, flag, zmap; };
    std::vector<SegOff> so(K);
    for (int r = 0; r < K; r++) {
        const Seg& s = sg[r];
        if (loc[r] < 0) continue;
        so[r].ints = ni; ni = ai4(ni + dag_ints(s.n));
        so[r].perm = ni; ni = ai4(ni + s.n);
        so[r].rf = ni; ni = ai4(ni + s.NT);
        so[r].toff = ni; ni = ai4(ni + s.plan.toff.size());
        so[r].tasks = ni; ni = ai4(ni + s.plan.tasks.size());
        so[r].flag = ni; ni = ai4(ni + 4);
        so[r].zmap = ni; ni = ai4(ni + s.zmap.size());
    }
    const size_t oZ_ints = ni; ni = ai4(ni + dag_ints(nZ));
    const size_t oZ_rf = ni; ni = ai4(ni + rfZ.size());
    const size_t oZ_toff = ni; ni = ai4(ni + pZ.toff.size());
    const size_t oZ_tasks = ni; ni = ai4(ni + pZ.tasks.size());
    const size_t oZ_flag = ni; ni = ai4(ni + 4);
    const size_t o_zt = ni; ni = ai4(ni + 5 * (size_t)nZ);
    const size_t o_wg = ni; ni = ai4(ni + KL + 1);
    const size_t kb = (dag_k_bytes() + 15) & ~size_t(15);
    const size_t rb_ks = 0, rb_segs = KL * kb, rb = rb_segs + KL * sizeof(NdSegDev);
    if (W->dbl.ensure(nd) != hipSuccess || W->ints.ensure(ni) != hipSuccess || W->rec.ensure(rb) != hipSuccess ||
        W->hint.ensure(ni) != hipSuccess || W->hrec.ensure(rb) != hipSuccess)
        return -3;
    double* D = W->dbl.p;
    int* I = W->ints.p;
    int* H = W->hint.p;
    std::memset(H, 0, ni * sizeof(int));
    auto put = [&](size_t off, const std::vector<int>& v) { if (!v.empty()) std::memcpy(H + off, v.data(), v.size() * sizeof(int)); };
    std::vector<DagProb> probs(KL);
    std::vector<NdSegDev> segs(KL);
    W->tw.clear();
    for (int r = 0; r < K; r++) {
        const Seg& s = sg[r];
        if (loc[r] < 0) continue;
        put(so[r].perm, s.perm); put(so[r].rf, s.rf); put(so[r].toff, s.plan.toff); put(so[r].tasks, s.plan.tasks);
        put(so[r].zmap, s.zmap);
        DagProb& q = probs[loc[r]];
        q.S = S; q.ld = n; q.perm = I + so[r].perm; q.n = s.n; q.nti = s.nti; q.rf = I + so[r].rf; q.bs = bs;
        q.x = nullptr; q.flag = I + so[r].flag;
        q.d = DagDev{D + o_buf[r], I + so[r].ints, I + so[r].toff, I + so[r].tasks, s.plan.G, s.plan.pb,
                     s.plan.toff.empty() ? 0 : s.plan.toff[s.plan.G]};
        NdSegDev& g = segs[loc[r]];
        g.buf = D + o_buf[r]; g.rf = I + so[r].rf; g.flag = I + so[r].flag; g.perm = I + so[r].perm;
        g.zmap = I + so[r].zmap; g.n = s.n; g.NT = s.NT; g.nti = s.nti; g.nip = s.nip;
        g.own0 = g.own1 = 0;
        if (s.own >= 0) { g.own1 = s.n; g.own0 = s.n - 6 * w; }
        W->tw.push_back(I + so[r].ints + 3);
    }
    put(oZ_rf, rfZ); put(oZ_toff, pZ.toff); put(oZ_tasks, pZ.tasks);
    {
        std::vector<int> zt;
        zt.reserve(5 * (size_t)nZ);
        for (auto* v : {&zg, &zsa, &zla, &zsb, &zlb}) zt.insert(zt.end(), v->begin(), v->end());
        put(o_zt, zt);
    }
    W->tw.push_back(I + oZ_ints + 3);
    size_t lds = 0;
    const int grid = dag_multi_fill(probs.data(), KL, W->hrec.p + rb_ks, H + o_wg, gate, &lds);
    std::memcpy(W->hrec.p + rb_segs, segs.data(), KL * sizeof(NdSegDev));
    if (hipMemcpyAsync(I, H, ni * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(W->rec.p, W->hrec.p, rb, hipMemcpyHostToDevice, st) != hipSuccess)
        return -3;
    W->K = KL; W->grid = grid; W->lds = lds;
    W->d_ks = W->rec.p + rb_ks;
    W->d_wgoff = I + o_wg;
    NdDev& d = W->dev;
    d.S = S; d.bs = bs; d.x = x; d.flag = flag; d.gate = gate; d.ld = n; d.K = KL; d.nZ = nZ; d.n = n;
    d.segs = (const NdSegDev*)(W->rec.p + rb_segs);
    d.zg = I + o_zt; d.zsa = d.zg + nZ; d.zla = d.zsa + nZ; d.zsb = d.zla + nZ; d.zlb = d.zsb + nZ;
    d.rfZ = I + oZ_rf;
    d.SZ = D + o_SZ; d.bZ = D + o_bZ; d.xZ = D + o_xZ; d.flagZ = I + oZ_flag;
    W->dZ = DagDev{D + o_bufZ, I + oZ_ints, I + oZ_toff, I + oZ_tasks, pZ.G, pZ.pb, pZ.toff.empty() ? 0 : pZ.toff[pZ.G]};
    W->rfZ = I + oZ_rf;
    W->flagZ = I + oZ_flag;
    int maxNT = 0;
    for (int r = 0; r < K; r++)
        if (loc[r] >= 0) maxNT = std::max(maxNT, sg[r].NT);
    W->bs_lds = bs_lds_bytes(maxNT);
    if (W->bs_lds > kBsMaxLds) return -5;   // a segment too long for the back-substitution's LDS
    // shard of a distributed solve: the packed separator envelope and the x buffers
    d.x_loc = nullptr;
    d.xg = nullptr;
    W->nZt = (int)rfZ.size();
    if (seg_sel >= 0) {
        std::vector<long long> off(rfZ.size() + 1, 0);
        for (size_t R = 0; R < rfZ.size(); R++)
            off[R + 1] = off[R] + (long long)std::min(kT, nZ - kT * (int)R) *
                                      (std::min(kT * (int)R + kT, nZ) - kT * rfZ[R]);
        W->pack_n = (size_t)off.back();
        if (W->envoff.ensure(off.size()) != hipSuccess || W->pack.ensure(W->pack_n) != hipSuccess ||
            W->xl.ensure(2 * (size_t)(n + 1)) != hipSuccess)
            return -3;
        if (hipMemcpy(W->envoff.p, off.data(), off.size() * sizeof(long long), hipMemcpyHostToDevice) != hipSuccess)
            return -3;
        d.x_loc = W->xl.p;
        d.xg = W->xl.p + n + 1;
    }
    // the second level: a cyclic separator system of >= 6 separators is itself dissected (the even
    // separators eliminated in one more k_chol_dag_multi, the odd ones solved densely), which
    // replaces the dense solve's chain of nZ / 32 intervals by ~(6w + 6w K/2) / 32 + 3. Every
    // shard of a distributed solve runs it on the summed system (replicated: the levels' work is
    // spread over the CUs anyway, a collective per level would only add latency).
    W->use_inner = false;
    NdPlan P2;
    if (cyc && nd_levels() > 1 && nd_inner_plan(nsep, w, P2)) {
        std::vector<int> b2i, b2j;
        for (int t = 0; t < nsep; t++)   // every separator's own block
            for (int p = 0; p < w; p++)
                for (int q = p; q < w; q++) { b2i.push_back(t * w + p); b2j.push_back(t * w + q); }
        for (int r = 0; r < K; r++)   // the fill of each segment's elimination: Z_prev x Z_own
            if (sg[r].prev >= 0 && sg[r].own >= 0)
                for (int p = 0; p < w; p++)
                    for (int q = 0; q < w; q++) {
                        const int a = sg[r].prev * w + p, b = sg[r].own * w + q;
                        b2i.push_back(std::min(a, b));
                        b2j.push_back(std::max(a, b));
                    }
        if (!W->inner) W->inner = nd_create();
        const int rc = nd_setup(W->inner, P2, b2i.data(), b2j.data(), (int)b2i.size(), d.SZ, d.bZ,
                                const_cast<double*>(d.xZ), W->flagZ, gate, st, -1);
        if (rc != 0) return rc;
        W->use_inner = true;
        nd_timeout_words(W->inner, W->tw);
    }
    return 0;
}

hipError_t nd_factor_assemble(NdWorkspace* W, hipStream_t st) {
    const hipError_t e = chol_dag_multi_launch(W->d_ks, W->d_wgoff, W->K, W->grid, W->lds, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_nd_assemble, dim3((unsigned)W->dev.nZ), dim3(256), 0, st, W->dev);
    return hipGetLastError();
}

hipError_t nd_separator_backsolve(NdWorkspace* W, hipStream_t st) {
    const NdDev& d = W->dev;
    hipError_t e = W->use_inner ? nd_solve(W->inner, st)
                                : chol_dag_solve(d.SZ, d.nZ, W->rfZ, d.bZ, const_cast<double*>(d.xZ), W->flagZ, W->dZ,
                                                 st, d.gate);
    if (e != hipSuccess) return e;
    if (d.x_loc && (e = hipMemsetAsync(d.x_loc, 0, sizeof(double) * (d.n + 1), st)) != hipSuccess) return e;
    static LdsAttrOnce bs_attr;   // per device, thread-safe
    if ((e = bs_attr.ensure((const void*)k_nd_backsolve, (int)kBsMaxLds)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_nd_backsolve, dim3((unsigned)W->K), dim3(256), W->bs_lds, st, d);
    return hipGetLastError();
}

hipError_t nd_sep_pack(NdWorkspace* W, int dir, hipStream_t st) {
    hipLaunchKernelGGL(k_nd_env_pack, dim3(8, (unsigned)W->nZt), dim3(256), 0, st, W->dev, W->envoff.p, W->pack.p, dir);
    return hipGetLastError();
}

NdSepBufs nd_sep_bufs(NdWorkspace* W) {
    NdSepBufs b;
    b.pack = W->pack.p; b.pack_n = W->pack_n;
    b.bZ = W->dev.bZ; b.nZ = W->dev.nZ;
    b.x_loc = W->dev.x_loc; b.xg = const_cast<double*>(W->dev.xg);
    b.n = W->dev.n;
    return b;
}

hipError_t nd_finish(NdWorkspace* W, hipStream_t st) {
    hipLaunchKernelGGL(k_nd_finish, dim3((unsigned)std::max(1, std::min(64, (W->dev.n + 255) / 256))), dim3(256), 0, st,
                       W->dev);
    return hipGetLastError();
}

hipError_t nd_solve(NdWorkspace* W, hipStream_t st) {
    const hipError_t e = nd_factor_assemble(W, st);
    return e != hipSuccess ? e : nd_separator_backsolve(W, st);
}

int nd_test(const double* A, const double* b, double* x, int np, const int* bi, const int* bj, int nblk, int K,
            int reps, float* ms, int* K_used, float* stage_ms, int* seg_out) {
    NdPlan P;
    if (!nd_plan(np, bi, bj, nblk, K, P)) return -5;
    if (K_used) *K_used = P.K;
    if (seg_out) {   // the plan's segment starts (pose index), K + 1 entries, then the band's half-width
        for (int r = 0; r <= P.K; r++) seg_out[r] = P.seg[r];
        seg_out[P.K + 1] = P.w;
    }
    const int n = 6 * np;
    double *dA = nullptr, *db = nullptr, *dx = nullptr;
    int* dflag = nullptr;
    int rc = 0;
    auto ok = [&](hipError_t e) { if (e != hipSuccess && rc == 0) rc = -3; return e == hipSuccess; };
    ok(hipMalloc((void**)&dA, sizeof(double) * n * n));
    ok(hipMalloc((void**)&db, sizeof(double) * n));
    ok(hipMalloc((void**)&dx, sizeof(double) * n));
    ok(hipMalloc((void**)&dflag, 4 * sizeof(int)));
    NdWorkspace* W = nd_create();
    if (rc == 0) {
        ok(hipMemcpy(dA, A, sizeof(double) * n * n, hipMemcpyHostToDevice));
        ok(hipMemcpy(db, b, sizeof(double) * n, hipMemcpyHostToDevice));
        ok(hipMemset(dflag, 0, 4 * sizeof(int)));
        if (rc == 0 && nd_setup(W, P, bi, bj, nblk, dA, db, dx, dflag, nullptr, nullptr) != 0) rc = -3;
        if (rc == 0) ok(nd_solve(W, nullptr));   // warm-up
        ok(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        ok(hipEventCreate(&e0));
        ok(hipEventCreate(&e1));
        ok(hipEventRecord(e0, nullptr));
        for (int r = 0; r < reps && rc == 0; r++) ok(nd_solve(W, nullptr));
        ok(hipEventRecord(e1, nullptr));
        ok(hipDeviceSynchronize());
        float t = 0;
        ok(hipEventElapsedTime(&t, e0, e1));
        if (ms) *ms = t / std::max(1, reps);
        if (stage_ms && rc == 0) {   // the two halves alone: interiors + assembly, separator + back-substitution
            for (int st = 0; st < 2; st++) {
                ok(hipEventRecord(e0, nullptr));
                for (int r = 0; r < reps && rc == 0; r++)
                    ok(st == 0 ? nd_factor_assemble(W, nullptr) : nd_separator_backsolve(W, nullptr));
                ok(hipEventRecord(e1, nullptr));
                ok(hipDeviceSynchronize());
                float ts = 0;
                ok(hipEventElapsedTime(&ts, e0, e1));
                stage_ms[st] = ts / std::max(1, reps);
            }
            ok(nd_solve(W, nullptr));   // x and the flags of a whole solve again
            ok(hipDeviceSynchronize());
        }
        int f = 0;
        ok(hipMemcpy(&f, dflag, sizeof(int), hipMemcpyDeviceToHost));
        ok(hipMemcpy(x, dx, sizeof(double) * n, hipMemcpyDeviceToHost));
        std::vector<const int*> tw;
        nd_timeout_words(W, tw);
        for (const int* p : tw) {
            int v = 0;
            ok(hipMemcpy(&v, p, sizeof(int), hipMemcpyDeviceToHost));
            if (rc == 0 && v) rc = -7;
        }
        if (rc == 0 && !f) rc = -4;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    nd_destroy(W);
    (void)hipFree(dA); (void)hipFree(db); (void)hipFree(dx); (void)hipFree(dflag);
    return rc;
}

}  // namespace orbhip
