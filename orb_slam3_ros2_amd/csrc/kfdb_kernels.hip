// KeyFrameDatabase place-recognition queries on the device:
//   U:src/KeyFrameDatabase.cc::DetectRelocalizationCandidates(Frame* F, Map* pMap)
//   U:src/KeyFrameDatabase.cc::DetectNBestCandidates(pKF, vpLoopCand, vpMergeCand, nNumCandidates)
// with DBoW2 L1Scoring::score (Thirdparty/DBoW2/DBoW2/ScoringObject.cpp).
//
// MI355X formulation. The database keeps every KeyFrame's BowVector (ascending words, values)
// in one device pool, plus the KeyFrame members the queries read and write (mnRelocQuery,
// mnRelocWords, mRelocScore, mnPlaceRecognition*), which persist across queries as they do on
// the KeyFrames. The inverted file is implicit: a KeyFrame shares a word iff the word is in its
// BowVector, and the inverted-list order of a word is insertion order, so the reference's
// first-encounter order of the shared KeyFrames is (first common query word, insertion
// sequence). A query is two launches:
//   k_kfdb_share   one wave per KeyFrame slot: the query BowVector in LDS, each KF word binary-
//                  searched in it; common-word count, first common word, and the L1 score with
//                  the reference's summation order (terms compacted in word order, summed in
//                  order by one lane, fp64).
//   k_kfdb_select  one 1024-thread work-group: the shared list, 0.8 * max common words, member
//                  updates, first-encounter order (rank sort), covisibility accumulation over
//                  the 10 best covisible KFs, then the relocalisation filter (0.75 * best,
//                  same map, first occurrence of pBestKF) or the N-best walk (stable sort by
//                  accScore, loop / merge split by map).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/orbhip.h"
#include "kfdb.h"
#include "orbhip_device.h"

namespace orbhip {

namespace {

constexpr int kQMax = 3072;      // query BowVector words held in LDS (ORB-SLAM3: <= ~1250)
constexpr int kTermChunk = 512;  // scored terms per wave per summation chunk
constexpr int kCovis = 10;       // GetBestCovisibilityKeyFrames(10)

struct DbDev {
    const int32_t* pool_w;
    const double* pool_v;
    const int32_t* off;
    const int32_t* len;
    const long long* seq;
    const uint8_t* active;
    long long* m_query;   // mnRelocQuery | mnPlaceRecognitionQuery (by mode)
    int32_t* m_words;
    float* m_score;
    int n_slots;
};

__global__ __launch_bounds__(256) void k_kfdb_share(DbDev db, const int32_t* __restrict__ qw,
                                                    const double* __restrict__ qv, int nq,
                                                    int32_t* __restrict__ common, unsigned long long* __restrict__ firstkey,
                                                    double* __restrict__ score) {
    __shared__ int32_t sw[kQMax];
    __shared__ double sv[kQMax];
    __shared__ double terms[4][kTermChunk];
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    for (int i = tid; i < nq; i += 256) { sw[i] = qw[i]; sv[i] = qv[i]; }
    __syncthreads();
    const int s = blockIdx.x * 4 + wid;
    if (s >= db.n_slots) return;
    if (!db.active[s]) {
        if (lane == 0) common[s] = 0;
        return;
    }
    const int off = db.off[s], n = db.len[s];
    const int32_t* w = db.pool_w + off;
    const double* v = db.pool_v + off;
    int cnt = 0, first = INT_MAX;
    double acc = 0.0;   // lane 0: the running L1 sum in word order
    for (int c0 = 0; c0 < n; c0 += kTermChunk) {
        int nt = 0;
        for (int e0 = c0; e0 < min(n, c0 + kTermChunk); e0 += 64) {
            const int e = e0 + lane;
            int j = -1;
            double t = 0.0;
            if (e < n) {
                const int32_t x = w[e];
                int lo = 0, hi = nq - 1;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (sw[mid] < x) lo = mid + 1; else hi = mid;
                }
                if (nq > 0 && sw[lo] == x) {
                    j = lo;
                    const double vi = sv[lo], vj = v[e];
                    t = fabs(vi - vj) - fabs(vi) - fabs(vj);
                }
            }
            const uint64_t m = __ballot(j >= 0);
            if (j >= 0) {
                terms[wid][nt + __popcll(m & ((1ull << lane) - 1ull))] = t;
                first = min(first, j);
            }
            nt += __popcll(m);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0)
            for (int i = 0; i < nt; i++) acc += terms[wid][i];
        __builtin_amdgcn_wave_barrier();
        cnt += nt;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o, 64));
    if (lane == 0) {
        common[s] = cnt;
        firstkey[s] = ((unsigned long long)(uint32_t)first << 32) | (unsigned long long)(uint32_t)db.seq[s];
        score[s] = -acc / 2.0;
    }
}

__device__ __forceinline__ int block_max_i32(int v, int* scratch) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    int r = lane < nw ? scratch[lane] : INT_MIN;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r = max(r, __shfl_xor(r, o, 64));
    __syncthreads();
    return r;
}
__device__ __forceinline__ float block_max_f32(float v, float* scratch) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    float r = lane < nw ? scratch[lane] : -INFINITY;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r = fmaxf(r, __shfl_xor(r, o, 64));
    __syncthreads();
    return r;
}

// ordered compaction of flag[i] (i < n) into out (global), returns the count (block-uniform).
// Ends in a barrier: the callers read entries other threads wrote.
template <typename F>
__device__ int block_compact(int n, F&& pred, int32_t* __restrict__ out, int* scratch) {
    int run = 0;
    for (int i0 = 0; i0 < n; i0 += blockDim.x) {
        const int i = i0 + threadIdx.x;
        const int f = (i < n && pred(i)) ? 1 : 0;
        int tot;
        const int pos = block_excl_scan(f, scratch, &tot);
        if (f) out[run + pos] = i;
        run += tot;
    }
    __syncthreads();
    return run;
}

// Descending rank sort of n unique 64-bit keys (global) into out (global): out[#greater] = key.
__device__ void block_rank_sort_desc_g(const unsigned long long* __restrict__ a, unsigned long long* __restrict__ out,
                                       int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long x = a[i];
        int r = 0;
        for (int j = 0; j < n; j++) r += a[j] > x ? 1 : 0;
        out[r] = x;
    }
    __syncthreads();
}

struct SelScratch {
    int32_t* list;                 // shared KFs (slot ids, slot order)
    int32_t* scored;               // scored KFs (slot ids)
    unsigned long long* key;       // sort keys
    unsigned long long* key2;
    float* acc;                    // per entry (first-encounter order)
    int32_t* best;                 // pBestKF per entry
    int32_t* firstpos;             // per slot: first entry with that pBestKF (INT_MAX = none)
    int32_t* out;                  // results
    int32_t* counts;               // [0] reloc count / n_loop, [1] n_merge
};

// mode 0: relocalisation, 1: N-best (loop / merge)
__global__ __launch_bounds__(1024) void k_kfdb_select(DbDev db, int mode, long long qid,
                                                      const int32_t* __restrict__ common,
                                                      const unsigned long long* __restrict__ firstkey,
                                                      const double* __restrict__ score,
                                                      const int32_t* __restrict__ covis,
                                                      const uint8_t* __restrict__ connected,
                                                      const int32_t* __restrict__ kf_map, int query_map,
                                                      const uint8_t* __restrict__ flags, int ncand, SelScratch S) {
    __shared__ int scratch[20];
    __shared__ float fscratch[20];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int ns = db.n_slots;
    // 1. KFs sharing a word (connected KFs of the query KF never enter the N-best list)
    const int nl = block_compact(ns, [&](int s) { return common[s] > 0 && !(mode == 1 && connected && connected[s]); },
                                 S.list, scratch);
    if (nl == 0) {
        if (tid == 0) { S.counts[0] = 0; S.counts[1] = 0; }
        return;
    }
    int mx = 0;
    for (int i = tid; i < nl; i += nt) mx = max(mx, common[S.list[i]]);
    const int maxCommon = block_max_i32(mx, scratch);
    const int minCommon = (int)(maxCommon * 0.8f);
    // 2. member updates (query id, common words, the score of the scored ones)
    for (int i = tid; i < nl; i += nt) {
        const int s = S.list[i];
        db.m_query[s] = qid;
        db.m_words[s] = common[s];
        if (common[s] > minCommon) db.m_score[s] = (float)score[s];
    }
    __syncthreads();
    // 3. scored KFs in first-encounter order: rank sort of (first common word, insertion seq)
    const int nsc = block_compact(nl, [&](int i) { return common[S.list[i]] > minCommon; }, S.scored, scratch);
    for (int i = tid; i < nsc; i += nt) {
        const int s = S.list[S.scored[i]];
        S.scored[i] = s;
        S.key[i] = firstkey[s];   // unique: (first common query word, insertion sequence)
    }
    __syncthreads();
    // entry e = rank of the key among the scored ones (ascending); S.best[e] = its slot for now
    for (int i = tid; i < nsc; i += nt) {
        const unsigned long long k = S.key[i];
        int r = 0;
        for (int j = 0; j < nsc; j++) r += S.key[j] < k ? 1 : 0;
        S.best[r] = S.scored[i];
    }
    __syncthreads();
    // 4. covisibility accumulation (entry e: slot S.best[e])
    float bestAcc = 0.f;
    for (int e = tid; e < nsc; e += nt) {
        const int s = S.best[e];
        float best = db.m_score[s];
        float a = best;
        int pBest = s;
        for (int t = 0; t < kCovis; t++) {
            const int nb = covis[kCovis * s + t];
            if (nb < 0) break;
            if (db.m_query[nb] != qid) continue;
            const float sc = db.m_score[nb];
            a += sc;
            if (sc > best) { pBest = nb; best = sc; }
        }
        S.acc[e] = a;
        S.key[e] = (unsigned long long)pBest;   // pBestKF of entry e
        bestAcc = fmaxf(bestAcc, a);
    }
    __syncthreads();
    for (int e = tid; e < nsc; e += nt) S.best[e] = (int32_t)S.key[e];
    __syncthreads();
    if (mode == 0) {
        // 5a. relocalisation: acc > 0.75 * best, same map, first occurrence of pBestKF
        const float minRetain = 0.75f * block_max_f32(bestAcc, fscratch);
        auto keep = [&](int e) {
            return S.acc[e] > minRetain && !(kf_map && kf_map[S.best[e]] != query_map);
        };
        for (int e = tid; e < nsc; e += nt)
            if (keep(e)) atomicMin(&S.firstpos[S.best[e]], e);
        __syncthreads();
        const int m = block_compact(nsc, [&](int e) { return keep(e) && S.firstpos[S.best[e]] == e; }, S.out,
                                    scratch);
        for (int i = tid; i < m; i += nt) S.out[i] = S.best[S.out[i]];
        __syncthreads();
        for (int e = tid; e < nsc; e += nt) S.firstpos[S.best[e]] = INT_MAX;   // reset for the next query
        if (tid == 0) S.counts[0] = m;
    } else {
        // 5b. N best: stable sort by accScore descending, then the walk (one thread)
        for (int e = tid; e < nsc; e += nt) {
            // descending float key (accScore >= 0 here), ties by entry order ascending
            const uint32_t fb = __float_as_uint(S.acc[e]);
            const uint32_t ord = (fb & 0x80000000u) ? ~fb : (fb | 0x80000000u);
            S.key[e] = ((unsigned long long)ord << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)e);
        }
        __syncthreads();
        block_rank_sort_desc_g(S.key, S.key2, nsc);
        if (tid == 0) {
            int nlp = 0, nmg = 0;
            for (int r = 0; r < nsc && (nlp < ncand || nmg < ncand); r++) {
                const int e = (int)(0xFFFFFFFFu - (uint32_t)(S.key2[r] & 0xFFFFFFFFu));
                const int kfi = S.best[e];
                if (flags && (flags[kfi] & 1)) continue;
                if (S.firstpos[kfi] != INT_MAX) continue;   // already added
                S.firstpos[kfi] = e;
                const bool same = !kf_map || kf_map[kfi] == query_map;
                if (same && nlp < ncand) S.out[nlp++] = kfi;
                else if (!same && nmg < ncand && !(flags && (flags[kfi] & 2))) S.out[ncand + nmg++] = kfi;
            }
            S.counts[0] = nlp;
            S.counts[1] = nmg;
        }
        __syncthreads();
        for (int e = tid; e < nsc; e += nt) S.firstpos[S.best[e]] = INT_MAX;
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
#define KDOK(x)                                                                                    \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "orbhip kfdb: %s: %s\n", #x, hipGetErrorString(e_));              \
            return ORBHIP_ERR_DEVICE;                                                              \
        }                                                                                          \
    } while (0)

template <typename T>
static hipError_t dalloc(T** p, size_t n) { return hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)); }

struct KfDb {
    hipStream_t st = nullptr;
    int n_slots = 0;
    long long next_seq = 0;
    // pool
    int32_t* pool_w = nullptr;
    double* pool_v = nullptr;
    size_t pool_cap = 0, pool_fill = 0;
    // slots
    int32_t *off = nullptr, *len = nullptr;
    long long* seq = nullptr;
    uint8_t* active = nullptr;
    long long* rq = nullptr; int32_t* rw = nullptr; float* rs = nullptr;   // reloc members
    long long* pq = nullptr; int32_t* pw = nullptr; float* ps = nullptr;   // place recognition members
    std::vector<uint8_t> h_active;
    // per-query scratch
    int32_t *common = nullptr, *qw = nullptr, *covis = nullptr, *kf_map = nullptr;
    unsigned long long *firstkey = nullptr, *key = nullptr, *key2 = nullptr;
    double *score = nullptr, *qv = nullptr;
    uint8_t *connected = nullptr, *flags = nullptr;
    float* acc = nullptr;
    int32_t *list = nullptr, *scored = nullptr, *best = nullptr, *firstpos = nullptr, *out = nullptr, *counts = nullptr;
    ~KfDb() {
        void* ps_[] = {pool_w, pool_v, off, len, seq, active, rq, rw, rs, pq, pw, this->ps, common, qw, covis, kf_map,
                       firstkey, key, key2, score, qv, connected, flags, acc, list, scored, best, firstpos, out, counts};
        for (void* p : ps_)
            if (p) (void)hipFree(p);
    }
};

KfDb* kfdb_create(int max_kf, hipStream_t st, int* rc) {
    *rc = ORBHIP_ERR_DEVICE;
    if (max_kf <= 0 || max_kf > (1 << 24)) { *rc = ORBHIP_ERR_ARG; return nullptr; }
    KfDb* d = new KfDb();
    d->st = st;
    d->n_slots = max_kf;
    const size_t n = (size_t)max_kf;
    bool ok = dalloc(&d->off, n) == hipSuccess && dalloc(&d->len, n) == hipSuccess && dalloc(&d->seq, n) == hipSuccess &&
              dalloc(&d->active, n) == hipSuccess && dalloc(&d->rq, n) == hipSuccess && dalloc(&d->rw, n) == hipSuccess &&
              dalloc(&d->rs, n) == hipSuccess && dalloc(&d->pq, n) == hipSuccess && dalloc(&d->pw, n) == hipSuccess &&
              dalloc(&d->ps, n) == hipSuccess && dalloc(&d->common, n) == hipSuccess &&
              dalloc(&d->firstkey, n) == hipSuccess && dalloc(&d->score, n) == hipSuccess &&
              dalloc(&d->covis, n * kCovis) == hipSuccess && dalloc(&d->kf_map, n) == hipSuccess &&
              dalloc(&d->connected, n) == hipSuccess && dalloc(&d->flags, n) == hipSuccess &&
              dalloc(&d->key, n) == hipSuccess && dalloc(&d->key2, n) == hipSuccess && dalloc(&d->acc, n) == hipSuccess &&
              dalloc(&d->list, n) == hipSuccess && dalloc(&d->scored, n) == hipSuccess &&
              dalloc(&d->best, n) == hipSuccess && dalloc(&d->firstpos, n) == hipSuccess &&
              dalloc(&d->out, n + 64) == hipSuccess && dalloc(&d->counts, 4) == hipSuccess &&
              dalloc(&d->qw, kQMax) == hipSuccess && dalloc(&d->qv, kQMax) == hipSuccess;
    if (ok) {
        // members start as "never queried" (-1), slots inactive, firstpos empty
        ok = hipMemsetAsync(d->active, 0, n, st) == hipSuccess && hipMemsetAsync(d->rq, 0xFF, n * 8, st) == hipSuccess &&
             hipMemsetAsync(d->pq, 0xFF, n * 8, st) == hipSuccess && hipMemsetAsync(d->rw, 0, n * 4, st) == hipSuccess &&
             hipMemsetAsync(d->pw, 0, n * 4, st) == hipSuccess && hipMemsetAsync(d->rs, 0, n * 4, st) == hipSuccess &&
             hipMemsetAsync(d->ps, 0, n * 4, st) == hipSuccess &&
             hipMemsetD32Async((hipDeviceptr_t)d->firstpos, 0x7FFFFFFF, n, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
    }
    if (!ok) { delete d; return nullptr; }
    d->h_active.assign(n, 0);
    *rc = ORBHIP_OK;
    return d;
}

void kfdb_destroy(KfDb* d) { delete d; }

int kfdb_add(KfDb* d, int kf, const int32_t* words, const double* values, int n) {
    if (!d || kf < 0 || kf >= d->n_slots || n < 0 || (n > 0 && (!words || !values))) return ORBHIP_ERR_ARG;
    if (d->h_active[kf]) return ORBHIP_ERR_ARG;   // KeyFrameDatabase::add of a KF already in
    for (int i = 1; i < n; i++)
        if (words[i] <= words[i - 1]) return ORBHIP_ERR_ARG;   // a BowVector: ascending, unique
    if (d->pool_fill + n > d->pool_cap) {
        size_t cap = std::max<size_t>(d->pool_cap * 2, std::max<size_t>(d->pool_fill + n, 1 << 16));
        int32_t* nw = nullptr;
        double* nv = nullptr;
        KDOK(dalloc(&nw, cap));
        KDOK(dalloc(&nv, cap));
        if (d->pool_fill) {
            KDOK(hipMemcpyAsync(nw, d->pool_w, d->pool_fill * 4, hipMemcpyDeviceToDevice, d->st));
            KDOK(hipMemcpyAsync(nv, d->pool_v, d->pool_fill * 8, hipMemcpyDeviceToDevice, d->st));
        }
        KDOK(hipStreamSynchronize(d->st));
        if (d->pool_w) (void)hipFree(d->pool_w);
        if (d->pool_v) (void)hipFree(d->pool_v);
        d->pool_w = nw; d->pool_v = nv; d->pool_cap = cap;
    }
    const int32_t o = (int32_t)d->pool_fill;
    const long long sq = d->next_seq++;
    const uint8_t one = 1;
    if (n) {
        KDOK(hipMemcpyAsync(d->pool_w + o, words, (size_t)n * 4, hipMemcpyHostToDevice, d->st));
        KDOK(hipMemcpyAsync(d->pool_v + o, values, (size_t)n * 8, hipMemcpyHostToDevice, d->st));
    }
    KDOK(hipMemcpyAsync(d->off + kf, &o, 4, hipMemcpyHostToDevice, d->st));
    KDOK(hipMemcpyAsync(d->len + kf, &n, 4, hipMemcpyHostToDevice, d->st));
    KDOK(hipMemcpyAsync(d->seq + kf, &sq, 8, hipMemcpyHostToDevice, d->st));
    KDOK(hipMemcpyAsync(d->active + kf, &one, 1, hipMemcpyHostToDevice, d->st));
    KDOK(hipStreamSynchronize(d->st));   // the host values above are stack locals
    d->pool_fill += n;
    d->h_active[kf] = 1;
    return ORBHIP_OK;
}

int kfdb_erase(KfDb* d, int kf) {
    if (!d || kf < 0 || kf >= d->n_slots) return ORBHIP_ERR_ARG;
    const uint8_t zero = 0;
    KDOK(hipMemcpyAsync(d->active + kf, &zero, 1, hipMemcpyHostToDevice, d->st));
    KDOK(hipStreamSynchronize(d->st));
    d->h_active[kf] = 0;
    return ORBHIP_OK;
}

static int run_query(KfDb* d, int mode, const orbhip_kfdb_query* q, const uint8_t* connected, int ncand) {
    if (!q || q->n < 0 || q->n > kQMax || (q->n && (!q->words || !q->values)) || !q->covis) return ORBHIP_ERR_ARG;
    for (int i = 1; i < q->n; i++)
        if (q->words[i] <= q->words[i - 1]) return ORBHIP_ERR_ARG;
    const size_t ns = (size_t)d->n_slots;
    if (q->n) {
        KDOK(hipMemcpyAsync(d->qw, q->words, (size_t)q->n * 4, hipMemcpyHostToDevice, d->st));
        KDOK(hipMemcpyAsync(d->qv, q->values, (size_t)q->n * 8, hipMemcpyHostToDevice, d->st));
    }
    KDOK(hipMemcpyAsync(d->covis, q->covis, ns * kCovis * 4, hipMemcpyHostToDevice, d->st));
    if (q->kf_map) KDOK(hipMemcpyAsync(d->kf_map, q->kf_map, ns * 4, hipMemcpyHostToDevice, d->st));
    if (q->kf_flags) KDOK(hipMemcpyAsync(d->flags, q->kf_flags, ns, hipMemcpyHostToDevice, d->st));
    if (connected) KDOK(hipMemcpyAsync(d->connected, connected, ns, hipMemcpyHostToDevice, d->st));
    DbDev db{d->pool_w, d->pool_v, d->off, d->len, d->seq, d->active, mode ? d->pq : d->rq, mode ? d->pw : d->rw,
             mode ? d->ps : d->rs, d->n_slots};
    hipLaunchKernelGGL(k_kfdb_share, dim3((unsigned)((ns + 3) / 4)), dim3(256), 0, d->st, db, (const int32_t*)d->qw,
                       (const double*)d->qv, q->n, d->common, d->firstkey, d->score);
    SelScratch S{d->list, d->scored, d->key, d->key2, d->acc, d->best, d->firstpos, d->out, d->counts};
    hipLaunchKernelGGL(k_kfdb_select, dim3(1), dim3(1024), 0, d->st, db, mode, (long long)q->query_id,
                       (const int32_t*)d->common, (const unsigned long long*)d->firstkey, (const double*)d->score,
                       (const int32_t*)d->covis, connected ? (const uint8_t*)d->connected : nullptr,
                       q->kf_map ? (const int32_t*)d->kf_map : nullptr, q->query_map,
                       q->kf_flags ? (const uint8_t*)d->flags : nullptr, ncand, S);
    KDOK(hipGetLastError());
    return ORBHIP_OK;
}

int kfdb_detect_relocalization(KfDb* d, const orbhip_kfdb_query* q, int32_t* out, int cap) {
    if (!d || (cap > 0 && !out) || cap < 0) return ORBHIP_ERR_ARG;
    if (int rc = run_query(d, 0, q, nullptr, 0)) return rc;
    int32_t cnt[2] = {0, 0};
    KDOK(hipMemcpyAsync(cnt, d->counts, 8, hipMemcpyDeviceToHost, d->st));
    KDOK(hipStreamSynchronize(d->st));
    const int m = std::min(cnt[0], cap);
    if (m) {
        KDOK(hipMemcpyAsync(out, d->out, (size_t)m * 4, hipMemcpyDeviceToHost, d->st));
        KDOK(hipStreamSynchronize(d->st));
    }
    return cnt[0];
}

int kfdb_detect_nbest(KfDb* d, const orbhip_kfdb_query* q, const uint8_t* connected, int ncand, int32_t* loop_out,
                      int32_t* n_loop, int32_t* merge_out, int32_t* n_merge) {
    if (!d || ncand < 0 || ncand > 32 || !n_loop || !n_merge || (ncand > 0 && (!loop_out || !merge_out)))
        return ORBHIP_ERR_ARG;
    if (int rc = run_query(d, 1, q, connected, ncand)) return rc;
    int32_t cnt[2] = {0, 0};
    std::vector<int32_t> o((size_t)2 * ncand + 1);
    KDOK(hipMemcpyAsync(cnt, d->counts, 8, hipMemcpyDeviceToHost, d->st));
    KDOK(hipMemcpyAsync(o.data(), d->out, (size_t)(2 * ncand + 1) * 4, hipMemcpyDeviceToHost, d->st));
    KDOK(hipStreamSynchronize(d->st));
    *n_loop = cnt[0];
    *n_merge = cnt[1];
    for (int i = 0; i < cnt[0]; i++) loop_out[i] = o[i];
    for (int i = 0; i < cnt[1]; i++) merge_out[i] = o[ncand + i];
    return cnt[0] + cnt[1];
}

}  // namespace orbhip
