// gfx950 bag-of-words path:
//   k_bow_transform  DBoW2 TemplatedVocabulary::transform, one lane per descriptor: descend the
//                    k-ary tree keeping the first child at minimum Hamming distance (descriptors
//                    as two uint4, v_xor + v_bcnt); word id, IDF weight and the node at level
//                    L - levelsup. The vocabulary (~1.1 M nodes x 32 B for ORBvoc) stays in HBM /
//                    L2; the top levels are shared by every lane.
//   k_search_bow     ORBmatcher::SearchByBoW(KeyFrame, Frame), one 1024-thread workgroup per pair:
//                    both FeatureVectors are rank-sorted in LDS by (node, feature index); each wave
//                    takes a shared node and runs the reference's greedy loop over the node's KF
//                    features in index order (lanes = the node's frame features, skipping taken
//                    ones; best / second by (distance, index)); then the rotation histogram
//                    (HISTO_LENGTH 30, ComputeThreeMaxima) drops matches outside the main bins.
//                    Nodes never share a frame feature, so nodes are independent.
#include <hip/hip_runtime.h>

#include "orbhip_device.h"
#include "dev_attr.h"
#include "orbhip_kernels.h"

namespace orbhip {

__device__ __forceinline__ int ham2(uint4 a, uint4 b, uint4 c, uint4 d) {
    return __popc(a.x ^ c.x) + __popc(a.y ^ c.y) + __popc(a.z ^ c.z) + __popc(a.w ^ c.w) + __popc(b.x ^ d.x) +
           __popc(b.y ^ d.y) + __popc(b.z ^ d.z) + __popc(b.w ^ d.w);
}

__global__ __launch_bounds__(256) void k_bow_transform(VocabView V, const uint8_t* __restrict__ desc,
                                                       const int32_t* __restrict__ n_arr, int n_fixed, int cap,
                                                       int levelsup, int32_t* __restrict__ word,
                                                       int32_t* __restrict__ node, double* __restrict__ weight) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = n_arr ? n_arr[f] : n_fixed;
    if (i >= n) return;
    const uint4* q = (const uint4*)(desc + ((int64_t)f * cap + i) * 32);
    const uint4 qa = q[0], qb = q[1];
    const int nid_level = V.L - levelsup;
    int nid = 0, fid = 0, level = 0;
    do {
        ++level;
        const int* ch = V.children + V.first_child[fid];
        const int nc = V.n_child[fid];
        int best = ch[0];
        int bd = ham2(qa, qb, V.desc[2 * best], V.desc[2 * best + 1]);
        for (int c = 1; c < nc; c++) {
            const int id = ch[c];
            const int d = ham2(qa, qb, V.desc[2 * id], V.desc[2 * id + 1]);
            if (d < bd) { bd = d; best = id; }
        }
        fid = best;
        if (level == nid_level) nid = fid;
    } while (V.n_child[fid] > 0);
    const int64_t o = (int64_t)f * cap + i;
    word[o] = V.word_id[fid];
    weight[o] = V.weight[fid];
    node[o] = nid;
}

void launch_bow_transform(const VocabView& V, const uint8_t* desc, const int32_t* n_arr, int n_fixed, int B, int cap,
                          int levelsup, int32_t* word, int32_t* node, double* weight, hipStream_t st) {
    dim3 grid((unsigned)((cap + 255) / 256), (unsigned)B);
    hipLaunchKernelGGL(k_bow_transform, grid, dim3(256), 0, st, V, desc, n_arr, n_fixed, cap, levelsup, word, node,
                       weight);
}

// ---------------------------------------------------------------------------------------
struct SearchLds {
    unsigned long long ka[kBowMax], kb[kBowMax];   // KF keys (node << 16 | idx): raw, sorted
    unsigned long long fa[kBowMax], fb[kBowMax];   // frame keys
    int seg[kBowMax + 1];                           // starts of KF node runs in the sorted keys
    int8_t bin[kBowMax];                            // rotation bin of frame feature f's match
    int8_t taken[kBowMax];                          // by sorted frame position
    int hist[32];
    int keep[3];
    int cnt[4];
};

__device__ __forceinline__ void rank_sort_asc(const unsigned long long* a, unsigned long long* out, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long x = a[i];
        int r = 0;
        for (int j = 0; j < n; j++) r += a[j] < x ? 1 : 0;
        out[r] = x;
    }
}

__global__ __launch_bounds__(1024) void k_search_bow(BowSide K, BowSide F, float ratio, int check_orientation,
                                                     int th_low, int32_t* __restrict__ match,
                                                     int32_t* __restrict__ nmatch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    SearchLds& S = *(SearchLds*)smem_raw;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
    const int nk = K.n, nf = F.n;
    // ---- 1. FeatureVector keys (weight > 0; KF side: valid map point) ----
    if (tid < 4) S.cnt[tid] = 0;
    if (tid < 32) S.hist[tid] = 0;
    for (int i = tid; i < nf; i += blockDim.x) { match[i] = -1; S.bin[i] = -1; }
    __syncthreads();
    for (int i0 = 0; i0 < nk; i0 += blockDim.x) {
        const int i = i0 + tid;
        const bool in = i < nk && K.node[i] >= 0 && K.weight[i] > 0.0 && (!K.valid || K.valid[i]);
        int tot;
        const int pos = block_excl_scan(in ? 1 : 0, S.seg, &tot);
        if (in) S.ka[S.cnt[0] + pos] = ((unsigned long long)K.node[i] << 16) | (unsigned)i;
        __syncthreads();
        if (tid == 0) S.cnt[0] += tot;
        __syncthreads();
    }
    for (int i0 = 0; i0 < nf; i0 += blockDim.x) {
        const int i = i0 + tid;
        const bool in = i < nf && F.node[i] >= 0 && F.weight[i] > 0.0;
        int tot;
        const int pos = block_excl_scan(in ? 1 : 0, S.seg, &tot);
        if (in) S.fa[S.cnt[1] + pos] = ((unsigned long long)F.node[i] << 16) | (unsigned)i;
        __syncthreads();
        if (tid == 0) S.cnt[1] += tot;
        __syncthreads();
    }
    const int mk = S.cnt[0], mf = S.cnt[1];
    rank_sort_asc(S.ka, S.kb, mk);
    rank_sort_asc(S.fa, S.fb, mf);
    for (int i = tid; i < mf; i += blockDim.x) S.taken[i] = 0;
    __syncthreads();
    // ---- 2. KF node runs ----
    for (int i0 = 0; i0 < mk; i0 += blockDim.x) {
        const int i = i0 + tid;
        const bool head = i < mk && (i == 0 || (S.kb[i] >> 16) != (S.kb[i - 1] >> 16));
        int tot;
        const int pos = block_excl_scan(head ? 1 : 0, (int*)S.ka, &tot);   // ka is free now
        if (head) S.seg[S.cnt[2] + pos] = i;
        __syncthreads();
        if (tid == 0) S.cnt[2] += tot;
        __syncthreads();
    }
    const int nseg = S.cnt[2];
    if (tid == 0) S.seg[nseg] = mk;
    __syncthreads();
    const float factor = 1.0f / 30;
    // ---- 3. one wave per shared node: the reference's greedy loop ----
    for (int sgi = wid; sgi < nseg; sgi += nw) {
        const int a = S.seg[sgi], b = S.seg[sgi + 1];
        const unsigned long long nd = S.kb[a] >> 16;
        // frame range of the node: [lower_bound(nd << 16), lower_bound((nd + 1) << 16))
        int lo = 0, hi = mf;
        while (lo < hi) { const int m = (lo + hi) >> 1; if ((S.fb[m] >> 16) < nd) lo = m + 1; else hi = m; }
        const int fa = lo;
        hi = mf;
        while (lo < hi) { const int m = (lo + hi) >> 1; if ((S.fb[m] >> 16) <= nd) lo = m + 1; else hi = m; }
        const int fbnd = lo;
        if (fa == fbnd) continue;   // node absent from the frame
        for (int t = a; t < b; t++) {
            const int kidx = (int)(S.kb[t] & 0xFFFF);
            const uint4* kd = (const uint4*)(K.desc + (int64_t)kidx * 32);
            const uint4 ka = kd[0], kb2 = kd[1];
            int best = 256, bpos = 0x7fffffff, second = 256;
            for (int c0 = fa; c0 < fbnd; c0 += 64) {
                const int c = c0 + lane;
                int d = 256;
                if (c < fbnd && !S.taken[c]) {
                    const int fidx = (int)(S.fb[c] & 0xFFFF);
                    const uint4* fd = (const uint4*)(F.desc + (int64_t)fidx * 32);
                    d = ham2(ka, kb2, fd[0], fd[1]);
                }
                // chunk best by (distance, position) and the chunk's multiset second
                int key = (d << 20) | (c < fbnd ? (c - fa) : 0xFFFFF);
                int mn = key;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) mn = min(mn, __shfl_xor(mn, o, 64));
                const int cb = mn >> 20, cpos = (mn & 0xFFFFF) + fa;
                int d2 = (c == cpos) ? 256 : d;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) d2 = min(d2, __shfl_xor(d2, o, 64));
                // merge with the running (best, second): earlier chunks hold lower positions, so a
                // tie keeps the running best (first index wins, as the sequential scan)
                if (cb < best) { second = min(best, d2); best = cb; bpos = cpos; }
                else second = min(second, cb);
            }
            if (best <= th_low && (float)best < ratio * (float)second) {
                if (lane == 0) {
                    S.taken[bpos] = 1;
                    const int fidx = (int)(S.fb[bpos] & 0xFFFF);
                    match[fidx] = kidx;
                    int bin = -1;
                    if (check_orientation) {
                        float rot = K.angle[(int64_t)kidx * K.angle_stride] - F.angle[(int64_t)fidx * F.angle_stride];
                        if (rot < 0.0) rot += 360.0f;
                        bin = (int)roundf(rot * factor);
                        if (bin == 30) bin = 0;
                        atomicAdd(&S.hist[bin], 1);
                    }
                    S.bin[fidx] = (int8_t)bin;
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        }
    }
    __syncthreads();
    // ---- 4. rotation consistency ----
    if (check_orientation && tid == 0) {
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < 30; i++) {
            const int s = S.hist[i];
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
        S.keep[0] = ind1; S.keep[1] = ind2; S.keep[2] = ind3;
    }
    __syncthreads();
    int c = 0;
    for (int i = tid; i < nf; i += blockDim.x) {
        int m = match[i];
        if (m >= 0 && check_orientation) {
            const int bin = S.bin[i];
            if (bin != S.keep[0] && bin != S.keep[1] && bin != S.keep[2]) { m = -1; match[i] = -1; }
        }
        c += m >= 0;
    }
    c = wave_sum_i32(c);
    if (lane == 0) atomicAdd(&S.cnt[3], c);
    __syncthreads();
    if (tid == 0) *nmatch = S.cnt[3];
}

size_t search_bow_lds_bytes() { return sizeof(SearchLds); }

bool search_bow_set_lds_limit() {   // per device, thread-safe (dev_attr.h)
    static LdsAttrOnce attr;
    return attr.ensure((const void*)k_search_bow, (int)sizeof(SearchLds)) == hipSuccess;
}

void launch_search_bow(const BowSide& K, const BowSide& F, float ratio, int check_orientation, int th_low,
                       int32_t* match, int32_t* nmatch, hipStream_t st) {
    hipLaunchKernelGGL(k_search_bow, dim3(1), dim3(1024), sizeof(SearchLds), st, K, F, ratio, check_orientation,
                       th_low, match, nmatch);
}

}  // namespace orbhip
