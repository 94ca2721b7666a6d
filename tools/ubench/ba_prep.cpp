// CPU microbenchmark of the BA host preparation's structure build (ba_solver.hip prepare()):
// the r03 serial form, a row-wise form (each pose row builds its own blocks and pairs in a few KB)
// and serial2 (the form ba_solver.hip now has: one load per pair endpoint, the dense counts turned
// into fill cursors in place, scratch kept across calls), on edge lists dumped from
// synthetic_ba_problem (C4 / C5), and serial3 (serial2's pair passes over T landmark ranges on
// T threads). Checks that all produce identical lists. r04 on this container's CPU at C5: serial
// 3.1-3.7 ms, row-wise ~1.8x slower, serial2 1.9-2.3 ms, serial3 2.4 (T=2) / 2.8 (T=4): the
// threads' start-up and the T dense count arrays cost more than the split passes save.
//   g++ -O2 -std=c++17 -pthread tools/ubench/ba_prep.cpp -o /tmp/ba_prep && /tmp/ba_prep ep.bin et.bin fx.bin
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static std::vector<char> slurp(const char* f) {
    std::vector<char> v;
    FILE* fp = std::fopen(f, "rb");
    if (!fp) return v;
    char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) v.insert(v.end(), buf, buf + n);
    std::fclose(fp);
    return v;
}

struct Out {
    std::vector<int> opt, pt_ptr, pt_edges, ps_ptr, ps_edges, blk_i, blk_j, blk_ptr, blk_pairs;
    int np = 0;
};

static double now() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void serial(int P, int M, int E, const int* e_pose, const int* e_pt, const unsigned char* fixed, Out& o, double* t) {
    double t0 = now();
    o.opt.assign(P, -1);
    int np = 0;
    for (int i = 0; i < P; i++)
        if (!fixed[i]) o.opt[i] = np++;
    o.np = np;
    o.pt_ptr.assign(M + 1, 0);
    o.ps_ptr.assign(np + 1, 0);
    for (int e = 0; e < E; e++) {
        o.pt_ptr[e_pt[e] + 1]++;
        if (o.opt[e_pose[e]] >= 0) o.ps_ptr[o.opt[e_pose[e]] + 1]++;
    }
    for (int m = 0; m < M; m++) o.pt_ptr[m + 1] += o.pt_ptr[m];
    for (int i = 0; i < np; i++) o.ps_ptr[i + 1] += o.ps_ptr[i];
    o.pt_edges.resize(E);
    o.ps_edges.resize(o.ps_ptr[np]);
    {
        std::vector<int> fp(o.pt_ptr.begin(), o.pt_ptr.end() - 1), fq(o.ps_ptr.begin(), o.ps_ptr.end() - 1);
        for (int e = 0; e < E; e++) {
            o.pt_edges[fp[e_pt[e]]++] = e;
            const int oi = o.opt[e_pose[e]];
            if (oi >= 0) o.ps_edges[fq[oi]++] = e;
        }
    }
    t[0] += now() - t0; t0 = now();
    std::vector<int> cnt((size_t)np * np, 0);
    size_t npairs = 0;
    for (int m = 0; m < M; m++)
        for (int ka = o.pt_ptr[m]; ka < o.pt_ptr[m + 1]; ka++) {
            const int ia = o.opt[e_pose[o.pt_edges[ka]]];
            if (ia < 0) continue;
            for (int kb = o.pt_ptr[m]; kb < o.pt_ptr[m + 1]; kb++) {
                const int ib = o.opt[e_pose[o.pt_edges[kb]]];
                if (ib < 0 || ib < ia) continue;
                cnt[(size_t)ia * np + ib]++;
                npairs++;
            }
        }
    t[1] += now() - t0; t0 = now();
    std::vector<int> bid((size_t)np * np, -1);
    o.blk_ptr.assign(1, 0);
    for (int i = 0; i < np; i++)
        for (int j = i; j < np; j++) {
            const size_t k = (size_t)i * np + j;
            if (i == j || cnt[k] > 0) {
                bid[k] = (int)o.blk_i.size();
                o.blk_i.push_back(i);
                o.blk_j.push_back(j);
                o.blk_ptr.push_back(o.blk_ptr.back() + cnt[k]);
            }
        }
    t[2] += now() - t0; t0 = now();
    o.blk_pairs.resize(2 * npairs);
    std::vector<int> fill(o.blk_ptr.begin(), o.blk_ptr.end() - 1);
    for (int m = 0; m < M; m++)
        for (int ka = o.pt_ptr[m]; ka < o.pt_ptr[m + 1]; ka++) {
            const int ea = o.pt_edges[ka], ia = o.opt[e_pose[ea]];
            if (ia < 0) continue;
            for (int kb = o.pt_ptr[m]; kb < o.pt_ptr[m + 1]; kb++) {
                const int eb = o.pt_edges[kb], ib = o.opt[e_pose[eb]];
                if (ib < 0 || ib < ia) continue;
                const int slot = fill[bid[(size_t)ia * np + ib]]++;
                o.blk_pairs[2 * slot] = ea;
                o.blk_pairs[2 * slot + 1] = eb;
            }
        }
    t[3] += now() - t0;
}

template <typename F>
static void pfor(int n, int threads, F fn) {   // fn(t, lo, hi) over contiguous ranges
    threads = std::max(1, std::min(threads, n));
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++)
        pool.emplace_back([&, t] { fn(t, (int)((long long)n * t / threads), (int)((long long)n * (t + 1) / threads)); });
    fn(0, 0, (int)((long long)n / threads));
    for (auto& th : pool) th.join();
}

// row-wise: pose row ia walks its landmarks (landmark order) and their edges with opt >= ia; a
// row's blocks are consecutive in the (i, j) block order, so its counts, cursors and pair writes
// stay in a few KB; rows are independent given the rows' block / pair offsets
static void rowwise(int P, int M, int E, const int* e_pose, const int* e_pt, const unsigned char* fixed, Out& o,
                    double* t, int nth) {
    double t0 = now();
    o.opt.assign(P, -1);
    int np = 0;
    for (int i = 0; i < P; i++)
        if (!fixed[i]) o.opt[i] = np++;
    o.np = np;
    o.pt_ptr.assign(M + 1, 0);
    o.ps_ptr.assign(np + 1, 0);
    for (int e = 0; e < E; e++) {
        o.pt_ptr[e_pt[e] + 1]++;
        if (o.opt[e_pose[e]] >= 0) o.ps_ptr[o.opt[e_pose[e]] + 1]++;
    }
    for (int m = 0; m < M; m++) o.pt_ptr[m + 1] += o.pt_ptr[m];
    for (int i = 0; i < np; i++) o.ps_ptr[i + 1] += o.ps_ptr[i];
    o.pt_edges.resize(E);
    o.ps_edges.resize(o.ps_ptr[np]);
    std::vector<int> eopt(E), epm(E);   // per pt_edges slot: its pose's opt index, its landmark
    {
        std::vector<int> fp(o.pt_ptr.begin(), o.pt_ptr.end() - 1), fq(o.ps_ptr.begin(), o.ps_ptr.end() - 1);
        for (int e = 0; e < E; e++) {
            const int oi = o.opt[e_pose[e]];
            const int k = fp[e_pt[e]]++;
            o.pt_edges[k] = e;
            eopt[k] = oi;
            if (oi >= 0) o.ps_edges[fq[oi]++] = e;
        }
    }
    // row lists: the pt_edges slots of each pose row, in landmark order
    std::vector<int> rk(o.ps_ptr[np]);
    {
        std::vector<int> fq(o.ps_ptr.begin(), o.ps_ptr.end() - 1);
        for (int m = 0; m < M; m++)
            for (int k = o.pt_ptr[m]; k < o.pt_ptr[m + 1]; k++) {
                epm[k] = m;
                if (eopt[k] >= 0) rk[fq[eopt[k]]++] = k;
            }
    }
    t[0] += now() - t0; t0 = now();
    std::vector<int> rblk(np + 1, 0), rpair(np + 1, 0);
    auto row_counts = [&](int ia, int* c) {   // c[j] = pairs of block (ia, j); returns blocks
        for (int r = o.ps_ptr[ia]; r < o.ps_ptr[ia + 1]; r++) {
            const int m = epm[rk[r]];
            for (int kb = o.pt_ptr[m]; kb < o.pt_ptr[m + 1]; kb++)
                if (eopt[kb] >= ia) c[eopt[kb]]++;
        }
    };
    {
        std::vector<int> c(np, 0);
        for (int ia = 0; ia < np; ia++) {
            row_counts(ia, c.data());
            int nb = 0, npr = 0;
            for (int j = ia; j < np; j++) {
                nb += (j == ia || c[j] > 0);
                npr += c[j];
                c[j] = 0;
            }
            rblk[ia + 1] = nb;
            rpair[ia + 1] = npr;
        }
    }
    for (int i = 0; i < np; i++) { rblk[i + 1] += rblk[i]; rpair[i + 1] += rpair[i]; }
    t[1] += now() - t0; t0 = now();
    const int nblk = rblk[np];
    o.blk_i.resize(nblk);
    o.blk_j.resize(nblk);
    o.blk_ptr.resize(nblk + 1);
    o.blk_ptr[nblk] = rpair[np];
    o.blk_pairs.resize(2 * (size_t)rpair[np]);
    {
        std::vector<int> c(np, 0);
        for (int ia = 0; ia < np; ia++) {
            row_counts(ia, c.data());
            int b = rblk[ia], s = rpair[ia];
            for (int j = ia; j < np; j++)
                if (j == ia || c[j] > 0) {
                    o.blk_i[b] = ia; o.blk_j[b] = j; o.blk_ptr[b] = s;
                    b++;
                    const int n = c[j];
                    c[j] = s;   // the column's cursor
                    s += n;
                }
            for (int r = o.ps_ptr[ia]; r < o.ps_ptr[ia + 1]; r++) {
                const int ka = rk[r], ea = o.pt_edges[ka], m = epm[ka];
                for (int kb = o.pt_ptr[m]; kb < o.pt_ptr[m + 1]; kb++) {
                    const int ib = eopt[kb];
                    if (ib < ia) continue;
                    const int slot = c[ib]++;
                    o.blk_pairs[2 * (size_t)slot] = ea;
                    o.blk_pairs[2 * (size_t)slot + 1] = o.pt_edges[kb];
                }
            }
            for (int j = ia; j < np; j++) c[j] = 0;
        }
    }
    t[3] += now() - t0;
}

// serial2: the serial order with one load per pair endpoint (eopt: each pt_edges slot's opt
// index, filled with the CSR) and the dense count array turned into the blocks' fill cursors
// (no block-id array); scratch vectors kept across calls (as a workspace would)
static void serial2(int P, int M, int E, const int* e_pose, const int* e_pt, const unsigned char* fixed, Out& o, double* t) {
    double t0 = now();
    static std::vector<int> eopt, cnt, fp;
    o.opt.assign(P, -1);
    int np = 0;
    for (int i = 0; i < P; i++)
        if (!fixed[i]) o.opt[i] = np++;
    o.np = np;
    o.pt_ptr.assign(M + 1, 0);
    o.ps_ptr.assign(np + 1, 0);
    for (int e = 0; e < E; e++) {
        o.pt_ptr[e_pt[e] + 1]++;
        if (o.opt[e_pose[e]] >= 0) o.ps_ptr[o.opt[e_pose[e]] + 1]++;
    }
    for (int m = 0; m < M; m++) o.pt_ptr[m + 1] += o.pt_ptr[m];
    for (int i = 0; i < np; i++) o.ps_ptr[i + 1] += o.ps_ptr[i];
    o.pt_edges.resize(E);
    o.ps_edges.resize(o.ps_ptr[np]);
    eopt.resize(E);
    {
        fp.assign(o.pt_ptr.begin(), o.pt_ptr.end() - 1);
        std::vector<int> fq(o.ps_ptr.begin(), o.ps_ptr.end() - 1);
        for (int e = 0; e < E; e++) {
            const int oi = o.opt[e_pose[e]];
            const int k = fp[e_pt[e]]++;
            o.pt_edges[k] = e;
            eopt[k] = oi;
            if (oi >= 0) o.ps_edges[fq[oi]++] = e;
        }
    }
    t[0] += now() - t0; t0 = now();
    cnt.assign((size_t)np * np, 0);
    size_t npairs = 0;
    for (int m = 0; m < M; m++) {
        const int k0 = o.pt_ptr[m], k1 = o.pt_ptr[m + 1];
        for (int ka = k0; ka < k1; ka++) {
            const int ia = eopt[ka];
            if (ia < 0) continue;
            int* row = cnt.data() + (size_t)ia * np;
            for (int kb = k0; kb < k1; kb++) {
                const int ib = eopt[kb];
                if (ib < ia) continue;
                row[ib]++;
                npairs++;
            }
        }
    }
    t[1] += now() - t0; t0 = now();
    o.blk_ptr.assign(1, 0);
    int s = 0;
    for (int i = 0; i < np; i++) {
        int* row = cnt.data() + (size_t)i * np;
        for (int j = i; j < np; j++) {
            const int c = row[j];
            if (i == j || c > 0) {
                o.blk_i.push_back(i);
                o.blk_j.push_back(j);
                row[j] = s;   // the block's fill cursor
                s += c;
                o.blk_ptr.push_back(s);
            }
        }
    }
    t[2] += now() - t0; t0 = now();
    o.blk_pairs.resize(2 * npairs);
    int* bp = o.blk_pairs.data();
    for (int m = 0; m < M; m++) {
        const int k0 = o.pt_ptr[m], k1 = o.pt_ptr[m + 1];
        for (int ka = k0; ka < k1; ka++) {
            const int ia = eopt[ka];
            if (ia < 0) continue;
            const int ea = o.pt_edges[ka];
            int* row = cnt.data() + (size_t)ia * np;
            for (int kb = k0; kb < k1; kb++) {
                const int ib = eopt[kb];
                if (ib < ia) continue;
                const int slot = row[ib]++;
                bp[2 * slot] = ea;
                bp[2 * slot + 1] = o.pt_edges[kb];
            }
        }
    }
    t[3] += now() - t0;
}

// serial3: serial2 with the two pair passes split over T contiguous landmark ranges (T count
// arrays; a block's pairs from range t follow those of ranges < t, so the lists stay identical)
static void serial3(int P, int M, int E, const int* e_pose, const int* e_pt, const unsigned char* fixed, Out& o, double* t,
                    int T) {
    double t0 = now();
    static std::vector<int> eopt;
    static std::vector<std::vector<int>> cnts;
    o.opt.assign(P, -1);
    int np = 0;
    for (int i = 0; i < P; i++)
        if (!fixed[i]) o.opt[i] = np++;
    o.np = np;
    o.pt_ptr.assign(M + 1, 0);
    o.ps_ptr.assign(np + 1, 0);
    for (int e = 0; e < E; e++) {
        o.pt_ptr[e_pt[e] + 1]++;
        if (o.opt[e_pose[e]] >= 0) o.ps_ptr[o.opt[e_pose[e]] + 1]++;
    }
    for (int m = 0; m < M; m++) o.pt_ptr[m + 1] += o.pt_ptr[m];
    for (int i = 0; i < np; i++) o.ps_ptr[i + 1] += o.ps_ptr[i];
    o.pt_edges.resize(E);
    o.ps_edges.resize(o.ps_ptr[np]);
    eopt.resize(E);
    {
        std::vector<int> fp(o.pt_ptr.begin(), o.pt_ptr.end() - 1), fq(o.ps_ptr.begin(), o.ps_ptr.end() - 1);
        for (int e = 0; e < E; e++) {
            const int oi = o.opt[e_pose[e]];
            const int k = fp[e_pt[e]]++;
            o.pt_edges[k] = e;
            eopt[k] = oi;
            if (oi >= 0) o.ps_edges[fq[oi]++] = e;
        }
    }
    t[0] += now() - t0; t0 = now();
    if ((int)cnts.size() < T) cnts.resize(T);
    std::vector<size_t> npr(T, 0);
    auto range = [&](int q) { return std::make_pair((int)((long long)M * q / T), (int)((long long)M * (q + 1) / T)); };
    auto count = [&](int q) {
        std::vector<int>& cnt = cnts[q];
        cnt.assign((size_t)np * np, 0);
        size_t n = 0;
        const auto [m0, m1] = range(q);
        for (int m = m0; m < m1; m++) {
            const int k0 = o.pt_ptr[m], k1 = o.pt_ptr[m + 1];
            for (int ka = k0; ka < k1; ka++) {
                const int ia = eopt[ka];
                if (ia < 0) continue;
                int* row = cnt.data() + (size_t)ia * np;
                for (int kb = k0; kb < k1; kb++) {
                    const int ib = eopt[kb];
                    if (ib < ia) continue;
                    row[ib]++;
                    n++;
                }
            }
        }
        npr[q] = n;
    };
    {
        std::vector<std::thread> th;
        for (int q = 1; q < T; q++) th.emplace_back(count, q);
        count(0);
        for (auto& x : th) x.join();
    }
    size_t npairs = 0;
    for (int q = 0; q < T; q++) npairs += npr[q];
    t[1] += now() - t0; t0 = now();
    o.blk_ptr.assign(1, 0);
    int s = 0;
    for (int i = 0; i < np; i++) {
        for (int j = i; j < np; j++) {
            const size_t k = (size_t)i * np + j;
            int c = 0;
            for (int q = 0; q < T; q++) c += cnts[q][k];
            if (i == j || c > 0) {
                o.blk_i.push_back(i);
                o.blk_j.push_back(j);
                for (int q = 0; q < T; q++) { const int v = cnts[q][k]; cnts[q][k] = s; s += v; }
                o.blk_ptr.push_back(s);
            }
        }
    }
    t[2] += now() - t0; t0 = now();
    o.blk_pairs.resize(2 * npairs);
    int* bp = o.blk_pairs.data();
    auto fill = [&](int q) {
        std::vector<int>& cur = cnts[q];
        const auto [m0, m1] = range(q);
        for (int m = m0; m < m1; m++) {
            const int k0 = o.pt_ptr[m], k1 = o.pt_ptr[m + 1];
            for (int ka = k0; ka < k1; ka++) {
                const int ia = eopt[ka];
                if (ia < 0) continue;
                const int ea = o.pt_edges[ka];
                int* row = cur.data() + (size_t)ia * np;
                for (int kb = k0; kb < k1; kb++) {
                    const int ib = eopt[kb];
                    if (ib < ia) continue;
                    const int slot = row[ib]++;
                    bp[2 * (size_t)slot] = ea;
                    bp[2 * (size_t)slot + 1] = o.pt_edges[kb];
                }
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (int q = 1; q < T; q++) th.emplace_back(fill, q);
        fill(0);
        for (auto& x : th) x.join();
    }
    t[3] += now() - t0;
}

int main(int argc, char** argv) {
    if (argc < 4) return 1;
    auto a = slurp(argv[1]), b = slurp(argv[2]), c = slurp(argv[3]);
    const int E = (int)(a.size() / 4), P = (int)c.size();
    const int* ep = (const int*)a.data();
    const int* et = (const int*)b.data();
    int M = 0;
    for (int e = 0; e < E; e++) M = std::max(M, et[e] + 1);
    const int nth = argc > 4 ? std::atoi(argv[4]) : 8;
    Out o1, o2;
    double ts[4] = {0}, tt[4] = {0};
    const int R = 20;
    for (int r = 0; r < R; r++) { o1 = Out(); serial(P, M, E, ep, et, (const unsigned char*)c.data(), o1, ts); }
    for (int r = 0; r < R; r++) { o2 = Out(); rowwise(P, M, E, ep, et, (const unsigned char*)c.data(), o2, tt, nth); }
    Out o3;
    double t3[4] = {0};
    for (int r = 0; r < R; r++) { o3.blk_i.clear(); o3.blk_j.clear(); serial2(P, M, E, ep, et, (const unsigned char*)c.data(), o3, t3); }
    const bool same3 = o1.blk_i == o3.blk_i && o1.blk_j == o3.blk_j && o1.blk_ptr == o3.blk_ptr && o1.blk_pairs == o3.blk_pairs && o1.pt_edges == o3.pt_edges && o1.ps_edges == o3.ps_edges;
    for (int T : {2, 4}) {
        Out o4;
        double t4[4] = {0};
        for (int r = 0; r < R; r++) { o4.blk_i.clear(); o4.blk_j.clear(); serial3(P, M, E, ep, et, (const unsigned char*)c.data(), o4, t4, T); }
        const bool same4 = o1.blk_i == o4.blk_i && o1.blk_j == o4.blk_j && o1.blk_ptr == o4.blk_ptr && o1.blk_pairs == o4.blk_pairs;
        std::printf("serial3 T=%d ms: csr %.3f count %.3f blocks %.3f fill %.3f total %.3f identical=%d\n", T, t4[0] / R, t4[1] / R, t4[2] / R, t4[3] / R, (t4[0] + t4[1] + t4[2] + t4[3]) / R, same4);
    }
    std::printf("serial2  ms: csr %.3f count %.3f blocks %.3f fill %.3f total %.3f identical=%d\n", t3[0] / R, t3[1] / R, t3[2] / R, t3[3] / R, (t3[0] + t3[1] + t3[2] + t3[3]) / R, same3);
    const bool same = o1.blk_i == o2.blk_i && o1.blk_j == o2.blk_j && o1.blk_ptr == o2.blk_ptr &&
                      o1.blk_pairs == o2.blk_pairs && o1.pt_edges == o2.pt_edges && o1.ps_edges == o2.ps_edges;
    std::printf("P=%d M=%d E=%d blocks=%zu pairs=%zu identical=%d\n", P, M, E, o1.blk_i.size(), o1.blk_pairs.size() / 2, same);
    std::printf("serial   ms: csr %.3f count %.3f blocks %.3f fill %.3f total %.3f\n", ts[0] / R, ts[1] / R, ts[2] / R,
                ts[3] / R, (ts[0] + ts[1] + ts[2] + ts[3]) / R);
    std::printf("rowwise  ms: csr %.3f count %.3f - %.3f blocks+fill %.3f total %.3f (%d threads)\n", tt[0] / R,
                tt[1] / R, tt[2] / R, tt[3] / R, (tt[0] + tt[1] + tt[2] + tt[3]) / R, nth);
    return same ? 0 : 2;
}
