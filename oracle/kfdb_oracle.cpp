// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see orb_oracle.cpp header for the rules).
//
// CPU restatement of the place-recognition queries, recalled from
// upstream (the ORB_SLAM3 submodule is empty here):
//   U:src/KeyFrameDatabase.cc::add(pKF) / erase(pKF) — mvInvertedFile[word] is a list of
//       KeyFrames in insertion order; erase removes the KF from the lists of its words.
//   U:src/KeyFrameDatabase.cc::DetectRelocalizationCandidates(Frame* F, Map* pMap)
//       1. KFs sharing a word, first-encounter order (query words ascending, list order);
//          mnRelocWords reset on first encounter (mnRelocQuery != F->mnId), then counted.
//       2. minCommonWords = (int)(maxCommonWords * 0.8f); KFs with mnRelocWords > min get
//          mRelocScore = (float)mpVoc->score(F->mBowVec, pKFi->mBowVec) (DBoW2 L1Scoring:
//          sum over common words ascending of |vi - vj| - |vi| - |vj| in double, then -s/2).
//       3. accScore over GetBestCovisibilityKeyFrames(10) with mnRelocQuery == F->mnId (their
//          mRelocScore, possibly from an earlier query when not scored now: upstream keeps it),
//          pBestKF = max mRelocScore (strict >).
//       4. keep accScore > 0.75f * bestAccScore, same map, first occurrence of pBestKF.
//   U:src/KeyFrameDatabase.cc::DetectNBestCandidates(pKF, vpLoopCand, vpMergeCand, n)
//       the same with mnPlaceRecognition* members, connected KFs of pKF excluded from the list
//       (their word count is reset but they are never queued), then lAccScoreAndMatch sorted
//       by accScore descending (std::list::sort: stable), walked until both lists hold n:
//       same map -> loop candidate, other (not bad) map -> merge candidate, first occurrence of
//       pBestKF only. A bad pBestKF is skipped (upstream's `continue` there never advances the
//       iterator; the restatement advances).
// PARITY UNPINNED by the reference (no fixtures upstream).
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <list>
#include <set>
#include <vector>

namespace {

struct KF {
    bool active = false;
    std::vector<int32_t> words;
    std::vector<double> values;
    long long reloc_query = -1, pr_query = -1;
    int reloc_words = 0, pr_words = 0;
    float reloc_score = 0.f, pr_score = 0.f;
};

struct DB {
    std::vector<KF> kf;
    std::vector<std::list<int>> inv;   // word -> KFs in insertion order
};

double l1_score(const int32_t* w1, const double* v1, int n1, const int32_t* w2, const double* v2, int n2) {
    // DBoW2 L1Scoring::score; BowVector = std::map<WordId, WordValue> (ascending ids)
    double score = 0;
    int i = 0, j = 0;
    while (i < n1 && j < n2) {
        const double vi = v1[i], vj = v2[j];
        if (w1[i] == w2[j]) {
            score += std::fabs(vi - vj) - std::fabs(vi) - std::fabs(vj);
            ++i; ++j;
        } else if (w1[i] < w2[j]) {
            i = (int)(std::lower_bound(w1 + i, w1 + n1, w2[j]) - w1);   // v1.lower_bound(v2_it->first)
        } else {
            j = (int)(std::lower_bound(w2 + j, w2 + n2, w1[i]) - w2);
        }
    }
    return -score / 2.0;
}

}  // namespace

extern "C" {

void* orc_kfdb_create(int max_kf, int n_words) {
    DB* d = new DB();
    d->kf.resize(max_kf);
    d->inv.resize(n_words);
    return d;
}
void orc_kfdb_destroy(void* h) { delete (DB*)h; }

void orc_kfdb_add(void* h, int kf, const int32_t* words, const double* values, int n) {
    DB* d = (DB*)h;
    KF& k = d->kf[kf];
    k.active = true;
    k.words.assign(words, words + n);
    k.values.assign(values, values + n);
    for (int i = 0; i < n; i++) d->inv[words[i]].push_back(kf);
}

void orc_kfdb_erase(void* h, int kf) {
    DB* d = (DB*)h;
    KF& k = d->kf[kf];
    for (int32_t w : k.words) d->inv[w].remove(kf);
    k.active = false;
}

// covis: n_slots x 10 (GetBestCovisibilityKeyFrames(10), -1 padded); kf_map: map id per slot.
int orc_kfdb_detect_relocalization(void* h, long long qid, const int32_t* words, const double* values, int n,
                                   const int32_t* covis, const int32_t* kf_map, int query_map, int32_t* out) {
    DB* d = (DB*)h;
    std::list<int> shared;
    for (int i = 0; i < n; i++)
        for (int kf : d->inv[words[i]]) {
            KF& k = d->kf[kf];
            if (k.reloc_query != qid) { k.reloc_words = 0; k.reloc_query = qid; shared.push_back(kf); }
            k.reloc_words++;
        }
    if (shared.empty()) return 0;
    int maxCommon = 0;
    for (int kf : shared) maxCommon = std::max(maxCommon, d->kf[kf].reloc_words);
    const int minCommon = (int)(maxCommon * 0.8f);
    std::list<std::pair<float, int>> scored;
    for (int kf : shared) {
        KF& k = d->kf[kf];
        if (k.reloc_words > minCommon) {
            const float si = (float)l1_score(words, values, n, k.words.data(), k.values.data(), (int)k.words.size());
            k.reloc_score = si;
            scored.push_back({si, kf});
        }
    }
    if (scored.empty()) return 0;
    std::list<std::pair<float, int>> acc;
    float bestAcc = 0;
    for (auto& sm : scored) {
        float best = sm.first, a = best;
        int pBest = sm.second;
        for (int t = 0; t < 10; t++) {
            const int nb = covis[10 * sm.second + t];
            if (nb < 0) break;
            const KF& k2 = d->kf[nb];
            if (k2.reloc_query != qid) continue;
            a += k2.reloc_score;
            if (k2.reloc_score > best) { pBest = nb; best = k2.reloc_score; }
        }
        acc.push_back({a, pBest});
        if (a > bestAcc) bestAcc = a;
    }
    const float minRetain = 0.75f * bestAcc;
    std::set<int> added;
    int m = 0;
    for (auto& am : acc) {
        if (am.first > minRetain) {
            if (kf_map && kf_map[am.second] != query_map) continue;
            if (!added.count(am.second)) { out[m++] = am.second; added.insert(am.second); }
        }
    }
    return m;
}

// connected: per slot, 1 = in pKF->GetConnectedKeyFrames(); flags: bit0 bad KF, bit1 bad map.
void orc_kfdb_detect_nbest(void* h, long long qid, const int32_t* words, const double* values, int n,
                           const int32_t* covis, const uint8_t* connected, const int32_t* kf_map, int query_map,
                           const uint8_t* flags, int ncand, int32_t* loop_out, int32_t* n_loop, int32_t* merge_out,
                           int32_t* n_merge) {
    DB* d = (DB*)h;
    *n_loop = 0; *n_merge = 0;
    std::list<int> shared;
    for (int i = 0; i < n; i++)
        for (int kf : d->inv[words[i]]) {
            KF& k = d->kf[kf];
            if (k.pr_query != qid) {
                k.pr_words = 0;
                if (!(connected && connected[kf])) { k.pr_query = qid; shared.push_back(kf); }
            }
            k.pr_words++;
        }
    if (shared.empty()) return;
    int maxCommon = 0;
    for (int kf : shared) maxCommon = std::max(maxCommon, d->kf[kf].pr_words);
    const int minCommon = (int)(maxCommon * 0.8f);
    std::list<std::pair<float, int>> scored;
    for (int kf : shared) {
        KF& k = d->kf[kf];
        if (k.pr_words > minCommon) {
            const float si = (float)l1_score(words, values, n, k.words.data(), k.values.data(), (int)k.words.size());
            k.pr_score = si;
            scored.push_back({si, kf});
        }
    }
    if (scored.empty()) return;
    std::list<std::pair<float, int>> acc;
    for (auto& sm : scored) {
        float best = sm.first, a = best;
        int pBest = sm.second;
        for (int t = 0; t < 10; t++) {
            const int nb = covis[10 * sm.second + t];
            if (nb < 0) break;
            const KF& k2 = d->kf[nb];
            if (k2.pr_query != qid) continue;
            a += k2.pr_score;
            if (k2.pr_score > best) { pBest = nb; best = k2.pr_score; }
        }
        acc.push_back({a, pBest});
    }
    acc.sort([](const std::pair<float, int>& x, const std::pair<float, int>& y) { return x.first > y.first; });
    std::set<int> added;
    for (auto& am : acc) {
        if (*n_loop >= ncand && *n_merge >= ncand) break;
        const int kfi = am.second;
        if (flags && (flags[kfi] & 1)) continue;
        if (!added.count(kfi)) {
            const bool same = !kf_map || kf_map[kfi] == query_map;
            if (same && *n_loop < ncand) loop_out[(*n_loop)++] = kfi;
            else if (!same && *n_merge < ncand && !(flags && (flags[kfi] & 2))) merge_out[(*n_merge)++] = kfi;
            added.insert(kfi);
        }
    }
}

}  // extern "C"
