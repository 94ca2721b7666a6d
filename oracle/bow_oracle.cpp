// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see orb_oracle.cpp header for the rules).
//
// CPU restatement of the bag-of-words path:
//   Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h (vendored in the fork; absent here):
//     transform(feature, WordId&, WordValue&, NodeId*, levelsup) — descend from the root; at
//       each level the child with the smallest FORB::distance wins (strict <: first child on
//       ties); the node reached at level L - levelsup is the FeatureVector node (root if that
//       level is <= 0); the leaf gives word id + weight.
//     transform(features, BowVector&, FeatureVector&, levelsup) — TF_IDF weighting: features
//       with weight > 0 add their weight to their word and their index to their node; L1_NORM
//       scoring normalises the BowVector (mustNormalize), so no division by the word count.
//     loadFromTextFile — node i (i >= 1) is line i of the file; the root is node 0; children in
//       file order; word ids in order of leaf appearance.
//   U:src/ORBmatcher.cc::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) — walk both
//     FeatureVectors (std::map, ascending node id); for every shared node, every KF feature with
//     a valid map point (in index order) takes the nearest frame feature of the node that is not
//     matched yet (best/second, strict <); accept best <= TH_LOW and best < ratio * second; then
//     the rotation histogram (HISTO_LENGTH 30, ComputeThreeMaxima) drops matches outside the
//     three main bins. Monocular only (no right-camera branch).
// PARITY UNPINNED by the reference (submodule empty, DBoW2 absent, ORBvoc.txt gitignored):
// pinned by tests/test_bow.py KATs on hand-built vocabularies.
// ============================================================================
#include <cmath>
#include <cstdint>
#include <map>
#include <vector>

namespace {

inline int hamming32(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

struct Vocab {
    int L;
    const uint8_t* desc;        // n_nodes x 32 (row 0 = root, unused)
    const int32_t* first_child; // CSR into children
    const int32_t* n_child;
    const int32_t* children;
    const int32_t* word_id;     // -1 for internal nodes
    const double* weight;
};

void transform1(const Vocab& V, const uint8_t* f, int levelsup, int32_t& word, double& w, int32_t& nid) {
    const int nid_level = V.L - levelsup;
    if (nid_level <= 0) nid = 0;
    int final_id = 0, level = 0;
    do {
        ++level;
        const int32_t* ch = V.children + V.first_child[final_id];
        const int nc = V.n_child[final_id];
        final_id = ch[0];
        int best = hamming32(f, V.desc + 32 * (size_t)final_id);
        for (int c = 1; c < nc; c++) {
            const int d = hamming32(f, V.desc + 32 * (size_t)ch[c]);
            if (d < best) { best = d; final_id = ch[c]; }
        }
        if (level == nid_level) nid = final_id;
    } while (V.n_child[final_id] > 0);
    word = V.word_id[final_id];
    w = V.weight[final_id];
}

}  // namespace

extern "C" {

// per-feature transform: word id, weight, FeatureVector node (levelsup)
void orc_bow_transform(const uint8_t* desc, const int32_t* first_child, const int32_t* n_child,
                       const int32_t* children, const int32_t* word_id, const double* weight, int L,
                       const uint8_t* feat, int n, int levelsup, int32_t* out_word, int32_t* out_node,
                       double* out_weight) {
    Vocab V{L, desc, first_child, n_child, children, word_id, weight};
    for (int i = 0; i < n; i++) {
        int32_t nid = 0;
        transform1(V, feat + 32 * (size_t)i, levelsup, out_word[i], out_weight[i], nid);
        out_node[i] = nid;
    }
}

// BowVector from per-feature (word, weight): TF_IDF + L1_NORM. Writes the sorted words and their
// normalised values; returns the number of words.
int orc_bow_vector(const int32_t* word, const double* weight, int n, int32_t* out_words, double* out_values) {
    std::map<int32_t, double> v;
    for (int i = 0; i < n; i++)
        if (weight[i] > 0) v[word[i]] += weight[i];
    double norm = 0;
    for (auto& kv : v) norm += std::fabs(kv.second);
    int k = 0;
    for (auto& kv : v) {
        out_words[k] = kv.first;
        out_values[k] = norm > 0 ? kv.second / norm : kv.second;
        k++;
    }
    return k;
}

// SearchByBoW(KeyFrame, Frame): match[f] = KF feature index matched to frame feature f, or -1.
// node < 0 marks a feature outside the FeatureVector (weight 0). kf_valid: the KF feature has a
// good map point. Returns nmatches after the rotation filter.
int orc_search_bow(const uint8_t* kf_desc, const float* kf_angle, const int32_t* kf_node, const uint8_t* kf_valid,
                   int nkf, const uint8_t* f_desc, const float* f_angle, const int32_t* f_node, int nf,
                   float ratio, int check_orientation, int th_low, int32_t* match) {
    std::map<int32_t, std::vector<int>> fvk, fvf;   // FeatureVector: node -> feature indices
    for (int i = 0; i < nkf; i++)
        if (kf_node[i] >= 0) fvk[kf_node[i]].push_back(i);
    for (int i = 0; i < nf; i++)
        if (f_node[i] >= 0) fvf[f_node[i]].push_back(i);
    for (int i = 0; i < nf; i++) match[i] = -1;
    const int HISTO_LENGTH = 30;
    std::vector<int> rotHist[30];
    const float factor = 1.0f / HISTO_LENGTH;
    int nmatches = 0;
    auto KFit = fvk.begin(), Fit = fvf.begin();
    while (KFit != fvk.end() && Fit != fvf.end()) {
        if (KFit->first == Fit->first) {
            for (int realIdxKF : KFit->second) {
                if (!kf_valid[realIdxKF]) continue;
                const uint8_t* dKF = kf_desc + 32 * (size_t)realIdxKF;
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                for (int realIdxF : Fit->second) {
                    if (match[realIdxF] >= 0) continue;
                    const int dist = hamming32(dKF, f_desc + 32 * (size_t)realIdxF);
                    if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdxF = realIdxF; }
                    else if (dist < bestDist2) bestDist2 = dist;
                }
                if (bestDist1 <= th_low) {
                    if ((float)bestDist1 < ratio * (float)bestDist2) {
                        match[bestIdxF] = realIdxKF;
                        if (check_orientation) {
                            float rot = kf_angle[realIdxKF] - f_angle[bestIdxF];
                            if (rot < 0.0) rot += 360.0f;
                            int bin = (int)std::round(rot * factor);
                            if (bin == HISTO_LENGTH) bin = 0;
                            rotHist[bin].push_back(bestIdxF);
                        }
                        nmatches++;
                    }
                }
            }
            ++KFit;
            ++Fit;
        } else if (KFit->first < Fit->first) {
            KFit = fvk.lower_bound(Fit->first);
        } else {
            Fit = fvf.lower_bound(KFit->first);
        }
    }
    if (check_orientation) {
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < HISTO_LENGTH; i++) {
            const int s = (int)rotHist[i].size();
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j : rotHist[i]) { match[j] = -1; nmatches--; }
        }
    }
    return nmatches;
}

}  // extern "C"
