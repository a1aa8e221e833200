// ORACLE — test infrastructure only (see orb_oracle.h).
// DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB>::transform(features, BowVector&,
// FeatureVector&, levelsup) restated sequentially with the reference's containers:
//   transform (batch)        Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1194
//   transform (one feature)  :1217-1259  descent, F::distance, `if (d < best_d)` (first wins)
//   BowVector::addWeight / addIfNotExist / normalize   Thirdparty/DBoW2/DBoW2/BowVector.cpp:34-86
//   FeatureVector::addFeature                         Thirdparty/DBoW2/DBoW2/FeatureVector.cpp:31-45
//   FORB::distance           Thirdparty/DBoW2/DBoW2/FORB.cpp:81-101 (popcount of the XOR)
//   ScoringObject::mustNormalize                      Thirdparty/DBoW2/DBoW2/ScoringObject.h:60-92
// Deviation (documented): a leaf reached above level L - levelsup leaves the
// reference's node id unassigned (uninitialised NodeId in the caller); here it is the root, 0.
#include <cmath>
#include <cstdint>
#include <map>
#include <vector>

#include "../include/orbmi.h"

namespace {

int forb_distance(const uint8_t* a, const uint8_t* b) {
    // FORB::distance: 8 x 32-bit SWAR popcounts of a ^ b (same value as the plain popcount)
    int dist = 0;
    for (int i = 0; i < 32; i++) dist += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return dist;
}

}  // namespace

extern "C" int orc_transform(const orbmi_vocabulary_desc* V, const uint8_t* desc, int n, int levelsup,
                             uint32_t* bow_word, double* bow_value, uint32_t* fv_node, int32_t* fv_off,
                             int32_t* fv_feat, int* counts) {
    std::map<uint32_t, double> v;                  // BowVector
    std::map<uint32_t, std::vector<int>> fv;       // FeatureVector
    bool has_word = false;
    for (int i = 0; i < V->nnodes; i++) has_word |= V->word_id[i] >= 0;
    if (has_word) {  // if(empty()) return;
        int norm_type = 1;  // mustNormalize: L2 for L2_NORM, L1 otherwise; DOT_PRODUCT: none
        const bool must = V->scoring != 5;
        if (V->scoring == 1) norm_type = 2;
        const int nid_level = V->L - levelsup;
        const bool tf = V->weighting == 0 || V->weighting == 1;  // TF_IDF || TF
        for (int f = 0; f < n; f++) {
            const uint8_t* feat = desc + 32 * (size_t)f;
            int final_id = 0, current_level = 0;
            uint32_t nid = 0;  // nid_level <= 0: root (and the documented deviation above)
            do {
                ++current_level;
                const int c0 = V->child_off[final_id], c1 = V->child_off[final_id + 1];
                final_id = V->children[c0];
                double best_d = forb_distance(feat, V->desc + 32 * (size_t)final_id);
                for (int j = c0 + 1; j < c1; j++) {
                    const int id = V->children[j];
                    const double d = forb_distance(feat, V->desc + 32 * (size_t)id);
                    if (d < best_d) {
                        best_d = d;
                        final_id = id;
                    }
                }
                if (current_level == nid_level) nid = (uint32_t)final_id;
            } while (V->child_off[final_id] != V->child_off[final_id + 1]);  // !isLeaf()
            const uint32_t word = (uint32_t)V->word_id[final_id];
            const double w = V->weight[final_id];
            if (w > 0) {
                if (tf) {
                    auto it = v.lower_bound(word);
                    if (it != v.end() && it->first == word) it->second += w;
                    else v.insert(it, {word, w});
                } else {
                    if (!v.count(word)) v[word] = w;
                }
                fv[nid].push_back(f);
            }
        }
        if (tf && !v.empty() && !must) {
            const double nd = (double)v.size();
            for (auto& kv : v) kv.second /= nd;
        }
        if (must) {  // BowVector::normalize
            double norm = 0.0;
            if (norm_type == 1) {
                for (auto& kv : v) norm += fabs(kv.second);
            } else {
                for (auto& kv : v) norm += kv.second * kv.second;
                norm = sqrt(norm);
            }
            if (norm > 0.0)
                for (auto& kv : v) kv.second /= norm;
        }
    }
    int k = 0;
    for (auto& kv : v) { bow_word[k] = kv.first; bow_value[k] = kv.second; k++; }
    counts[0] = k;
    k = 0;
    int pos = 0;
    for (auto& kv : fv) {
        fv_node[k] = kv.first;
        fv_off[k] = pos;
        for (int f : kv.second) fv_feat[pos++] = f;
        k++;
    }
    fv_off[k] = pos;
    counts[1] = k;
    return 0;
}
