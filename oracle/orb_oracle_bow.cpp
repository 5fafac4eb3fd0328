// ============================================================================================
// orb_oracle_bow.cpp — CPU ORACLE of DBoW2's TemplatedVocabulary<FORB> (test infrastructure
// only; see orb_oracle.cpp's header for the rules and the parity status). Literal restatement of
//   TemplatedVocabulary::loadFromBinFile   Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1478-1540
//   TemplatedVocabulary::transform (v, fv)  :1139-1198 and the per-feature descent :1218-1262
//   BowVector::addWeight / addIfNotExist / normalize   BowVector.cpp
//   FeatureVector::addFeature                           FeatureVector.cpp
//   ScoringObject mustNormalize table                   ScoringObject.h:74-89
// with std::map containers in the reference's insertion order. FORB::distance = Hamming.
// ============================================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

namespace oracle {
int hamming(const uint8_t* a, const uint8_t* b);
}

namespace {

struct Node {
    int id = 0, parent = 0, word_id = 0;
    double weight = 0;
    std::vector<int> children;
    uint8_t desc[32] = {0};
    bool isLeaf() const { return children.empty(); }
};

struct Vocab {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    std::vector<Node> nodes;
    std::vector<int> words;   // word id -> node id
};

void add_node(Vocab& v, int pid, int is_leaf, const uint8_t* d, double w) {
    const int nid = (int)v.nodes.size();
    v.nodes.resize(v.nodes.size() + 1);
    v.nodes[nid].id = nid;
    v.nodes[nid].parent = pid;
    v.nodes[pid].children.push_back(nid);
    memcpy(v.nodes[nid].desc, d, 32);
    v.nodes[nid].weight = w;
    if (is_leaf > 0) {
        v.nodes[nid].word_id = (int)v.words.size();
        v.words.push_back(nid);
    }
}

// TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)
void transform1(const Vocab& v, const uint8_t* f, int& word_id, double& weight, int* nid, int levelsup) {
    const int nid_level = v.L - levelsup;
    if (nid_level <= 0 && nid != nullptr) *nid = 0;
    int final_id = 0, current_level = 0;
    do {
        ++current_level;
        const std::vector<int>& nodes = v.nodes[final_id].children;
        final_id = nodes[0];
        double best_d = oracle::hamming(f, v.nodes[final_id].desc);
        for (size_t j = 1; j < nodes.size(); j++) {
            const int id = nodes[j];
            const double d = oracle::hamming(f, v.nodes[id].desc);
            if (d < best_d) { best_d = d; final_id = id; }
        }
        if (nid != nullptr && current_level == nid_level) *nid = final_id;
    } while (!v.nodes[final_id].isLeaf());
    word_id = v.nodes[final_id].word_id;
    weight = v.nodes[final_id].weight;
}

}  // namespace

extern "C" {

void* oro_voc_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t* parents,
                     const uint8_t* is_leaf, const uint8_t* desc, const double* weights) {
    Vocab* v = new Vocab();
    v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting;
    v->nodes.resize(1);
    for (int i = 1; i < n_nodes; i++) add_node(*v, parents[i], is_leaf[i], desc + 32 * (size_t)i, weights[i]);
    return v;
}

// loadFromBinFile on an in-memory file (returns null where the reference returns false)
void* oro_voc_load_bin(const uint8_t* data, size_t size) {
    if (size < 16) return nullptr;
    int hdr[4];
    memcpy(hdr, data, 16);
    Vocab* v = new Vocab();
    v->k = hdr[0]; v->L = hdr[1];
    if (v->k < 0 || v->k > 20 || v->L < 1 || v->L > 10 || hdr[2] < 0 || hdr[2] > 5 || hdr[3] < 0 || hdr[3] > 3) {
        delete v;
        return nullptr;
    }
    v->scoring = hdr[2];
    v->weighting = hdr[3];
    const int expected = (int)((pow((double)v->k, (double)v->L + 1) - 1) / (v->k - 1));
    v->nodes.resize(1);
    size_t pos = 16;
    while (pos < size && v->nodes.size() < (unsigned)expected) {
        if (pos + 45 > size) { delete v; return nullptr; }
        int pid;
        memcpy(&pid, data + pos, 4);
        double w;
        memcpy(&w, data + pos + 37, 8);
        add_node(*v, pid, data[pos + 4], data + pos + 5, w);
        pos += 45;
    }
    return v;
}

void oro_voc_destroy(void* h) { delete (Vocab*)h; }

int oro_voc_transform(void* h, const uint8_t* desc, int n, int levelsup, uint32_t* bow_ids, double* bow_w, int* bow_n,
                      uint32_t* fv_ids, int32_t* fv_off, uint32_t* fv_idx, int* fv_n) {
    const Vocab& v = *(const Vocab*)h;
    std::map<uint32_t, double> bv;                       // DBoW2::BowVector
    std::map<uint32_t, std::vector<unsigned>> fv;        // DBoW2::FeatureVector
    *bow_n = 0;
    *fv_n = 0;
    fv_off[0] = 0;
    if (v.words.empty()) return 0;
    bool must = true, l1 = true;                          // ScoringObject.h:74-89
    if (v.scoring == 1) l1 = false;
    if (v.scoring == 5) must = false;
    const bool tf = v.weighting == 0 || v.weighting == 1;
    for (int i = 0; i < n; i++) {
        int id = 0, nid = 0;
        double w = 0;
        transform1(v, desc + 32 * (size_t)i, id, w, &nid, levelsup);
        if (w > 0) {
            if (tf) {
                auto it = bv.lower_bound(id);
                if (it != bv.end() && !(id < (int)it->first)) it->second += w;   // addWeight
                else bv.insert(it, {id, w});
            } else {
                auto it = bv.lower_bound(id);
                if (it == bv.end() || id < (int)it->first) bv.insert(it, {id, w});   // addIfNotExist
            }
            fv[nid].push_back(i);   // addFeature
        }
    }
    if (tf && !bv.empty() && !must) {
        const double nd = bv.size();
        for (auto& e : bv) e.second /= nd;
    }
    if (must) {   // BowVector::normalize
        double norm = 0.0;
        if (l1) {
            for (auto& e : bv) norm += fabs(e.second);
        } else {
            for (auto& e : bv) norm += e.second * e.second;
            norm = sqrt(norm);
        }
        if (norm > 0.0)
            for (auto& e : bv) e.second /= norm;
    }
    int j = 0;
    for (auto& e : bv) { bow_ids[j] = e.first; bow_w[j] = e.second; j++; }
    *bow_n = j;
    int f = 0, o = 0;
    for (auto& e : fv) {
        fv_ids[f] = e.first;
        fv_off[f] = o;
        for (unsigned x : e.second) fv_idx[o++] = x;
        f++;
    }
    fv_off[f] = o;
    *fv_n = f;
    return 0;
}

}  // extern "C"
