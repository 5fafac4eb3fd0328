// DBoW2 TemplatedVocabulary<FORB>::transform on CDNA4 (included into orbfe_engine.hip after the
// matcher, which provides the per-thread arena / stream helpers).
//
// k_bow_descend: one thread per descriptor walks the tree from the root, at every level taking the
// FIRST child with the smallest Hamming distance (strict <, TemplatedVocabulary.h:1231-1243) and
// remembering the node at level L - levelsup; the leaf gives (word id, weight).
// k_bow_assemble (one block): the reference builds std::maps in feature order, so the BowVector
// weights are summed per word in feature order (TF / TF-IDF: addWeight; IDF / BINARY:
// addIfNotExist keeps the first), normalised with the norm summed in ascending word order, and
// the FeatureVector lists feature indices per node in ascending order. Sorting (word, feature) and
// (node, feature) keys reproduces exactly those orders.
#pragma once

struct orbfe_vocabulary {
    int k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0, n_words = 0;
    int device = 0;
    uint32_t* d_desc = nullptr;    // [n_nodes][8]
    int* d_child_off = nullptr;    // [n_nodes + 1] CSR into d_child
    int* d_child = nullptr;        // [n_nodes - 1] child node ids, in insertion order
    int* d_word = nullptr;         // [n_nodes] word id (0 for non-leaf nodes, as Node())
    double* d_weight = nullptr;    // [n_nodes]
};

#define BOW_MAXN 4096

__global__ __launch_bounds__(MT_NT) void k_bow_descend(const uint32_t* __restrict__ vdesc, const int* __restrict__ coff,
                                                       const int* __restrict__ child, const int* __restrict__ vword,
                                                       const double* __restrict__ vweight, const uint32_t* fdesc,
                                                       int n, int nid_level, int* o_word, double* o_w, int* o_nid) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t f[8];
#pragma unroll
    for (int w = 0; w < 8; w++) f[w] = fdesc[8 * i + w];
    int nid = 0;   // nid_level <= 0 -> root (TemplatedVocabulary.h:1222)
    int fin = 0, level = 0;
    while (coff[fin + 1] > coff[fin]) {   // !isLeaf(): children not empty
        ++level;
        const int c0 = coff[fin], c1 = coff[fin + 1];
        int best = child[c0];
        int best_d = 0;
#pragma unroll
        for (int w = 0; w < 8; w++) best_d += __popc(f[w] ^ vdesc[8 * best + w]);
        for (int c = c0 + 1; c < c1; c++) {
            const int id = child[c];
            int d = 0;
#pragma unroll
            for (int w = 0; w < 8; w++) d += __popc(f[w] ^ vdesc[8 * id + w]);
            if (d < best_d) { best_d = d; best = id; }
        }
        fin = best;
        if (level == nid_level) nid = fin;
    }
    o_word[i] = vword[fin];
    o_w[i] = vweight[fin];
    o_nid[i] = nid;
}

__device__ void bow_sort_u64(unsigned long long* a, int n) {
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = n + threadIdx.x; i < P; i += blockDim.x) a[i] = ~0ull;
    SYNC();
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long x = a[i], y = a[ixj];
                    if ((x > y) == ((i & k) == 0)) { a[i] = y; a[ixj] = x; }
                }
            }
            SYNC();
        }
}

__global__ __launch_bounds__(1024) void k_bow_assemble(const int* o_word, const double* o_w, const int* o_nid, int n,
                                                       int weighting, int must, int norm_l1, uint32_t* bow_ids,
                                                       double* bow_w, uint32_t* fv_ids, int* fv_off, uint32_t* fv_idx,
                                                       int* counts) {
    __shared__ unsigned long long s_a[BOW_MAXN];
    __shared__ int s_cnt;
    // BowVector: (word, feature) keys of the features that are not stopped (w > 0)
    if (threadIdx.x == 0) s_cnt = 0;
    SYNC();
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (o_w[i] > 0) s_a[atomicAdd(&s_cnt, 1)] = ((unsigned long long)(uint32_t)o_word[i] << 32) | (uint32_t)i;
    SYNC();
    const int m = s_cnt;
    bow_sort_u64(s_a, m);
    // one entry per word, weights summed in feature order (a serial pass: m <= BOW_MAXN)
    if (threadIdx.x == 0) {
        int nb = 0;
        for (int j = 0; j < m; j++) {
            const uint32_t w = (uint32_t)(s_a[j] >> 32);
            const int f = (int)(s_a[j] & 0xffffffffu);
            if (j == 0 || (uint32_t)(s_a[j - 1] >> 32) != w) {
                bow_ids[nb] = w;
                bow_w[nb] = o_w[f];
                nb++;
            } else if (weighting == ORBFE_TF_IDF || weighting == ORBFE_TF) {
                bow_w[nb - 1] += o_w[f];   // addWeight, feature order
            }                              // IDF / BINARY: addIfNotExist keeps the first
        }
        if (weighting == ORBFE_TF_IDF || weighting == ORBFE_TF) {
            if (nb > 0 && !must) {
                const double nd = (double)nb;
                for (int j = 0; j < nb; j++) bow_w[j] /= nd;
            }
        }
        if (must) {   // BowVector::normalize, ascending word order
            double norm = 0.0;
            if (norm_l1) {
                for (int j = 0; j < nb; j++) norm += fabs(bow_w[j]);
            } else {
                for (int j = 0; j < nb; j++) norm += bow_w[j] * bow_w[j];
                norm = sqrt(norm);
            }
            if (norm > 0.0)
                for (int j = 0; j < nb; j++) bow_w[j] /= norm;
        }
        counts[0] = nb;
    }
    SYNC();
    // FeatureVector: (node, feature) keys of the same features
    if (threadIdx.x == 0) s_cnt = 0;
    SYNC();
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (o_w[i] > 0) s_a[atomicAdd(&s_cnt, 1)] = ((unsigned long long)(uint32_t)o_nid[i] << 32) | (uint32_t)i;
    SYNC();
    bow_sort_u64(s_a, m);
    for (int j = threadIdx.x; j < m; j += blockDim.x) fv_idx[j] = (uint32_t)(s_a[j] & 0xffffffffu);
    if (threadIdx.x == 0) {
        int nf = 0;
        for (int j = 0; j < m; j++) {
            const uint32_t nd = (uint32_t)(s_a[j] >> 32);
            if (j == 0 || (uint32_t)(s_a[j - 1] >> 32) != nd) {
                fv_ids[nf] = nd;
                fv_off[nf] = j;
                nf++;
            }
        }
        fv_off[nf] = m;
        counts[1] = nf;
    }
}

namespace {

int voc_build(int k, int L, int scoring, int weighting, const std::vector<int>& parents,
              const std::vector<uint8_t>& leaf, const std::vector<uint8_t>& desc, const std::vector<double>& weight,
              orbfe_vocabulary** out) {
    const int nn = (int)parents.size();
    if (nn < 1 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3) return ORBFE_E_ARG;
    std::vector<int> nchild(nn + 1, 0), word(nn, 0);
    for (int i = 1; i < nn; i++) {
        if (parents[i] < 0 || parents[i] >= i) return ORBFE_E_ARG;
        nchild[parents[i]]++;
    }
    std::vector<int> off(nn + 1, 0);
    for (int i = 0; i < nn; i++) off[i + 1] = off[i] + nchild[i];
    std::vector<int> fillp(off.begin(), off.end() - 1), child(std::max(nn - 1, 1), 0);
    for (int i = 1; i < nn; i++) child[fillp[parents[i]]++] = i;   // children in insertion order
    int nw = 0;
    for (int i = 1; i < nn; i++)
        if (leaf[i]) word[i] = nw++;
    orbfe_vocabulary* v = new orbfe_vocabulary();
    v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting; v->n_nodes = nn; v->n_words = nw;
    hipError_t e = hipGetDevice(&v->device);
    auto up = [&](void** dst, const void* src, size_t bytes) {
        if (e != hipSuccess) return;
        e = hipMalloc(dst, std::max<size_t>(bytes, 16));
        if (e == hipSuccess && bytes) e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
    };
    up((void**)&v->d_desc, desc.data(), (size_t)nn * 32);
    up((void**)&v->d_child_off, off.data(), (size_t)(nn + 1) * 4);
    up((void**)&v->d_child, child.data(), child.size() * 4);
    up((void**)&v->d_word, word.data(), (size_t)nn * 4);
    up((void**)&v->d_weight, weight.data(), (size_t)nn * 8);
    if (e != hipSuccess) {
        orbfe_vocabulary_destroy(v);
        fprintf(stderr, "orbfe: HIP error %s in vocabulary upload\n", hipGetErrorString(e));
        return ORBFE_E_DEVICE;
    }
    *out = v;
    return ORBFE_OK;
}

}  // namespace

extern "C" {

int orbfe_vocabulary_create(int32_t k, int32_t L, int32_t scoring, int32_t weighting, int32_t n_nodes,
                            const int32_t* parents, const uint8_t* is_leaf, const uint8_t* desc,
                            const double* weights, orbfe_vocabulary** out) {
    if (!out || n_nodes < 1 || !parents || !is_leaf || !desc || !weights) return ORBFE_E_ARG;
    std::vector<int> par(parents, parents + n_nodes);
    std::vector<uint8_t> leaf(is_leaf, is_leaf + n_nodes), d(desc, desc + (size_t)n_nodes * 32);
    std::vector<double> w(weights, weights + n_nodes);
    return voc_build(k, L, scoring, weighting, par, leaf, d, w, out);
}

int orbfe_vocabulary_load_bin(const uint8_t* data, size_t size, orbfe_vocabulary** out) {
    if (!data || !out || size < 16) return ORBFE_E_ARG;
    int hdr[4];
    memcpy(hdr, data, 16);
    const int k = hdr[0], L = hdr[1], n1 = hdr[2], n2 = hdr[3];
    // the reference's sanity checks (TemplatedVocabulary.h:1499-1503)
    if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return ORBFE_E_ARG;
    if (k < 2) return ORBFE_E_ARG;   // the reference divides by k - 1
    const long long expected = (long long)((std::pow((double)k, (double)L + 1) - 1) / (k - 1));
    const size_t rec = 4 + 1 + 32 + 8;
    std::vector<int> par(1, 0);
    std::vector<uint8_t> leaf(1, 0), desc(32, 0);
    std::vector<double> w(1, 0.0);
    size_t pos = 16;
    // nodes are read while the stream has data and fewer than `expected` exist; a truncated
    // trailing record is an error here (the reference would append an uninitialised node)
    while (pos < size && (long long)par.size() < expected) {
        if (pos + rec > size) return ORBFE_E_ARG;
        int pid;
        memcpy(&pid, data + pos, 4);
        par.push_back(pid);
        leaf.push_back(data[pos + 4]);
        desc.insert(desc.end(), data + pos + 5, data + pos + 37);
        double wt;
        memcpy(&wt, data + pos + 37, 8);
        w.push_back(wt);
        pos += rec;
    }
    return voc_build(k, L, n1, n2, par, leaf, desc, w, out);
}

void orbfe_vocabulary_destroy(orbfe_vocabulary* v) {
    if (!v) return;
    void* bufs[] = {v->d_desc, v->d_child_off, v->d_child, v->d_word, v->d_weight};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    delete v;
}

int orbfe_vocabulary_info(const orbfe_vocabulary* v, int32_t* k, int32_t* L, int32_t* n_nodes, int32_t* n_words) {
    if (!v) return ORBFE_E_ARG;
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (n_nodes) *n_nodes = v->n_nodes;
    if (n_words) *n_words = v->n_words;
    return ORBFE_OK;
}

int orbfe_vocabulary_transform(const orbfe_vocabulary* voc, const uint8_t* desc, int32_t n, int32_t levelsup,
                               uint32_t* bow_word_ids, double* bow_weights, int32_t* bow_n,
                               uint32_t* fv_node_ids, int32_t* fv_offsets, uint32_t* fv_indices, int32_t* fv_n) {
    if (!voc || n < 0 || (n > 0 && (!desc || !bow_word_ids || !bow_weights || !fv_node_ids || !fv_indices)) ||
        !bow_n || !fv_n || !fv_offsets)
        return ORBFE_E_ARG;
    *bow_n = 0;
    *fv_n = 0;
    fv_offsets[0] = 0;
    if (voc->n_words == 0 || n == 0) return ORBFE_OK;   // empty(): v and fv cleared
    if (n > BOW_MAXN) return ORBFE_E_CAPACITY;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    if (dev != voc->device) return ORBFE_E_ARG;
    Plan p;
    const size_t o_d = p.upload(desc, (size_t)n * 32);
    const size_t o_word = p.scratch((size_t)n * 4), o_w = p.scratch((size_t)n * 8), o_nid = p.scratch((size_t)n * 4);
    const size_t o_bid = p.scratch((size_t)n * 4), o_bw = p.scratch((size_t)n * 8);
    const size_t o_fid = p.scratch((size_t)n * 4), o_foff = p.scratch((size_t)(n + 1) * 4);
    const size_t o_fidx = p.scratch((size_t)n * 4), o_cnt = p.scratch(16);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    int must = 1, norm_l1 = 1;   // ScoringObject.h:74-89
    if (voc->scoring == ORBFE_L2_NORM) norm_l1 = 0;
    if (voc->scoring == ORBFE_DOT_PRODUCT) must = 0;
    hipLaunchKernelGGL(k_bow_descend, dim3((n + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, voc->d_desc,
                       voc->d_child_off, voc->d_child, voc->d_word, voc->d_weight, ms_ptr<const uint32_t>(o_d), n,
                       voc->L - levelsup, ms_ptr<int>(o_word), ms_ptr<double>(o_w), ms_ptr<int>(o_nid));
    hipLaunchKernelGGL(k_bow_assemble, dim3(1), dim3(1024), 0, s, ms_ptr<const int>(o_word),
                       ms_ptr<const double>(o_w), ms_ptr<const int>(o_nid), n, voc->weighting, must, norm_l1,
                       ms_ptr<uint32_t>(o_bid), ms_ptr<double>(o_bw), ms_ptr<uint32_t>(o_fid), ms_ptr<int>(o_foff),
                       ms_ptr<uint32_t>(o_fidx), ms_ptr<int>(o_cnt));
    HIPCHK(hipGetLastError());
    timer.end();
    int cnt[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(cnt, ms_ptr<int>(o_cnt), 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const int nb = cnt[0], nf = cnt[1];
    if (nb > 0) {
        HIPCHK(hipMemcpyAsync(bow_word_ids, ms_ptr<uint32_t>(o_bid), (size_t)nb * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(bow_weights, ms_ptr<double>(o_bw), (size_t)nb * 8, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipMemcpyAsync(fv_offsets, ms_ptr<int>(o_foff), (size_t)(nf + 1) * 4, hipMemcpyDeviceToHost, s));
    if (nf > 0) HIPCHK(hipMemcpyAsync(fv_node_ids, ms_ptr<uint32_t>(o_fid), (size_t)nf * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    int nidx = 0;
    if (nf > 0) {
        nidx = fv_offsets[nf];
        if (nidx > 0) {
            HIPCHK(hipMemcpyAsync(fv_indices, ms_ptr<uint32_t>(o_fidx), (size_t)nidx * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
    }
    *bow_n = nb;
    *fv_n = nf;
    return ORBFE_OK;
}

}  // extern "C"
