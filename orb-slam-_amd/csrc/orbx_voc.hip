// DBoW2 vocabulary on the device:
//   TemplatedVocabulary::loadFromTextFile   Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424
//   TemplatedVocabulary::transform          :1125-1259
//   BowVector addWeight / addIfNotExist / normalize, FeatureVector addFeature
//
// V1 k_voc_descend  one lane per descriptor: descend from the root, k Hamming
//                   distances per level (first strict minimum), record the node at
//                   depth L - levelsup, the word id and its weight
// V2 k_voc_vectors  one workgroup per frame: bitonic sort of (word, feature) and
//                   (node, feature) keys in LDS -> BowVector (weights accumulated in
//                   feature order, then normalised in word order, as the std::map
//                   walk does) and the FeatureVector as CSR
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <new>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/orbx.h"
#include "orbx_host.hpp"

struct orbx_vocabulary {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0;
    int nnodes = 0, nwords = 0;
    int* d_cbegin = nullptr;    // [nnodes + 1] children CSR
    int* d_child = nullptr;     // [nnodes]
    uint8_t* d_desc = nullptr;  // [nnodes][32]
    int* d_word = nullptr;      // [nnodes] word id (0 unless the file flags the node as a leaf)
    double* d_weight = nullptr; // [nnodes]
};

namespace orbx {

__device__ __forceinline__ int voc_ham(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1)
{
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ __launch_bounds__(256) void k_voc_descend(const int* __restrict__ cbegin, const int* __restrict__ child,
                                                     const uint8_t* __restrict__ vdesc, const int* __restrict__ vword,
                                                     const double* __restrict__ vweight, int nid_level,
                                                     const uint8_t* __restrict__ desc, const int* __restrict__ counts,
                                                     int cap, int* __restrict__ out_word, double* __restrict__ out_w,
                                                     int* __restrict__ out_nid)
{
    const int fr = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    if (i >= min(counts[fr], cap)) return;
    const size_t o = (size_t)fr * cap + i;
    const uint4* d = reinterpret_cast<const uint4*>(desc + o * 32);
    const uint4 a0 = d[0], a1 = d[1];
    int node = 0, level = 0, nid = 0;
    int c0 = cbegin[0], c1 = cbegin[1];
    do {   // TemplatedVocabulary.h:1224-1248
        ++level;
        int best = child[c0];
        const uint4* b = reinterpret_cast<const uint4*>(vdesc + (size_t)best * 32);
        int best_d = voc_ham(a0, a1, b[0], b[1]);
        for (int c = c0 + 1; c < c1; ++c) {
            const int id = child[c];
            const uint4* e = reinterpret_cast<const uint4*>(vdesc + (size_t)id * 32);
            const int dd = voc_ham(a0, a1, e[0], e[1]);
            if (dd < best_d) {
                best_d = dd;
                best = id;
            }
        }
        node = best;
        if (level == nid_level) nid = node;
        c0 = cbegin[node];
        c1 = cbegin[node + 1];
    } while (c1 > c0);   // isLeaf() = no children
    if (nid_level <= 0) nid = 0;
    else if (level < nid_level) nid = node;   // leaf above nid_level: unset in the reference
    out_word[o] = vword[node];
    out_w[o] = vweight[node];
    out_nid[o] = nid;
}

__device__ __forceinline__ void voc_bitonic_u64(unsigned long long* k, int p2)
{
    for (int size = 2; size <= p2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < (p2 >> 1); i += blockDim.x) {
                const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long a = k[lo], b = k[hi];
                if ((a > b) == up) {
                    k[lo] = b;
                    k[hi] = a;
                }
            }
            __syncthreads();
        }
    }
}

// block-wide exclusive scan of 0/1 flags held one per thread-slot: returns the prefix
__device__ int voc_scan(int* s_tmp, int v)
{
    const int tid = threadIdx.x;
    s_tmp[tid] = v;
    __syncthreads();
    for (int o = 1; o < (int)blockDim.x; o <<= 1) {
        const int t = tid >= o ? s_tmp[tid - o] : 0;
        __syncthreads();
        s_tmp[tid] += t;
        __syncthreads();
    }
    const int incl = s_tmp[tid];
    __syncthreads();
    return incl - v;
}

constexpr int kVocNT = 512;

// kG: frames whose p2 keys and weights (16 bytes each) outgrow a workgroup's LDS sort them in a per-frame
// global scratch region of p2max entries (the same network; only the memory differs)
template <bool kG>
__global__ __launch_bounds__(kVocNT) void k_voc_vectors(const int* __restrict__ counts, int cap, int scoring,
                                                        int weighting, const int* __restrict__ fword,
                                                        const double* __restrict__ fw, const int* __restrict__ fnid,
                                                        int* __restrict__ bow_word, double* __restrict__ bow_weight,
                                                        int* __restrict__ bow_n, int* __restrict__ fv_node,
                                                        int* __restrict__ fv_ptr, int* __restrict__ fv_idx,
                                                        int* __restrict__ fv_nn, unsigned long long* __restrict__ gsort,
                                                        int p2max)
{
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_dyn[];
    __shared__ int s_tmp[kVocNT];
    __shared__ int s_total, s_run;
    __shared__ double s_norm;
    const int fr = blockIdx.x, tid = threadIdx.x;
    const int n = min(counts[fr], cap);
    int p2 = 1;
    while (p2 < n) p2 <<= 1;
    unsigned long long* s_key = kG ? gsort + (size_t)fr * 2 * p2max : s_dyn;
    double* s_w = reinterpret_cast<double*>(s_key + p2);   // [p2] BowVector weights
    const size_t base = (size_t)fr * cap;
    const unsigned long long kNone = ~0ull;
    const bool tf = weighting == 0 || weighting == 1;       // TF_IDF / TF: addWeight; IDF / BINARY: addIfNotExist
    const bool must = scoring != 5;                         // DOT_PRODUCT does not normalise (ScoringObject.h:89)

    for (int pass = 0; pass < 2; ++pass) {   // 0: BowVector by word, 1: FeatureVector by node
        for (int i = tid; i < p2; i += kVocNT) {
            unsigned long long key = kNone;
            if (i < n && fw[base + i] > 0)   // stopped words are skipped (:1151)
                key = ((unsigned long long)(uint32_t)(pass ? fnid[base + i] : fword[base + i]) << 20) | (uint32_t)i;
            s_key[i] = key;
        }
        __syncthreads();
        voc_bitonic_u64(s_key, p2);
        // group heads: the first key of each word / node
        if (tid == 0) s_run = 0;
        __syncthreads();
        for (int c0 = 0; c0 < p2; c0 += kVocNT) {
            const int i = c0 + tid;
            const unsigned long long key = i < p2 ? s_key[i] : kNone;
            const bool valid = key != kNone;
            const bool head = valid && (i == 0 || (s_key[i - 1] >> 20) != (key >> 20));
            const int before = voc_scan(s_tmp, head ? 1 : 0);
            const int g = s_run + before + (head ? 0 : -1);   // group index of this key
            if (pass == 0) {
                if (head) {
                    const int f = (int)(key & 0xFFFFF);
                    const double w = fw[base + f];
                    double sum = w;
                    if (tf)
                        for (int j = i + 1; j < p2 && s_key[j] != kNone && (s_key[j] >> 20) == (key >> 20); ++j)
                            sum += w;   // BowVector::addWeight in feature order
                    bow_word[base + s_run + before] = (int)(key >> 20);
                    s_w[s_run + before] = sum;
                }
            } else if (valid) {
                if (head) {
                    fv_node[base + s_run + before] = (int)(key >> 20);
                    fv_ptr[(size_t)fr * (cap + 1) + s_run + before] = i;
                }
                fv_idx[base + i] = (int)(key & 0xFFFFF);
            }
            __syncthreads();
            if (tid == kVocNT - 1) s_run += before + (head ? 1 : 0);
            (void)g;
            __syncthreads();
        }
        if (pass == 0) {
            const int nb = s_run;
            if (tid == 0) {
                double norm = 0.0;
                if (tf && !must && nb > 0) norm = -1.0;   // divide by the word count (:1155-1161)
                if (must) {   // BowVector::normalize, in ascending word order (BowVector.cpp:62-84)
                    if (scoring == 1) {
                        for (int i = 0; i < nb; ++i) norm += s_w[i] * s_w[i];
                        norm = sqrt(norm);
                    } else {
                        for (int i = 0; i < nb; ++i) norm += fabs(s_w[i]);
                    }
                }
                s_norm = norm;
                s_total = nb;
                bow_n[fr] = nb;
            }
            __syncthreads();
            const double norm = s_norm;
            for (int i = tid; i < s_total; i += kVocNT) {
                double v = s_w[i];
                if (norm == -1.0) v /= (double)s_total;
                else if (must && norm > 0.0) v /= norm;
                bow_weight[base + i] = v;
            }
        } else if (tid == 0) {
            int nv = 0;   // features not stopped
            for (int i = p2 - 1; i >= 0; --i)
                if (s_key[i] != kNone) {
                    nv = i + 1;
                    break;
                }
            fv_ptr[(size_t)fr * (cap + 1) + s_run] = nv;
            fv_nn[fr] = s_run;
        }
        __syncthreads();
    }
}

}  // namespace orbx

namespace {

template <class T>
bool vput(T*& d, const T* h, size_t n)
{
    if (hipMalloc((void**)&d, sizeof(T) * (n ? n : 1)) != hipSuccess) return false;
    return n == 0 || hipMemcpy(d, h, sizeof(T) * n, hipMemcpyHostToDevice) == hipSuccess;
}

}  // namespace

extern "C" {

orbx_status orbv_create(int k, int L, int scoring, int weighting, int nnodes, const int32_t* parent,
                        const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device,
                        orbx_vocabulary** out)
{
    if (!out || nnodes < 2 || !parent || !is_leaf || !desc || !weight || L < 1 || scoring < 0 || scoring > 5 ||
        weighting < 0 || weighting > 3)
        return ORBX_EINVAL;
    *out = nullptr;
    for (int i = 1; i < nnodes; ++i)
        if (parent[i] < 0 || parent[i] >= i) return ORBX_EINVAL;   // parents precede children (file order)
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBX_EDEVICE;
    orbx::DeviceGuard guard(device);
    std::vector<int> cbegin(nnodes + 1, 0), child(nnodes, 0), fill(nnodes, 0), word(nnodes, 0);
    for (int i = 1; i < nnodes; ++i) cbegin[parent[i] + 1]++;
    for (int i = 0; i < nnodes; ++i) cbegin[i + 1] += cbegin[i];
    int nwords = 0;
    for (int i = 1; i < nnodes; ++i) {   // children in file order (loadFromTextFile :1385)
        child[cbegin[parent[i]] + fill[parent[i]]++] = i;
        if (is_leaf[i]) word[i] = nwords++;
    }
    if (cbegin[1] == 0) return ORBX_EINVAL;   // the root has no children
    orbx_vocabulary* v = new (std::nothrow) orbx_vocabulary();
    if (!v) return ORBX_ENOMEM;
    v->device = device;
    v->k = k;
    v->L = L;
    v->scoring = scoring;
    v->weighting = weighting;
    v->nnodes = nnodes;
    v->nwords = nwords;
    if (!vput(v->d_cbegin, cbegin.data(), cbegin.size()) || !vput(v->d_child, child.data(), child.size()) ||
        !vput(v->d_desc, desc, (size_t)nnodes * 32) || !vput(v->d_word, word.data(), word.size()) ||
        !vput(v->d_weight, weight, (size_t)nnodes)) {
        orbv_destroy(v);
        return ORBX_ENOMEM;
    }
    *out = v;
    return ORBX_OK;
}

orbx_status orbv_load_text(const char* path, int device, orbx_vocabulary** out)
{
    if (!path || !out) return ORBX_EINVAL;
    std::ifstream f(path);
    if (!f.is_open()) return ORBX_EINVAL;
    std::string s;
    if (!std::getline(f, s)) return ORBX_EINVAL;
    std::stringstream hs(s);
    int k = -1, L = -1, n1 = -1, n2 = -1;
    hs >> k >> L >> n1 >> n2;
    if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return ORBX_EINVAL;   // :1359-1363
    std::vector<int32_t> parent(1, 0);
    std::vector<uint8_t> leaf(1, 0), desc(32, 0);
    std::vector<double> weight(1, 0.0);
    while (std::getline(f, s)) {
        // one node per line; blank lines are skipped (the reference's eof loop turns a trailing
        // newline into an extra root child with an uninitialised descriptor: UB, not reproduced)
        if (s.find_first_not_of(" \t\r\n") == std::string::npos) continue;
        std::stringstream ns(s);
        int pid = 0, isleaf = 0;
        ns >> pid >> isleaf;
        uint8_t d[32];
        for (int i = 0; i < 32; ++i) {
            int x = 0;
            ns >> x;
            d[i] = (uint8_t)x;
        }
        double w = 0.0;
        ns >> w;
        if (ns.fail() || pid < 0 || pid >= (int)parent.size()) return ORBX_EINVAL;
        parent.push_back(pid);
        leaf.push_back(isleaf > 0 ? 1 : 0);
        desc.insert(desc.end(), d, d + 32);
        weight.push_back(w);
    }
    return orbv_create(k, L, n1, n2, (int)parent.size(), parent.data(), leaf.data(), desc.data(), weight.data(),
                       device, out);
}

void orbv_destroy(orbx_vocabulary* v)
{
    if (!v) return;
    orbx::DeviceGuard guard(v->device);
    if (v->d_cbegin) hipFree(v->d_cbegin);
    if (v->d_child) hipFree(v->d_child);
    if (v->d_desc) hipFree(v->d_desc);
    if (v->d_word) hipFree(v->d_word);
    if (v->d_weight) hipFree(v->d_weight);
    delete v;
}

orbx_status orbv_info(const orbx_vocabulary* v, int* k, int* L, int* scoring, int* weighting, int* nnodes,
                      int* nwords)
{
    if (!v) return ORBX_EINVAL;
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (scoring) *scoring = v->scoring;
    if (weighting) *weighting = v->weighting;
    if (nnodes) *nnodes = v->nnodes;
    if (nwords) *nwords = v->nwords;
    return ORBX_OK;
}

orbx_status orbv_transform_batch_device(const orbx_vocabulary* v, const uint8_t* d_desc, const int* d_counts,
                                        int nframes, int cap, int levelsup, int32_t* d_bow_word,
                                        double* d_bow_weight, int* d_bow_n, int32_t* d_fv_node, int32_t* d_fv_ptr,
                                        int32_t* d_fv_idx, int* d_fv_nnodes, void* stream)
{
    if (!v || !d_desc || !d_counts || nframes < 0 || cap <= 0 || cap > ORBV_MAX_FEATURES || !d_bow_word || !d_bow_weight ||
        !d_bow_n || !d_fv_node || !d_fv_ptr || !d_fv_idx || !d_fv_nnodes)
        return ORBX_EINVAL;
    if (nframes == 0) return ORBX_OK;
    orbx::DeviceGuard guard(v->device);
    hipStream_t s = (hipStream_t)stream;
    const size_t nf = (size_t)nframes * cap;
    int p2 = 1;
    while (p2 < cap) p2 <<= 1;
    // sort keys + weights: in LDS up to 8192 features (128 KiB), else in global scratch
    const bool glob = (size_t)p2 * 16 > 128 * 1024;
    void* scratch = nullptr;
    const size_t sort_b = glob ? (size_t)nframes * p2 * 16 : 0;
    if (hipMallocAsync(&scratch, sort_b + nf * (4 + 8 + 4), s) != hipSuccess) return ORBX_ENOMEM;
    unsigned long long* gsort = (unsigned long long*)scratch;
    double* fw = (double*)((uint8_t*)scratch + sort_b);
    int* fword = (int*)(fw + nf);
    int* fnid = fword + nf;
    hipLaunchKernelGGL(orbx::k_voc_descend, dim3((cap + 255) / 256, nframes), dim3(256), 0, s, v->d_cbegin,
                       v->d_child, v->d_desc, v->d_word, v->d_weight, v->L - levelsup, d_desc, d_counts, cap, fword,
                       fw, fnid);
    if (glob) {
        hipLaunchKernelGGL(orbx::k_voc_vectors<true>, dim3(nframes), dim3(orbx::kVocNT), 0, s, d_counts, cap,
                           v->scoring, v->weighting, fword, fw, fnid, d_bow_word, d_bow_weight, d_bow_n, d_fv_node,
                           d_fv_ptr, d_fv_idx, d_fv_nnodes, gsort, p2);
    } else {
        const size_t smem = (size_t)p2 * 16;
        hipFuncSetAttribute((const void*)orbx::k_voc_vectors<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)smem);
        hipLaunchKernelGGL(orbx::k_voc_vectors<false>, dim3(nframes), dim3(orbx::kVocNT), smem, s, d_counts, cap,
                           v->scoring, v->weighting, fword, fw, fnid, d_bow_word, d_bow_weight, d_bow_n, d_fv_node,
                           d_fv_ptr, d_fv_idx, d_fv_nnodes, gsort, p2);
    }
    hipFreeAsync(scratch, s);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbv_transform(const orbx_vocabulary* v, const uint8_t* desc, int n, int levelsup, int32_t* bow_word,
                           double* bow_weight, int* bow_n, int32_t* fv_node, int32_t* fv_ptr, int32_t* fv_idx,
                           int* fv_nnodes)
{
    if (!v || n < 0 || n > ORBV_MAX_FEATURES || !bow_n || !fv_nnodes || !fv_ptr) return ORBX_EINVAL;
    *bow_n = 0;
    *fv_nnodes = 0;
    fv_ptr[0] = 0;
    if (n == 0) return ORBX_OK;
    if (!desc || !bow_word || !bow_weight || !fv_node || !fv_idx) return ORBX_EINVAL;
    const size_t cap = (size_t)n;
    orbx::HostCall c(v->device);
    const size_t ocnt = c.in(&n, sizeof(int));
    const size_t odesc = c.in(desc, cap * 32);
    const size_t ometa = c.out(2 * sizeof(int));   // bow_n, fv_nnodes
    const size_t obw = c.out(cap * sizeof(double));
    const size_t obwd = c.out(cap * sizeof(int32_t));
    const size_t ofnode = c.out(cap * sizeof(int32_t));
    const size_t ofptr = c.out((cap + 1) * sizeof(int32_t));
    const size_t ofidx = c.out(cap * sizeof(int32_t));
    orbx_status st = c.prepare();
    if (st == ORBX_OK) st = c.upload();
    if (st != ORBX_OK) return st;
    int* meta = c.dev_as<int>(ometa);
    st = orbv_transform_batch_device(v, c.dev(odesc), c.dev_as<const int>(ocnt), 1, n, levelsup,
                                     c.dev_as<int32_t>(obwd), c.dev_as<double>(obw), meta, c.dev_as<int32_t>(ofnode),
                                     c.dev_as<int32_t>(ofptr), c.dev_as<int32_t>(ofidx), meta + 1, c.stream());
    if (st != ORBX_OK) return st;
    // every output has room for n entries: fetch them whole with the counts (one round trip)
    int m[2] = {0, 0};
    c.fetch(ometa, m, sizeof(m));
    c.fetch(obwd, bow_word, cap * sizeof(int32_t));
    c.fetch(obw, bow_weight, cap * sizeof(double));
    c.fetch(ofnode, fv_node, cap * sizeof(int32_t));
    c.fetch(ofptr, fv_ptr, (cap + 1) * sizeof(int32_t));
    c.fetch(ofidx, fv_idx, cap * sizeof(int32_t));
    if ((st = c.finish()) != ORBX_OK) return st;
    *bow_n = m[0];
    *fv_nnodes = m[1];
    return ORBX_OK;
}

}  // extern "C"
