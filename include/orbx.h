/*
 * orbx.h — C ABI of the MI355X-native ORB front-end (liborbx.so).
 *
 * Drop-in boundary for the ORB-SLAM2 hot path.  Plain C types
 * only; no OpenCV, no torch.  Every entry point names the reference interface
 * it replaces.  All functions return an orbx_status and never throw.
 *
 * Threading: a handle is single-threaded and owns one HIP stream plus its
 * device workspace (one extractor per thread, like the reference's left/right
 * extractors, src/Frame.cc:94-103).  The orbm_* matchers are re-entrant and
 * thread-safe: each synchronous host call runs on a non-blocking stream of its
 * own with pooled pinned / device buffers (no per-call device allocation, no
 * device-wide synchronisation), so concurrent callers (Tracking, LocalMapping,
 * LoopClosing) never wait on each other's or an extractor's stream.  Every
 * entry point leaves the calling thread's current HIP device as it found it.
 */
#ifndef ORBX_H
#define ORBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    ORBX_OK = 0,
    ORBX_EMPTY = 1,        /* empty input image: outputs untouched (src/ORBextractor.cc:1252) */
    ORBX_EINVAL = -22,
    ORBX_ENOMEM = -12,
    ORBX_EDEVICE = -5,
    ORBX_ENOSPC = -28      /* caller capacity too small */
} orbx_status;

/* Keypoints per frame the matcher searches take (SearchByBoW / SearchForTriangulation views and the
 * projection searches' frames): per-frame state of the greedy replays lives in a workgroup's LDS.  The
 * vocabulary transform takes up to ORBV_MAX_FEATURES descriptors per frame.  The reference has neither
 * limit (src/ORBmatcher.cc:45-129, 159-288; TemplatedVocabulary::transform); INTEGRATION.md §6. */
#define ORBM_MAX_FEATURES 16384
#define ORBV_MAX_FEATURES 65536

/* Layout-identical to cv::KeyPoint {Point2f pt; float size, angle, response; int octave, class_id;} */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbx_keypoint;

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
 * include/ORBextractor.h:51-52; YAML keys ORBextractor.* (src/Tracking.cc:118-122). */
typedef struct {
    int nfeatures;
    float scale_factor;
    int nlevels;
    int ini_th_fast;
    int min_th_fast;
} orbx_params;

typedef struct orbx_handle orbx_handle;

/* Replaces ORBextractor::ORBextractor (src/ORBextractor.cc:466-540). device = HIP ordinal. */
orbx_status orbx_create(const orbx_params* params, int device, orbx_handle** out);
void orbx_destroy(orbx_handle* h);

/* Getters GetLevels/GetScaleFactor/GetScaleFactors/GetInverseScaleFactors/
 * GetScaleSigmaSquares/GetInverseScaleSigmaSquares (include/ORBextractor.h:63-83).
 * Each array has nlevels entries. Any pointer may be NULL. */
orbx_status orbx_get_tables(const orbx_handle* h, int* nlevels, float* scale_factor,
                            float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                            int* features_per_level);

/* OpenCV build the extractor reproduces.  The reference links whatever OpenCV 2.4 / 3.x
 * its user has (CMakeLists.txt:31-37), and the builds differ in the last bit of two primitives it calls:
 *   resize  cv::resize INTER_LINEAR's vertical pass in ComputePyramid (src/ORBextractor.cc:1361):
 *           ORBX_RESIZE_SCALAR  the generic FixedPtCast (h0 b0 + h1 b1 + 2^21) >> 22 (cv::setUseOptimized(false));
 *           ORBX_RESIZE_SSE2    x86 VResizeLinearVec_32s8u on all but a 0..4-px row tail (a stock x86 build).
 *   blur    GaussianBlur(7x7, 2) before computeDescriptors (src/ORBextractor.cc:1300-1306):
 *           ORBX_BLUR_SCALAR    OpenCV <= 3.4.1 integer column pass, kernel [18 34 49 55 49 34 18] / 2^8;
 *           ORBX_BLUR_SSE2      OpenCV <= 3.4.1 x86 SymmColumnVec_32s8u: the same sums rounded half to even on
 *                               every column but the row's width % 4 tail;
 *           ORBX_BLUR_BITEXACT  OpenCV >= 3.4.6 / 4.x fixed-point GaussianBlur, kernel [18 34 48 56 48 34 18] / 2^8.
 * The default is SCALAR / SCALAR, the path the CPU oracle pins.  DESIGN.md section 3 tabulates how far each mode
 * moves the output.  Takes effect from the next extract on the handle. */
enum { ORBX_RESIZE_SCALAR = 0, ORBX_RESIZE_SSE2 = 1 };
enum { ORBX_BLUR_SCALAR = 0, ORBX_BLUR_SSE2 = 1, ORBX_BLUR_BITEXACT = 2 };
orbx_status orbx_set_cv_modes(orbx_handle* h, int resize_mode, int blur_mode);

/* Per-frame keypoint capacity the extractor may need (nfeatures + slack per level).
 * -1 (and ORBX_EINVAL from the extract calls) for a geometry the kernels do not run:
 *   - a level narrower or shorter than one 30-px FAST cell inside its border (the
 *     reference divides by zero there, src/ORBextractor.cc:941-949);
 *   - a level whose quadtree region is less than half as wide as it is tall (nIni = 0,
 *     :650);
 *   - an image whose sides' bit widths sum to more than 24 (keypoint coordinates are packed in 24 bits,
 *     split between x and y by the image's shape: up to 4096 x 4096, 8192 x 2048, 16384 x 1024, ...);
 *   - a level whose resize source rows outgrow a workgroup's 160 KiB of LDS (sides above ~9,700 px).
 * Any keypoint budget runs: a level whose quadtree node list outgrows a workgroup's LDS
 * (about 1,700 keypoints, e.g. Tracking's 2 * nFeatures initialisation extractor at 4,000
 * features, src/Tracking.cc:133) keeps its node arrays in device memory instead. */
int orbx_capacity(const orbx_handle* h, int rows, int cols);

/* Replaces ORBextractor::operator()(image, mask, keypoints, descriptors)
 * (include/ORBextractor.h:58-61, src/ORBextractor.cc:1248-1334).
 * Host image in, host keypoints/descriptors out (desc: cap x 32 bytes, row i
 * belongs to kps[i]).  Synchronous on the handle's stream.  Mask is ignored,
 * as in the reference.  The call's device work (upload, kernels, result copies)
 * is replayed as one hipGraph captured on the first call for an image size and
 * re-captured when the size changes; ORBX_NO_GRAPH=1 in the environment, or a
 * failed capture, falls back to direct launches with identical results. */
orbx_status orbx_extract(orbx_handle* h, const uint8_t* img, int rows, int cols, size_t step,
                         orbx_keypoint* kps, int cap, uint8_t* desc, int* n_out);

/* The public ORBextractor::mvImagePyramid (include/ORBextractor.h:85): level l of
 * the last orbx_extract, copied to host on the first call after each extract (cached
 * until the next one).  The level is unpadded (rows x cols bytes, pitch `step`); the
 * reference's level is a view inside a buffer with an EDGE_THRESHOLD = 19 px
 * BORDER_REFLECT_101 border (src/ORBextractor.cc:1352-1373), which copyMakeBorder of
 * this level rebuilds exactly (FetchPyramid). */
orbx_status orbx_get_level(orbx_handle* h, int level, const uint8_t** data, int* rows, int* cols,
                           size_t* step);

/* Batched device-resident replay (config 2/4): `batch` frames of rows x cols u8 at
 * d_imgs + f*frame_stride (row pitch `step`; frame_stride is not read when batch == 1), already in HBM.
 * Outputs per frame f:
 * d_kps[f*cap + i], d_desc[(f*cap + i)*32], d_counts[f].  Asynchronous on `stream`
 * (a hipStream_t taken literally: NULL is the HIP null stream). */
orbx_status orbx_extract_batch_device(orbx_handle* h, const uint8_t* d_imgs, int batch, int rows,
                                      int cols, size_t step, size_t frame_stride,
                                      orbx_keypoint* d_kps, uint8_t* d_desc, int* d_counts, int cap,
                                      void* stream);

/* The same extraction as orbx_extract_batch_device, issued one stage at a time so that a caller can
 * software-pipeline batches across streams (the VALU-bound FAST / describe stages of one batch beside
 * the latency-bound pyramid / quadtree stages of others).  stage 0: pyramid (and the counts reset),
 * 1: FAST, 2: quadtree (DistributeOctTree; writes d_counts), 3: describe (writes d_kps / d_desc).
 * Every stage takes the batch's full arguments and runs on its own `stream`; the caller orders the
 * four stages of a batch (events) and starts stage 0 of the handle's next batch only after stage 3 of
 * this one has completed (the stages share the handle's workspace).  Stage 0 sizes the workspace for
 * rows x cols x batch; later stages with other sizes return ORBX_EINVAL. */
orbx_status orbx_extract_stage_device(orbx_handle* h, int stage, const uint8_t* d_imgs, int batch, int rows,
                                      int cols, size_t step, size_t frame_stride, orbx_keypoint* d_kps,
                                      uint8_t* d_desc, int* d_counts, int cap, void* stream);

/* Wait for the work queued on `stream` (NULL = HIP null stream) and
 * return the device-side status (ORBX_ENOSPC when a frame exceeded `cap`). */
orbx_status orbx_sync(orbx_handle* h, void* stream);

/* Per-stage device timing (ms, HIP events recorded on the launch stream between
 * the stage kernels).  orbx_set_timing(h, 1) starts a new accumulation window;
 * orbx_get_stage_times returns the per-stage sums over every extract since then, host
 * (orbx_extract, launched directly instead of as a graph while timing is on), batched and
 * stage-split (orbx_extract_stage_device: each stage timed on its own stream).
 * Stages: 0 pyramid (all levels), 1 fast, 2 quadtree, 3 describe. */
orbx_status orbx_set_timing(orbx_handle* h, int enable);
orbx_status orbx_get_stage_times(orbx_handle* h, float* ms, int n);

/* Test hooks: device stage dumps of the last batch, frame f (host buffers).
 * pyramid: concatenated levels w_l*h_l; cand: per level (x_rel,y_rel,score) triples in
 * reference order (vToDistributeKeys); cand_counts[l]. */
orbx_status orbx_debug_pyramid(orbx_handle* h, int frame, uint8_t* out, size_t out_size);
orbx_status orbx_debug_candidates(orbx_handle* h, int frame, int level, int* xys, int cap, int* n);
/* Kernel launches per stage of one batched extract of `batch` frames of rows x cols (measurement
 * hook: per-launch roofline figures): counts[0] pyramid, [1] FAST, [2] quadtree, [3] describe;
 * counts[4]: bit l set if a pyramid launch reads level l. */
orbx_status orbx_debug_launches(orbx_handle* h, int rows, int cols, int batch, int* counts, int n);

/* ---- Stereo (Frame::ComputeStereoMatches, src/Frame.cc:630-872) ----
 * bf = Camera.bf (mbf), fx = K(0,0).  The search limits follow :676-681 with
 * mb = bf / fx (the value src/Frame.cc:140 assigns; the reference reads mb one
 * statement before that assignment).  Outputs mvuRight / mvDepth per left
 * keypoint (-1 = no stereo match) and the number of matches kept after the
 * median cut. */

/* Host path: `left` / `right` are the extractor handles (mpORBextractorLeft/Right)
 * right after their orbx_extract on the two images; kps/desc are what those calls
 * returned.  The SAD stage reads both handles' device pyramids (no pyramid D2H). */
orbx_status orbx_compute_stereo_matches(orbx_handle* left, orbx_handle* right, const orbx_keypoint* kps_l,
                                        const uint8_t* desc_l, int n_l, const orbx_keypoint* kps_r,
                                        const uint8_t* desc_r, int n_r, float bf, float fx, float* u_right,
                                        float* depth, int* n_good);

/* Batched device path (config 3): `npairs` stereo pairs of the handle's last
 * orbx_extract_batch_device batch, left frame d_left[p], right frame d_right[p]
 * (kps/desc/counts/cap as produced by that call; its level-0 images must still be
 * resident).  Outputs d_u_right[p*cap + i], d_depth[p*cap + i], d_n_good[p].
 * Asynchronous on `stream`. */
orbx_status orbx_stereo_batch_device(orbx_handle* h, const orbx_keypoint* d_kps, const uint8_t* d_desc,
                                     const int* d_counts, int cap, const int* d_left, const int* d_right,
                                     int npairs, float bf, float fx, float* d_u_right, float* d_depth,
                                     int* d_n_good, void* stream);

/* ---- Matcher (ORBmatcher Hamming inner loops, include/ORBmatcher.h:37-102) ---- */

/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1728-1744), host helper. */
int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b);

enum { ORBM_TOP2 = 0, ORBM_FULL_U16 = 1 };

/* Config-5 brute force over device descriptors (32 B rows).  TOP2: per query the
 * first-min index and the best/second distances (SearchByBoW tie rule,
 * src/ORBmatcher.cc:214-224).  FULL_U16: the nq x nt distance matrix. */
orbx_status orbm_allpairs_device(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int mode,
                                 int* d_best_idx, int* d_best, int* d_second, uint16_t* d_full,
                                 void* stream);
/* The same on host arrays (SURVEY.md 8b orbm_allpairs), on HIP device `device`; synchronous.
 * nt == 0: TOP2 gives -1 / 256 / 256 per query. */
orbx_status orbm_allpairs(int device, const uint8_t* q, int nq, const uint8_t* t, int nt, int mode, int* best_idx,
                          int* best, int* second, uint16_t* full);

/* The inner loop every ORBmatcher search shares (SURVEY.md 8b orbm_best2_csr): query q's
 * candidates are d_cand_idx[d_cand_ptr[q] .. d_cand_ptr[q+1]) in the caller's visiting order (a
 * GetFeaturesInArea window, a FeatureVector node, ...).  tie_mode ORBM_TIE_FIRST keeps the first
 * candidate at the minimum distance (strict <, e.g. src/ORBmatcher.cc:214-224, 489-505);
 * ORBM_TIE_LAST the last one (dist > bestDist skip, SearchForTriangulation :806-823).  Outputs per
 * query: the best target index (-1 when the list is empty), its distance and the multiset second
 * distance (256 = none, the reference's initial value).  Candidate indices must lie in [0, nt).
 * Asynchronous on `stream`. */
enum { ORBM_TIE_FIRST = 0, ORBM_TIE_LAST = 1 };
orbx_status orbm_best2_csr_device(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, const int* d_cand_ptr,
                                  const int* d_cand_idx, int tie_mode, int* d_best_idx, int* d_best, int* d_second,
                                  void* stream);
/* Host arrays, on HIP device `device`; checks every candidate index.  Synchronous. */
orbx_status orbm_best2_csr(int device, const uint8_t* q, int nq, const uint8_t* t, int nt, const int* cand_ptr,
                           const int* cand_idx, int tie_mode, int* best_idx, int* best, int* second);

/* The coarse stage of Frame::ComputeStereoMatches alone (SURVEY.md 8b orbm_stereo_band,
 * src/Frame.cc:645-757), for callers that keep their own SAD refinement.  Per left keypoint: the right
 * keypoints whose row band [floor(y - 2*scale[o]), ceil(y + 2*scale[o])] holds the left row (int)y,
 * with octave within the left octave +- 1 and x in [xL - max_d, xL - min_d]; the first minimum of the
 * Hamming distance in increasing right index.  Outputs best_idx (-1 when no candidate is below
 * TH_HIGH = 100) and best_dist (100 then); the caller applies thOrbDist (:762).  Left keypoints with
 * y < 0, (int)y >= rows or xL - min_d < 0 get -1 / 100.  scale = the extractor's scale factors
 * (nlevels <= 32); right octaves must lie in [0, nlevels).  n_l, n_r <= 65535, and the row buckets
 * (4 * rows + 11 * cap bytes) must fit one workgroup's LDS (ORBX_ENOSPC otherwise). */
orbx_status orbm_stereo_band(int device, const orbx_keypoint* kps_l, const uint8_t* desc_l, int n_l,
                             const orbx_keypoint* kps_r, const uint8_t* desc_r, int n_r, int rows, const float* scale,
                             int nlevels, float min_d, float max_d, int* best_idx, int* best_dist);
/* Batched: pairs (d_left[p], d_right[p]) of a device batch (kps / desc / counts / cap as
 * orbx_extract_batch_device writes them); outputs d_best_idx[p*cap + i], d_best_dist[p*cap + i].
 * `scale` is a host array.  Asynchronous on `stream`. */
orbx_status orbm_stereo_band_device(const orbx_keypoint* d_kps, const uint8_t* d_desc, const int* d_counts, int cap,
                                    const int* d_left, const int* d_right, int npairs, int rows, const float* scale,
                                    int nlevels, float min_d, float max_d, int* d_best_idx, int* d_best_dist,
                                    void* stream);

/* The Frame grid (Frame's static members, src/Frame.cc:32-33): the image bounds of
 * Frame::ComputeImageBounds (src/Frame.cc:563-621; 0..cols x 0..rows without distortion, the
 * undistorted corners otherwise) and the FRAME_GRID_COLS x FRAME_GRID_ROWS = 64 x 48 cells over
 * them, mfGridElementWidthInv = 64.f / (mnMaxX - mnMinX) and HeightInv = 48.f / (mnMaxY - mnMinY)
 * in float (src/Frame.cc:127-128). */
typedef struct {
    float min_x, min_y;              /* mnMinX, mnMinY */
    float grid_w_inv, grid_h_inv;    /* mfGridElementWidthInv, mfGridElementHeightInv */
} orbm_grid;

/* ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
 * (src/ORBmatcher.cc:417-588) for `npairs` frame pairs (F1 = pair_a[p], F2 = pair_b[p]) of an
 * `nframes` device batch in orbx_extract_batch_device's layout (kps/desc/counts, per-frame
 * capacity `cap`).  The keypoints are the frames' mvKeysUn (the extractor's own output for an
 * undistorted camera) in extractor order: level 0 first.  Candidates come from
 * F2.GetFeaturesInArea (src/Frame.cc:410-495) over `grid`.
 * d_prev_matched: vbPrevMatched per pair, d_prev_matched[(p*cap + i1)*2 + {0,1}] = (x, y), read as
 * the window centres and updated in place with F2's matched keypoint positions (:580-584), as
 * Tracking::MonocularInitialization keeps it across attempts (src/Tracking.cc:599-602, 639-644);
 * NULL = F1's own keypoint positions (the first attempt), not written.
 * Outputs: d_matches12[p*cap + i1] (-1 = none) and d_nmatches[p] (the return value).
 * cap <= 32767.  Pairs with more level-0 keypoints than one workgroup's LDS holds for the greedy
 * pass (about 43 bytes each, ~3,800) run it from device memory.  Asynchronous on `stream`. */
orbx_status orbm_search_for_initialization_device(const orbx_keypoint* d_kps, const uint8_t* d_desc,
                                                  const int* d_counts, int nframes, int cap, const int* d_pair_a,
                                                  const int* d_pair_b, int npairs, const orbm_grid* grid,
                                                  int window, float nnratio, int check_ori, float* d_prev_matched,
                                                  int* d_matches12, int* d_nmatches, void* stream);

/* Host path for one (F1, F2) pair (host arrays), on HIP device `device`: kps1/desc1 = F1.mvKeysUn /
 * mDescriptors (n1), kps2/desc2 = F2's (n2), prev_matched = vbPrevMatched (n1 (x, y) pairs, in/out),
 * matches12 = vnMatches12 (n1), *nmatches = the return value.  nnratio / check_ori are the
 * ORBmatcher(nnratio, checkOri) arguments (Tracking uses 0.9, true).  Synchronous. */
orbx_status orbm_search_for_initialization(int device, const orbx_keypoint* kps1, const uint8_t* desc1, int n1,
                                           const orbx_keypoint* kps2, const uint8_t* desc2, int n2,
                                           const orbm_grid* grid, float* prev_matched, int window, float nnratio,
                                           int check_ori, int* matches12, int* nmatches);

/* The undistorted-camera shorthand of orbm_search_for_initialization_device: bounds 0..cols x
 * 0..rows and vbPrevMatched = F1's keypoints (the benchmark's replay of consecutive pairs). */
orbx_status orbm_search_init_batch_device(const orbx_keypoint* d_kps, const uint8_t* d_desc,
                                          const int* d_counts, int nframes, int cap, const int* d_pair_a,
                                          const int* d_pair_b, int npairs, int rows, int cols,
                                          int window, float nnratio, int check_ori,
                                          int* d_matches12, int* d_nmatches, void* stream);

/* ---- Vocabulary-node searches (SearchByBoW x2, SearchForTriangulation) ----
 * The candidate sets are the shared nodes of two DBoW2::FeatureVector maps
 * (std::map<NodeId, vector<unsigned>>, Thirdparty/DBoW2/DBoW2/FeatureVector.h),
 * passed as CSR: node ids ascending, the feature indices of node k at
 * fv_idx[fv_ptr[k] .. fv_ptr[k+1]) in insertion order.  Nodes hold disjoint
 * feature sets, so every shared node is one independent greedy search on the
 * device; the rotation-consistency filter runs per pair afterwards. */
typedef struct {
    const orbx_keypoint* kps;   /* n keypoints: mvKeysUn (KeyFrame) or mvKeys (Frame) */
    const uint8_t* desc;        /* n x 32 descriptors */
    const uint8_t* has_mp;      /* n flags (see the modes below); NULL = all 0 */
    const float* u_right;       /* n mvuRight values (triangulation); NULL = all -1 (monocular) */
    const int32_t* fv_node;     /* [fv_nnodes] ascending node ids */
    const int32_t* fv_ptr;      /* [fv_nnodes + 1] */
    const int32_t* fv_idx;      /* [fv_ptr[fv_nnodes]] feature indices */
    int32_t n;
    int32_t fv_nnodes;
} orbm_bow_view;

enum {
    /* ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, ...), src/ORBmatcher.cc:159-288.
     * view1 = KF (has_mp = MapPoint present and !isBad), view2 = F.
     * match[iF] = KF feature whose MapPoint is assigned to F feature iF, -1 none. */
    ORBM_BOW_KF_F = 0,
    /* ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, ...), :590-723.
     * has_mp = MapPoint present and !isBad on both sides.  match[idx1] = idx2. */
    ORBM_BOW_KF_KF = 1,
    /* ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12, ...), :725-891 (+ CheckDistEpipolarLine
     * :140-157).  has_mp = GetMapPoint(idx) != NULL.  match[idx1] = idx2 (vMatchedPairs). */
    ORBM_TRIANGULATION = 2
};

typedef struct {
    float F12[9];        /* fundamental matrix KF1 -> KF2, row-major */
    float ex, ey;        /* epipole of KF1's centre in KF2 (src/ORBmatcher.cc:731-736) */
    float scale2[16];    /* KF2 mvScaleFactors */
    float sigma2_2[16];  /* KF2 mvLevelSigma2 */
    int32_t only_stereo; /* bOnlyStereo */
} orbm_triang_params;

/* Batched device path: `npairs` searches; d_view1 / d_view2 / d_tp are device arrays of
 * the structs above whose pointers are device pointers (d_tp only for
 * ORBM_TRIANGULATION).  max_nodes1 >= every view1 fv_nnodes; every view2.n <= ORBM_MAX_FEATURES.  Outputs d_match[p *
 * match_stride + i] (i < view2.n for ORBM_BOW_KF_F, view1.n otherwise) and
 * d_nmatches[p].  nnratio = ORBmatcher::mfNNratio, check_ori = mbCheckOrientation.
 * Asynchronous on `stream`. */
orbx_status orbm_bow_search_device(int mode, const orbm_bow_view* d_view1, const orbm_bow_view* d_view2,
                                   const orbm_triang_params* d_tp, int npairs, int max_nodes1, float nnratio,
                                   int check_ori, int* d_match, int match_stride, int* d_nmatches, void* stream);

/* Host path for one pair (host pointers in the views and tp), run on HIP device `device`.
 * match: view2.n (ORBM_BOW_KF_F) or view1.n ints.  Synchronous. */
orbx_status orbm_bow_search(int device, int mode, const orbm_bow_view* view1, const orbm_bow_view* view2,
                            const orbm_triang_params* tp, float nnratio, int check_ori, int* match, int* nmatches);

/* ---- Projection search: ORBmatcher::SearchByProjection(Frame& F, vector<MapPoint*>, th) ----
 * src/ORBmatcher.cc:45-129, the local-map search of Tracking::SearchLocalPoints (src/Tracking.cc:1234-1244),
 * over Frame::GetFeaturesInArea (src/Frame.cc:410-495).  Per MapPoint, what Frame::isInFrustum left in it: */
typedef struct {
    float proj_x, proj_y, proj_xr;   /* mTrackProjX, mTrackProjY, mTrackProjXR */
    float view_cos;                  /* mTrackViewCos */
    int32_t level;                   /* mnTrackScaleLevel */
    int32_t flags;                   /* bit 0: mbTrackInView && !isBad(); bit 1: Observations() > 0 */
} orbm_proj_point;

typedef struct {
    float min_x, min_y;              /* Frame::mnMinX, mnMinY (image bounds, src/Frame.cc:563-621) */
    float grid_w_inv, grid_h_inv;    /* mfGridElementWidthInv / HeightInv */
    float th;                        /* the th argument */
    float nnratio;                   /* ORBmatcher::mfNNratio */
    float scale[16];                 /* F.mvScaleFactors */
} orbm_proj_params;

/* Batched device path: frame f has d_counts[f] keypoints (mvKeysUn), descriptors, mvuRight and
 * d_claimed (F.mvpMapPoints[i] && Observations() > 0) at f * cap; d_npts[f] MapPoints and their
 * descriptors at f * pcap.  Outputs d_match[f * cap + i] = the MapPoint (index) this call
 * assigned to feature i, -1 (the last one when it overwrote), and d_nmatches[f] (the
 * reference's return value).  cap <= ORBM_MAX_FEATURES.  Asynchronous on `stream`. */
orbx_status orbm_search_by_projection_device(const orbx_keypoint* d_kps, const uint8_t* d_desc, const float* d_uright,
                                             const uint8_t* d_claimed, const int* d_counts, int nframes, int cap,
                                             const orbm_proj_point* d_pts, const uint8_t* d_pdesc, const int* d_npts,
                                             int pcap, const orbm_proj_params* params, int* d_match,
                                             int* d_nmatches, void* stream);

/* Host path for one frame (host arrays), on HIP device `device`.  Synchronous. */
orbx_status orbm_search_by_projection(int device, const orbx_keypoint* kps, const uint8_t* desc, const float* uright,
                                      const uint8_t* claimed, int n, const orbm_proj_point* pts, const uint8_t* pdesc,
                                      int np, const orbm_proj_params* params, int* match, int* nmatches);

/* ---- Pose-projection searches: the other SearchByProjection overloads and Fuse ----
 * Each projects MapPoints with a camera pose and keeps, per MapPoint, the first minimum Hamming
 * distance over the GetFeaturesInArea window (Frame: src/Frame.cc:410-495, KeyFrame:
 * src/KeyFrame.cc:569-608):
 *   ORBM_PROJ_LAST_FRAME  SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
 *                         src/ORBmatcher.cc:1396-1538 (Tracking::TrackWithMotionModel, src/Tracking.cc:937)
 *   ORBM_PROJ_KEYFRAME    SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, sAlreadyFound, th, ORBdist)
 *                         src/ORBmatcher.cc:1540-1667 (Tracking::Relocalization, src/Tracking.cc:1504,1518)
 *   ORBM_PROJ_SIM3        SearchByProjection(KeyFrame* pKF, Scw, vpPoints, vpMatched, th)
 *                         src/ORBmatcher.cc:290-403 (LoopClosing::ComputeSim3, src/LoopClosing.cc:375)
 *   ORBM_FUSE             Fuse(KeyFrame* pKF, vpMapPoints, th)            src/ORBmatcher.cc:893-1043
 *                         (LocalMapping::SearchInNeighbors, src/LocalMapping.cc:489,514)
 *   ORBM_FUSE_SIM3        Fuse(KeyFrame* pKF, Scw, vpPoints, th, vpReplacePoint)  src/ORBmatcher.cc:1045-1168
 *                         (LoopClosing::SearchAndFuse, src/LoopClosing.cc:599)
 * The three searches resolve the reference's in-call claims in MapPoint order (a feature taken
 * earlier in the call is skipped by later MapPoints) and apply the rotation histogram; the two
 * Fuse overloads make no claims during the search, so their per-MapPoint results are
 * independent and the caller applies Replace / AddObservation in MapPoint order. */
enum { ORBM_PROJ_LAST_FRAME = 0, ORBM_PROJ_KEYFRAME = 1, ORBM_PROJ_SIM3 = 2, ORBM_FUSE = 3, ORBM_FUSE_SIM3 = 4 };

typedef struct {
    float x, y, z;                /* MapPoint::GetWorldPos() */
    float nx, ny, nz;             /* GetNormal() (SIM3 and the Fuse modes) */
    float max_dist, min_dist;     /* mfMaxDistance, mfMinDistance (GetMax/MinDistanceInvariance's 1.2f / 0.8f applied inside) */
    float angle;                  /* LAST_FRAME: LastFrame.mvKeysUn[i].angle; KEYFRAME: pKF->mvKeysUn[i].angle */
    int32_t octave;               /* LAST_FRAME: LastFrame.mvKeys[i].octave */
    int32_t flags;                /* bit 0: take part -- LAST_FRAME: pMP && !mvbOutlier[i]; KEYFRAME: pMP && !isBad() &&
                                     !sAlreadyFound.count(pMP); SIM3 / FUSE_SIM3: !isBad() && not already found;
                                     FUSE: pMP && !isBad() && !IsInKeyFrame(pKF).  bit 1: Observations() > 0 */
    int32_t pad;
} orbm_map_point;

typedef struct {
    float fx, fy, cx, cy, bf, b;            /* intrinsics, mbf, mb */
    float min_x, max_x, min_y, max_y;       /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    float grid_w_inv, grid_h_inv;           /* mfGridElementWidthInv / HeightInv */
    float log_scale;                        /* mfLogScaleFactor */
    int32_t nlevels;                        /* mnScaleLevels (1..16) */
    float th;                               /* the th argument */
    int32_t mono;                           /* bMono (LAST_FRAME) */
    int32_t orb_dist;                       /* ORBdist (KEYFRAME) */
    int32_t check_ori;                      /* ORBmatcher::mbCheckOrientation (LAST_FRAME, KEYFRAME) */
    float scale[16];                        /* mvScaleFactors */
    float inv_sigma2[16];                   /* mvInvLevelSigma2 (FUSE) */
} orbm_pose_params;

/* Batched device path.  Frame / KeyFrame f: d_counts[f] keypoints (mvKeysUn), descriptors,
 * mvuRight and d_claimed at f * cap (d_claimed[i] = the reference's "already taken" test on entry:
 * LAST_FRAME mvpMapPoints[i] && Observations() > 0; KEYFRAME mvpMapPoints[i]; SIM3 vpMatched[i];
 * ignored by the Fuse modes); d_pose[f * 24 ..]: row-major 3x4 mTcw (Scw for the SIM3 modes) then,
 * for LAST_FRAME, LastFrame.mTcw; d_npts[f] MapPoints and their descriptors at f * pcap.
 * Search modes: d_match[f * cap + i] = the MapPoint this call assigned to feature i (the last one),
 * -1 untouched, -2 set to NULL by the rotation filter; d_nmatches[f] = the reference's return value.
 * Fuse modes: d_match[f * pcap + m] = the feature MapPoint m fuses into (bestDist <= TH_LOW), -1;
 * d_nmatches[f] = nFused.  cap <= ORBM_MAX_FEATURES.  Asynchronous on `stream`. */
orbx_status orbm_project_search_device(int mode, const orbx_keypoint* d_kps, const uint8_t* d_desc,
                                       const float* d_uright, const uint8_t* d_claimed, const int* d_counts,
                                       int nframes, int cap, const float* d_pose, const orbm_map_point* d_pts,
                                       const uint8_t* d_pdesc, const int* d_npts, int pcap,
                                       const orbm_pose_params* params, int* d_match, int* d_nmatches, void* stream);

/* Host path for one Frame / KeyFrame (host arrays; pose = 24 floats as above), on HIP device
 * `device`.  match: n ints (search modes) or np ints (Fuse modes).  Synchronous. */
orbx_status orbm_project_search(int device, int mode, const orbx_keypoint* kps, const uint8_t* desc,
                                const float* uright, const uint8_t* claimed, int n, const float* pose,
                                const orbm_map_point* pts, const uint8_t* pdesc, int np,
                                const orbm_pose_params* params, int* match, int* nmatches);

/* ---- Image ingest ----
 * The per-frame preparation in front of ORBextractor::operator():
 *   cv::remap(im, imRect, M1, M2, cv::INTER_LINEAR) with the CV_32F maps of initUndistortRectifyMap and the
 *   default BORDER_CONSTANT 0 (Examples/Stereo/stereo_euroc.cc:97-98, 136-137), applied per channel, then
 *   cvtColor(CV_RGB2GRAY / CV_BGR2GRAY / CV_RGBA2GRAY / CV_BGRA2GRAY) for 3- and 4-channel input
 *   (Tracking::GrabImageStereo / GrabImageRGBD / GrabImageMonocular, src/Tracking.cc:180-270).
 * Frame f: d_src + f * src_frame_stride, rows x cols, `channels` (1, 3, 4) interleaved u8, row pitch
 * src_step; rgb = Tracking::mbRGB.  Maps: NULL for no remap (dst_rows x dst_cols must equal rows x cols),
 * else nmaps pairs of dst_rows x dst_cols floats, frame f using pair f % nmaps (2 for a batch holding
 * L0 R0 L1 R1 ...).  Output: gray u8 at d_dst + f * dst_frame_stride, pitch dst_step -- the input
 * layout of orbx_extract_batch_device.  Asynchronous on `stream`. */
orbx_status orbx_ingest_batch_device(const uint8_t* d_src, int batch, int rows, int cols, int channels, int rgb,
                                     size_t src_step, size_t src_frame_stride, const float* d_map_x,
                                     const float* d_map_y, int nmaps, int dst_rows, int dst_cols, uint8_t* d_dst,
                                     size_t dst_step, size_t dst_frame_stride, void* stream);

/* GrabImageRGBD's imDepth.convertTo(imDepth, CV_32F, mDepthMapFactor) (src/Tracking.cc:234-235; the caller
 * keeps the reference's condition for calling it).  depth_type 0: u16, 1: f32 input. */
orbx_status orbx_depth_batch_device(const void* d_src, int depth_type, int batch, int rows, int cols,
                                    size_t src_step, size_t src_frame_stride, float factor, float* d_dst,
                                    size_t dst_step, size_t dst_frame_stride, void* stream);

/* ---- DBoW2 vocabulary (TemplatedVocabulary, Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) ----
 * Frame::ComputeBoW / KeyFrame::ComputeBoW (src/Frame.cc:521-528, src/KeyFrame.cc:59-66) call
 * transform(descriptors, mBowVec, mFeatVec, 4); the FeatureVector it produces is the
 * candidate set of the SearchByBoW / SearchForTriangulation entry points above. */
typedef struct orbx_vocabulary orbx_vocabulary;

/* TemplatedVocabulary::loadFromTextFile (:1338-1424): header "k L scoring weighting", then one
 * node per line "parent is_leaf d0 .. d31 weight" (node ids 1, 2, ... in file order). */
orbx_status orbv_load_text(const char* path, int device, orbx_vocabulary** out);

/* The same vocabulary from arrays: nnodes entries including the root (index 0, whose
 * parent / is_leaf / descriptor / weight are ignored); parent[i] < i. */
orbx_status orbv_create(int k, int L, int scoring, int weighting, int nnodes, const int32_t* parent,
                        const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device,
                        orbx_vocabulary** out);
void orbv_destroy(orbx_vocabulary* v);
orbx_status orbv_info(const orbx_vocabulary* v, int* k, int* L, int* scoring, int* weighting, int* nnodes,
                      int* nwords);

/* TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup) (:1125-1259) for
 * one host descriptor set (n <= ORBV_MAX_FEATURES).  BowVector: bow_n words ascending with their weights
 * (n entries of room); FeatureVector as CSR: fv_nnodes node ids ascending, fv_ptr (n + 1),
 * fv_idx (n).  Synchronous. */
orbx_status orbv_transform(const orbx_vocabulary* v, const uint8_t* desc, int n, int levelsup, int32_t* bow_word,
                           double* bow_weight, int* bow_n, int32_t* fv_node, int32_t* fv_ptr, int32_t* fv_idx,
                           int* fv_nnodes);

/* Batched device path over an extract batch (d_desc [nframes][cap][32], d_counts[nframes],
 * cap <= ORBV_MAX_FEATURES).  Per frame f: d_bow_word / d_bow_weight / d_fv_node / d_fv_idx at f * cap,
 * d_fv_ptr at f * (cap + 1), counts d_bow_n[f] / d_fv_nnodes[f].  The FeatureVector CSR
 * plugs straight into orbm_bow_view.  Asynchronous on `stream`. */
orbx_status orbv_transform_batch_device(const orbx_vocabulary* v, const uint8_t* d_desc, const int* d_counts,
                                        int nframes, int cap, int levelsup, int32_t* d_bow_word,
                                        double* d_bow_weight, int* d_bow_n, int32_t* d_fv_node, int32_t* d_fv_ptr,
                                        int32_t* d_fv_idx, int* d_fv_nnodes, void* stream);

#ifdef __cplusplus
}
#endif
#endif
