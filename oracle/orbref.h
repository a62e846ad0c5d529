/*
 * orbref — CPU restatement of the ORB-SLAM2 ORB front-end hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity oracle for the
 * MI355X (HIP) implementation in orb-slam-_amd/.  Only tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it.
 * The product path never calls into it.
 *
 * It restates, line by line, the behaviour of
 *   /root/reference/src/ORBextractor.cc   (ORB_SLAM2::ORBextractor)
 *   /root/reference/src/ORBmatcher.cc     (DescriptorDistance, SearchForInitialization,
 *                                          ComputeThreeMaxima)
 *   /root/reference/src/Frame.cc          (AssignFeaturesToGrid / PosInGrid /
 *                                          GetFeaturesInArea, ComputeStereoMatches)
 * with the OpenCV 3.x primitives the reference calls (FAST, resize INTER_LINEAR,
 * GaussianBlur, fastAtan2, cvRound) restated from their published generic
 * scalar code paths, and glibc 2.35 cosf/sinf taken
 * from the host libm.
 *
 * Parity status (see DESIGN.md "Oracle"): the reference cannot be built here
 * (OpenCV absent; src/ORBextractor.cc:160-162 does not compile) and ships no
 * tests or golden vectors.  Pinned: every constant table the
 * reference holds (bit_pattern_31_, umax, level scales, per-level budgets,
 * level sizes, cell grids) via known-answer tests.  Pixel arithmetic at the
 * OpenCV boundary (FAST / resize / GaussianBlur / fastAtan2): PARITY UNPINNED
 * against real OpenCV; restated from its generic scalar path.
 *
 * Determinism: DistributeOctTree breaks size ties by heap address in the
 * reference (src/ORBextractor.cc:815).  This oracle uses the canonical
 * tie-break "creation order" (what a monotone allocator would give).
 */
#ifndef ORBREF_H
#define ORBREF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBREF_MAX_LEVELS 16

/* Layout-identical to cv::KeyPoint (28 bytes). */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbref_keypoint;

typedef struct {
    int nfeatures;
    float scale_factor;
    int nlevels;
    int ini_th_fast;
    int min_th_fast;
} orbref_params;

typedef struct {
    int nlevels;
    int nfeatures;
    float scale[ORBREF_MAX_LEVELS];
    float inv_scale[ORBREF_MAX_LEVELS];
    float sigma2[ORBREF_MAX_LEVELS];
    float inv_sigma2[ORBREF_MAX_LEVELS];
    int nfeat_level[ORBREF_MAX_LEVELS];
    int umax[16];
} orbref_tables;

/* a1: ORBextractor::ORBextractor  (src/ORBextractor.cc:466-540) */
int orbref_make_tables(const orbref_params* p, orbref_tables* t);

/* a3: level size, src/ORBextractor.cc:1347-1348 */
void orbref_level_size(const orbref_tables* t, int level, int cols, int rows, int* w, int* h);

/* OpenCV resize(INTER_LINEAR) u8 generic path. */
void orbref_resize_linear(const uint8_t* src, int sw, int sh, size_t sstep,
                          uint8_t* dst, int dw, int dh, size_t dstep);

/* SURVEY Appendix A's alternative OpenCV builds.  The reference links whatever OpenCV 2.4 / 3.x the user has
 * (CMakeLists.txt:31-37); the canonical modes (all 0) are OpenCV 3.x's generic scalar paths, what
 * cv::setUseOptimized(false) runs.  The others are restated from OpenCV's published source, not run here
 * (OpenCV is absent): PARITY UNPINNED like the canonical ones.
 *   resize  0 scalar VResizeLinear;  1 SSE2 VResizeLinearVec_32s8u on all but a 0..4-px row tail (A.2)
 *   blur    0 <= 3.4.1 scalar column pass;  1 <= 3.4.1 SSE2 float column pass SymmColumnVec_32s8u (A.3);
 *           2 >= 3.4.6 / 4.1 bit-exact fixed point, error-diffused kernel [18 34 48 56 48 34 18] (A.3)
 *   trig    0 glibc cosf / sinf;  1 correctly rounded (A.5) */
enum { ORBREF_RESIZE_SCALAR = 0, ORBREF_RESIZE_SSE2 = 1 };
enum { ORBREF_BLUR_SCALAR = 0, ORBREF_BLUR_SSE2 = 1, ORBREF_BLUR_BITEXACT = 2 };
enum { ORBREF_TRIG_GLIBC = 0, ORBREF_TRIG_CR = 1 };
typedef struct {
    int resize, blur, trig;
} orbref_cv_modes;
int orbref_resize_simd_end(int width);
void orbref_resize_linear_mode(const uint8_t* src, int sw, int sh, size_t sstep,
                               uint8_t* dst, int dw, int dh, size_t dstep, int mode);
void orbref_blur_kernel(int mode, int k[7]);
void orbref_gaussian_blur7_mode(const uint8_t* src, int w, int h, size_t sstep, uint8_t* dst, size_t dstep, int mode);
void orbref_brief_mode(const uint8_t* blur, size_t step, float kx, float ky, float angle_deg, uint8_t desc[32],
                       int trig_mode);

/* OpenCV FAST_t<16> with non-max suppression on a ROI.
 * Writes (x, y, score) triples in OpenCV emission order; returns the count,
 * or -1 if more than cap keypoints. */
int orbref_fast(const uint8_t* roi, size_t step, int rows, int cols, int threshold,
                int* out_xys, int cap);

/* a4: ComputeKeyPointsOctTree cell loop (src/ORBextractor.cc:932-1002) for one
 * level: returns vToDistributeKeys as (x_rel, y_rel, score) triples. */
int orbref_level_candidates(const uint8_t* level, size_t step, int w, int h,
                            int ini_th, int min_th, int* out_xys, int cap);

/* Number of FAST cells scanned on a w x h level (src/ORBextractor.cc:941-972). */
int orbref_level_cells(int w, int h);

/* a6: DistributeOctTree (src/ORBextractor.cc:644-907), canonical tie-break.
 * Input triples are relative to (minX, minY).  Writes the indices of the
 * retained keypoints in output (list) order; returns the count, -1 if > cap. */
int orbref_distribute(const int* xys, int n, int minX, int maxX, int minY, int maxY,
                      int N, int* out_idx, int cap);

/* a7: IC_Angle (src/ORBextractor.cc:84-128) + fastAtan2. */
float orbref_fast_atan2(float y, float x);
float orbref_ic_angle(const uint8_t* img, size_t step, int cx, int cy, const int* umax);

/* a8: GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) u8. */
void orbref_gaussian_blur7(const uint8_t* src, int w, int h, size_t sstep,
                           uint8_t* dst, size_t dstep);

/* a9: computeOrbDescriptor (src/ORBextractor.cc:141-192), explicit FMA per F6. */
void orbref_brief(const uint8_t* blur, size_t step, float kx, float ky, float angle_deg,
                  uint8_t desc[32]);

/* a2: ORBextractor::operator() (src/ORBextractor.cc:1248-1334).
 * Returns 0 ok, 1 empty image (outputs untouched), -22 bad args, -28 cap too small.
 * Optional stage dumps (may be NULL):
 *   pyramid:       concatenation of the nlevels level images, each w_l*h_l bytes
 *   level_counts:  keypoints retained per level
 *   cand_counts:   FAST candidates (vToDistributeKeys.size()) per level */
int orbref_extract(const orbref_params* p, const uint8_t* img, int rows, int cols, size_t step,
                   orbref_keypoint* kps, int cap, uint8_t* desc, int* n_out,
                   uint8_t* pyramid, int* level_counts, int* cand_counts);
/* The same under the OpenCV build modes m (NULL = canonical). */
int orbref_extract_mode(const orbref_params* p, const orbref_cv_modes* m, const uint8_t* img, int rows, int cols,
                        size_t step, orbref_keypoint* kps, int cap, uint8_t* desc, int* n_out,
                        uint8_t* pyramid, int* level_counts, int* cand_counts);

/* a11: ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1728-1744). */
int orbref_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* a14: ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:417-588) with
 * Frame::AssignFeaturesToGrid/PosInGrid/GetFeaturesInArea (src/Frame.cc:292-518)
 * for an undistorted frame of size cols x rows (ComputeImageBounds, k1 == 0).
 * prev_xy: vbPrevMatched (2*n1 floats), updated in place.  matches12: n1 ints.
 * Returns nmatches. */
int orbref_search_for_initialization(const orbref_keypoint* k1, const uint8_t* d1, int n1,
                                     const orbref_keypoint* k2, const uint8_t* d2, int n2,
                                     float min_x, float max_x, float min_y, float max_y, float* prev_xy,
                                     int* matches12, int window, float nnratio, int check_ori);

/* a15: Frame::ComputeStereoMatches (src/Frame.cc:630-872) for one rectified stereo
 * pair.  pyrL / pyrR: concatenated level images of the left / right extractor
 * (orbref_extract's `pyramid` dump, both rows x cols at level 0).  bf = Camera.bf,
 * fx = K(0,0).  Outputs mvuRight / mvDepth (nL floats, -1 = no match) and, if
 * sad_out != NULL, the best SAD of each pair accepted before the median cut (-1
 * otherwise).  Returns the number of stereo matches kept. */
int orbref_compute_stereo_matches(const orbref_params* p, int rows, int cols, const uint8_t* pyrL,
                                  const uint8_t* pyrR, const orbref_keypoint* kL, const uint8_t* dL, int nL,
                                  const orbref_keypoint* kR, const uint8_t* dR, int nR, float bf, float fx,
                                  float* uRight, float* depth, int* sad_out);

/* The coarse stage of a15 alone (SURVEY.md 8b orbm_stereo_band, src/Frame.cc:645-757): per
 * left keypoint the first-min Hamming right keypoint over its row band, octave +- 1 and
 * x in [xL - maxD, xL - minD].  best_idx -1 / best_dist 100 (TH_HIGH) when nothing beats
 * TH_HIGH or the keypoint is skipped (:699-708).  scale[octave] of the right keypoints. */
int orbref_stereo_band(const orbref_keypoint* kL, const uint8_t* dL, int nL, const orbref_keypoint* kR,
                       const uint8_t* dR, int nR, int rows, const float* scale, float minD, float maxD,
                       int* best_idx, int* best_dist);

/* DBoW2::FeatureVector as CSR: node ids ascending; the feature indices of node k are
 * idx[ptr[k] .. ptr[k+1]) in insertion order (Thirdparty/DBoW2/DBoW2/FeatureVector.cpp:31-47). */
typedef struct {
    const int* node;
    const int* ptr;
    const int* idx;
    int nnodes;
} orbref_featvec;

/* a13: ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches) (src/ORBmatcher.cc:159-288).
 * kf_has_mp[i]: KF feature i has a MapPoint that is not bad.  match_f[iF] = the KF
 * feature whose MapPoint was assigned (-1 none).  Returns nmatches. */
int orbref_search_by_bow_kf_f(const orbref_keypoint* kkf, const uint8_t* dkf, const uint8_t* kf_has_mp, int nkf,
                              const orbref_featvec* fvkf, const orbref_keypoint* kf, const uint8_t* df, int nf,
                              const orbref_featvec* fvf, float nnratio, int check_ori, int* match_f);

/* a13: ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12) (src/ORBmatcher.cc:590-723).
 * match12[idx1] = idx2 whose MapPoint vpMatches12[idx1] receives (-1 none). */
int orbref_search_by_bow_kf_kf(const orbref_keypoint* k1, const uint8_t* d1, const uint8_t* has_mp1, int n1,
                               const orbref_featvec* fv1, const orbref_keypoint* k2, const uint8_t* d2,
                               const uint8_t* has_mp2, int n2, const orbref_featvec* fv2, float nnratio,
                               int check_ori, int* match12);

/* a12: ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:725-891) + CheckDistEpipolarLine
 * (:140-157).  F12 row-major 3x3, (ex, ey) the epipole of KF1 in KF2 (:733-740, computed by the
 * caller), scale2 / sigma2_2 = KF2's mvScaleFactors / mvLevelSigma2.  match12[idx1] = idx2
 * (vMatchedPairs in idx1 order).  Returns nmatches. */
int orbref_search_for_triangulation(const orbref_keypoint* k1, const uint8_t* d1, const uint8_t* has_mp1,
                                    const float* uright1, int n1, const orbref_featvec* fv1,
                                    const orbref_keypoint* k2, const uint8_t* d2, const uint8_t* has_mp2,
                                    const float* uright2, int n2, const orbref_featvec* fv2, const float* F12,
                                    float ex, float ey, const float* scale2, const float* sigma2_2,
                                    int only_stereo, int check_ori, int* match12);

/* §8f row 2: DBoW2 TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)
 * (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1259).  Vocabulary as loaded by
 * loadFromTextFile: nnodes nodes (node 0 = root; parent/is_leaf_flag/desc/weight of node 0
 * unused), L = depth, scoring / weighting = the file's ScoringType / WeightingType.
 * Outputs: the BowVector (bow_n words ascending, their weights) and the FeatureVector as
 * CSR (fv_nnodes node ids ascending, fv_ptr[fv_nnodes + 1], fv_idx).  Arrays sized n (+1). */
int orbref_voc_transform(int nnodes, const int* parent, const uint8_t* is_leaf_flag, const uint8_t* desc,
                         const double* weight, int L, int scoring, int weighting, const uint8_t* feats, int n,
                         int levelsup, int* bow_word, double* bow_weight, int* bow_n, int* fv_node, int* fv_ptr,
                         int* fv_idx, int* fv_nnodes);

/* Per-MapPoint inputs of SearchByProjection(Frame&, vector<MapPoint*>, th) (what
 * Frame::isInFrustum leaves in the MapPoint, src/Frame.cc:345-404). */
typedef struct {
    float proj_x, proj_y, proj_xr;   /* mTrackProjX, mTrackProjY, mTrackProjXR */
    float view_cos;                  /* mTrackViewCos */
    int32_t level;                   /* mnTrackScaleLevel */
    int32_t flags;                   /* bit 0: mbTrackInView && !isBad(); bit 1: Observations() > 0 */
} orbref_proj_point;

/* §8f row 3: ORBmatcher::SearchByProjection(Frame& F, vector<MapPoint*>, th) (src/ORBmatcher.cc:45-129)
 * with GetFeaturesInArea over F's 64x48 grid.  kps = F.mvKeysUn, uright = F.mvuRight,
 * claimed_in[i] = F.mvpMapPoints[i] && Observations() > 0; grid bounds / inverse cell sizes are
 * F.mnMinX, mnMinY, mfGridElementWidthInv, mfGridElementHeightInv; scale = mvScaleFactors.
 * match[i] = the MapPoint index this call assigned to feature i (-1 none).  Returns nmatches. */
int orbref_search_by_projection(const orbref_keypoint* kps, const uint8_t* desc, const float* uright,
                                const uint8_t* claimed_in, int n, float min_x, float min_y, float grid_w_inv,
                                float grid_h_inv, const float* scale, const orbref_proj_point* pts,
                                const uint8_t* pdesc, int np, float th, float nnratio, int* match);

/* §8f row 3, the pose-projection searches.  Each projects MapPoints with a camera pose
 * into a Frame / KeyFrame and takes, per MapPoint, the first minimum Hamming distance over
 * the GetFeaturesInArea window:
 *   ORBREF_PROJ_LAST_FRAME  SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
 *                           src/ORBmatcher.cc:1396-1538
 *   ORBREF_PROJ_KEYFRAME    SearchByProjection(Frame& CurrentFrame, KeyFrame*, sAlreadyFound, th, ORBdist)
 *                           src/ORBmatcher.cc:1540-1667
 *   ORBREF_PROJ_SIM3        SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)  :290-403
 *   ORBREF_FUSE             Fuse(KeyFrame*, vpMapPoints, th)                             :893-1043
 *   ORBREF_FUSE_SIM3        Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint)           :1045-1168
 * Float arithmetic: see DESIGN.md "Projection arithmetic" (cv::Mat products as OpenCV 3.x's
 * small-matrix gemm, the reference's own expressions with GCC -march=native contractions). */
enum { ORBREF_PROJ_LAST_FRAME = 0, ORBREF_PROJ_KEYFRAME = 1, ORBREF_PROJ_SIM3 = 2, ORBREF_FUSE = 3,
       ORBREF_FUSE_SIM3 = 4 };

typedef struct {
    float x, y, z;                /* MapPoint::GetWorldPos() */
    float nx, ny, nz;             /* GetNormal() (Sim3 and Fuse modes) */
    float max_dist, min_dist;     /* mfMaxDistance, mfMinDistance (the 1.2f / 0.8f factors applied inside) */
    float angle;                  /* LAST_FRAME: LastFrame.mvKeysUn[i].angle; KEYFRAME: pKF->mvKeysUn[i].angle */
    int32_t octave;               /* LAST_FRAME: LastFrame.mvKeys[i].octave */
    int32_t flags;                /* bit 0: takes part (see orbx.h); bit 1: Observations() > 0 (LAST_FRAME claims) */
    int32_t pad;
} orbref_map_point;

typedef struct {
    float fx, fy, cx, cy, bf, b;            /* intrinsics, mbf, mb */
    float min_x, max_x, min_y, max_y;       /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    float grid_w_inv, grid_h_inv;           /* mfGridElementWidthInv / HeightInv */
    float log_scale;                        /* mfLogScaleFactor */
    int32_t nlevels;                        /* mnScaleLevels */
    float th;                               /* the th argument */
    int32_t mono;                           /* bMono (LAST_FRAME) */
    int32_t orb_dist;                       /* ORBdist (KEYFRAME) */
    int32_t check_ori;                      /* mbCheckOrientation (LAST_FRAME, KEYFRAME) */
    float scale[16];                        /* mvScaleFactors */
    float inv_sigma2[16];                   /* mvInvLevelSigma2 (FUSE) */
} orbref_pose_params;

/* pose[0..11]: row-major 3x4 mTcw (Scw for the Sim3 modes); pose[12..23]: LastFrame.mTcw (LAST_FRAME).
 * kps = mvKeysUn, uright = mvuRight, claimed_in[i] = the reference's "already taken" test on entry
 * (LAST_FRAME: mvpMapPoints[i] && Observations() > 0; KEYFRAME: mvpMapPoints[i]; SIM3: vpMatched[i];
 * Fuse modes: unused).  Search modes: match[i] (n entries) = MapPoint index assigned to feature i,
 * -1 untouched, -2 set to NULL by the rotation filter; returns nmatches.  Fuse modes: match[m]
 * (np entries) = the feature MapPoint m fuses into (bestDist <= TH_LOW) or -1; returns nFused. */
int orbref_project_search(int mode, const orbref_keypoint* kps, const uint8_t* desc, const float* uright,
                          const uint8_t* claimed_in, int n, const float* pose, const orbref_map_point* pts,
                          const uint8_t* pdesc, int np, const orbref_pose_params* P, int* match);

/* §8f row 4, image ingest.  cv::remap(src, dst, M1, M2, INTER_LINEAR) with CV_32FC1 maps and the
 * default BORDER_CONSTANT 0 (Examples/Stereo/stereo_euroc.cc:136-137; OpenCV 3.x RemapInvoker +
 * remapBilinear, fixed point: coordinates cvRound(m*32), weights (32-f)*..*32, (sum + 2^14) >> 15), then
 * cvtColor RGB/BGR(A)2GRAY (src/Tracking.cc:185-210; OpenCV 3.x RGB2Gray<uchar>: R 4899, G 9617,
 * B 1868, (sum + 2^13) >> 14).  map_x == NULL: no remap (dst is rows x cols).  channels 1, 3 or 4;
 * rgb = Tracking::mbRGB.  dst: dst_rows x dst_cols, pitch dst_step. */
void orbref_ingest(const uint8_t* src, int rows, int cols, int channels, int rgb, size_t src_step,
                   const float* map_x, const float* map_y, int dst_rows, int dst_cols, uint8_t* dst,
                   size_t dst_step);

/* GrabImageRGBD: imDepth.convertTo(imDepth, CV_32F, mDepthMapFactor) (src/Tracking.cc:234-235):
 * (float)d * factor + 0.0f for u16 (depth_type 0) or f32 (depth_type 1) input. */
void orbref_depth_convert(const void* src, int depth_type, int rows, int cols, size_t src_step, float factor,
                          float* dst, size_t dst_step);

/* The shared inner loop of the ORBmatcher searches over a CSR candidate list (SURVEY.md 8b
 * orbm_best2_csr): tie_last 0 keeps the first candidate at the minimum (strict <), 1 the last
 * (SearchForTriangulation's dist > bestDist skip, src/ORBmatcher.cc:806-823); second = the
 * multiset second distance; 256 / -1 for an empty list. */
void orbref_best2_csr(const uint8_t* q, int nq, const uint8_t* t, const int* cand_ptr, const int* cand_idx,
                      int tie_last, int* best_idx, int* best, int* second);

/* Config-5 brute force: per query best index (first min), best and second distance. */
void orbref_allpairs_top2(const uint8_t* q, int nq, const uint8_t* t, int nt,
                          int* best_idx, int* best_d, int* second_d);

#ifdef __cplusplus
}
#endif
#endif
