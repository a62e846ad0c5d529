// Compile check of INTEGRATION.md: every C ABI call the document shows, with the document's argument
// lists and plain types standing in for cv::Mat / cv::KeyPoint / the ORB-SLAM2 objects.  Built (not run)
// by the Makefile, so a snippet that drifts from include/orbx.h breaks the build.
#include <cstdint>
#include <vector>

#include "../../include/orbx.h"

namespace {

struct KeyPoint {   // cv::KeyPoint
    float x, y, size, angle, response;
    int octave, class_id;
};
struct Point2f {
    float x, y;
};
static_assert(sizeof(KeyPoint) == sizeof(orbx_keypoint), "cv::KeyPoint layout");

int snippets(orbx_handle* h, orbx_handle* hl, orbx_handle* hr, orbx_vocabulary* vocab_handle, void* stream)
{
    // section 2: ORBextractor adapter
    int nfeatures = 2000, nlevels = 8, iniThFAST = 20, minThFAST = 7;
    float scaleFactor = 1.2f;
    orbx_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
    orbx_handle* created = nullptr;
    orbx_create(&p, /*device*/ 0, &created);
    std::vector<float> sf(8), isf(8), s2(8), is2(8);
    std::vector<int> fpl(8);
    orbx_get_tables(h, nullptr, nullptr, sf.data(), isf.data(), s2.data(), is2.data(), fpl.data());
    orbx_set_cv_modes(h, ORBX_RESIZE_SSE2, ORBX_BLUR_SSE2);
    orbx_set_cv_modes(h, ORBX_RESIZE_SSE2, ORBX_BLUR_BITEXACT);
    int rows = 376, cols = 1241, cap = orbx_capacity(h, rows, cols), n = 0;
    std::vector<uint8_t> image((size_t)rows * cols), desc((size_t)cap * 32);
    std::vector<KeyPoint> kps(cap);
    orbx_extract(h, image.data(), rows, cols, (size_t)cols, (orbx_keypoint*)kps.data(), cap, desc.data(), &n);
    const uint8_t* d;
    int r, c;
    size_t s;
    orbx_get_level(h, 0, &d, &r, &c, &s);

    // image ingest
    const uint8_t* d_raw = nullptr;
    const float *d_mx = nullptr, *d_my = nullptr;
    uint8_t* d_gray = nullptr;
    orbx_keypoint* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int* d_counts = nullptr;
    int batch = 2, channels = 3, mbRGB = 0, rows_rect = 480, cols_rect = 752;
    orbx_ingest_batch_device(d_raw, batch, rows, cols, channels, mbRGB, cols * channels, (size_t)rows * cols * channels,
                             d_mx, d_my, 2, rows_rect, cols_rect, d_gray, cols_rect, (size_t)rows_rect * cols_rect,
                             stream);
    orbx_extract_batch_device(h, d_gray, batch, rows_rect, cols_rect, cols_rect, (size_t)rows_rect * cols_rect, d_kps,
                              d_desc, d_counts, cap, stream);
    const void* d_depth16 = nullptr;
    float* d_depth = nullptr;
    float mDepthMapFactor = 1.f / 5000;
    orbx_depth_batch_device(d_depth16, 0, batch, rows, cols, 2 * cols, 2 * rows * cols, mDepthMapFactor, d_depth,
                            4 * cols, 4 * rows * cols, stream);

    // section 3: ORBmatcher
    int dist = orbm_descriptor_distance(desc.data(), desc.data() + 32);
    std::vector<Point2f> vbPrevMatched(n);
    std::vector<int> vnMatches12(n);
    const orbm_grid g{0.f, 0.f, 64.f / cols, 48.f / rows};
    int nmatches = 0, windowSize = 100, mbCheckOrientation = 1;
    float mfNNratio = 0.9f;
    orbm_search_for_initialization(0, (const orbx_keypoint*)kps.data(), desc.data(), n, (const orbx_keypoint*)kps.data(),
                                   desc.data(), n, &g, (float*)vbPrevMatched.data(), windowSize, mfNNratio,
                                   mbCheckOrientation, vnMatches12.data(), &nmatches);
    int nframes = 2, npairs = 1;
    const int *d_pair_a = nullptr, *d_pair_b = nullptr;
    float* d_prev = nullptr;
    int *d_m12 = nullptr, *d_nm = nullptr;
    orbm_search_for_initialization_device(d_kps, d_desc, d_counts, nframes, cap, d_pair_a, d_pair_b, npairs, &g, 100,
                                          0.9f, 1, d_prev, d_m12, d_nm, stream);
    orbm_search_init_batch_device(d_kps, d_desc, d_counts, nframes, cap, d_pair_a, d_pair_b, npairs, rows, cols, 100,
                                  0.9f, 1, d_m12, d_nm, stream);

    // ComputeStereoMatches and its coarse stage
    std::vector<float> mvuRight(n, -1.f), mvDepth(n, -1.f), mvScaleFactors(8, 1.f);
    int ngood = 0;
    float mbf = 47.9f, fx = 435.2f, minD = 0.f, maxD = 435.2f;
    orbx_compute_stereo_matches(hl, hr, (const orbx_keypoint*)kps.data(), desc.data(), n,
                                (const orbx_keypoint*)kps.data(), desc.data(), n, mbf, fx, mvuRight.data(),
                                mvDepth.data(), &ngood);
    std::vector<int> bestIdxR(n), bestDist(n);
    orbm_stereo_band(0, (const orbx_keypoint*)kps.data(), desc.data(), n, (const orbx_keypoint*)kps.data(), desc.data(),
                     n, rows, mvScaleFactors.data(), (int)mvScaleFactors.size(), minD, maxD, bestIdxR.data(),
                     bestDist.data());

    // orbm_best2_csr
    std::vector<int> cand_ptr(n + 1), cand_idx(1), best_idx(n), best(n), second(n);
    orbm_best2_csr(0, desc.data(), n, desc.data(), n, cand_ptr.data(), cand_idx.data(), ORBM_TIE_FIRST, best_idx.data(),
                   best.data(), second.data());

    // SearchByProjection(Frame&, vector<MapPoint*>, th)
    float th = 1.f;
    orbm_proj_params prm{0.f, 0.f, 64.f / cols, 48.f / rows, th, mfNNratio, {}};
    std::vector<orbm_proj_point> pts(10);
    std::vector<uint8_t> pdesc(10 * 32), claimed(n);
    std::vector<int> match(n);
    orbm_search_by_projection(0, (const orbx_keypoint*)kps.data(), desc.data(), mvuRight.data(), claimed.data(), n,
                              pts.data(), pdesc.data(), (int)pts.size(), &prm, match.data(), &nmatches);

    // the pose-projection searches
    orbm_pose_params P{fx, fx, 600.f, 180.f, mbf, mbf / fx, 0.f, (float)cols, 0.f, (float)rows, 64.f / cols,
                       48.f / rows, 0.18232f, 8, th, 0, 0, 1, {}, {}};
    std::vector<orbm_map_point> mps(10);
    std::vector<uint8_t> taken(n);
    float pose[24] = {};
    orbm_project_search(0, ORBM_PROJ_LAST_FRAME, (const orbx_keypoint*)kps.data(), desc.data(), mvuRight.data(),
                        taken.data(), n, pose, mps.data(), pdesc.data(), (int)mps.size(), &P, match.data(), &nmatches);

    // ComputeBoW
    std::vector<int32_t> bw(n), node(n), ptr(n + 1), idx(n);
    std::vector<double> bv(n);
    int nb = 0, nn = 0;
    orbv_transform(vocab_handle, desc.data(), n, 4, bw.data(), bv.data(), &nb, node.data(), ptr.data(), idx.data(),
                   &nn);

    // SearchByBoW(KeyFrame*, Frame&)
    std::vector<uint8_t> hasmp(n);
    std::vector<int> n1(1), p1(2), i1(1);
    orbm_bow_view a{(const orbx_keypoint*)kps.data(), desc.data(), hasmp.data(), nullptr, n1.data(), p1.data(),
                    i1.data(), n, (int)n1.size()};
    orbm_bow_view b{(const orbx_keypoint*)kps.data(), desc.data(), nullptr, nullptr, n1.data(), p1.data(), i1.data(),
                    n, (int)n1.size()};
    orbm_bow_search(0, ORBM_BOW_KF_F, &a, &b, nullptr, mfNNratio, mbCheckOrientation, match.data(), &nmatches);
    return dist + nmatches + ngood + nb + nn;
}

}  // namespace

int (*volatile orbx_abi_snippets)(orbx_handle*, orbx_handle*, orbx_handle*, orbx_vocabulary*, void*) = snippets;
