// C++ mirror of ORB_SLAM2::ORBextractor / ORBmatcher::DescriptorDistance over
// the liborbx C ABI (include/orbx.h).  Same names, argument meaning and error
// behaviour as include/ORBextractor.h:45-111 and include/ORBmatcher.h:44;
// OpenCV types are replaced by layout-identical PODs so the header builds
// without OpenCV (INTEGRATION.md shows the cv::Mat / cv::KeyPoint adapter).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/orbx.h"

namespace ORB_SLAM2_AMD {

using KeyPoint = orbx_keypoint;   // == cv::KeyPoint {pt.x, pt.y, size, angle, response, octave, class_id}

// Non-owning 8-bit grayscale view (a CV_8UC1 cv::Mat without OpenCV).
struct GrayImage {
    const uint8_t* data = nullptr;
    int rows = 0, cols = 0;
    size_t step = 0;
    bool empty() const { return data == nullptr || rows <= 0 || cols <= 0; }
};

// N x 32 descriptor matrix (CV_8U), row i belongs to keypoint i.
struct Descriptors {
    std::vector<uint8_t> data;
    int rows = 0;
    const uint8_t* row(int i) const { return data.data() + 32 * (size_t)i; }
    void release() { data.clear(); rows = 0; }
};

class OrbxError : public std::runtime_error {
public:
    OrbxError(const char* fn, int code)
        : std::runtime_error(std::string(fn) + " failed with status " + std::to_string(code)), code(code) {}
    int code;
};

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0)
        : nfeatures_(nfeatures), scaleFactor_(scaleFactor), nlevels_(nlevels)
    {
        orbx_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
        int rc = orbx_create(&p, device, &h_);
        if (rc != ORBX_OK) throw OrbxError("orbx_create", rc);
        mvScaleFactor.resize(nlevels);
        mvInvScaleFactor.resize(nlevels);
        mvLevelSigma2.resize(nlevels);
        mvInvLevelSigma2.resize(nlevels);
        orbx_get_tables(h_, nullptr, nullptr, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                        mvInvLevelSigma2.data(), nullptr);
    }
    ~ORBextractor() { orbx_destroy(h_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // ORBextractor::operator() (src/ORBextractor.cc:1248-1334).  The mask is ignored, as in the
    // reference; an empty image returns without touching the outputs (:1252); zero keypoints
    // release the descriptors (:1274-1276).
    void operator()(const GrayImage& image, const GrayImage& /*mask*/, std::vector<KeyPoint>& keypoints,
                    Descriptors& descriptors)
    {
        if (image.empty()) return;
        const int cap = orbx_capacity(h_, image.rows, image.cols);
        if (cap < 0) throw OrbxError("orbx_capacity", cap);
        keypoints.resize(cap);
        descriptors.data.resize(32 * (size_t)cap);
        int n = 0;
        const int rc = orbx_extract(h_, image.data, image.rows, image.cols, image.step, keypoints.data(), cap,
                                    descriptors.data.data(), &n);
        if (rc != ORBX_OK) throw OrbxError("orbx_extract", rc);
        keypoints.resize(n);
        if (n == 0) {
            descriptors.release();
        } else {
            descriptors.data.resize(32 * (size_t)n);
            descriptors.rows = n;
        }
        pyramid_valid_ = false;
    }

    // Which OpenCV build's resize / GaussianBlur arithmetic to reproduce (orbx_set_cv_modes, SURVEY.md
    // Appendix A): ORBX_RESIZE_SCALAR / _SSE2 and ORBX_BLUR_SCALAR / _SSE2 / _BITEXACT.  Not in the reference's
    // interface: the reference gets whatever its linked OpenCV does.
    void SetOpenCVModes(int resize_mode, int blur_mode)
    {
        int rc = orbx_set_cv_modes(h_, resize_mode, blur_mode);
        if (rc != ORBX_OK) throw OrbxError("orbx_set_cv_modes", rc);
        pyramid_valid_ = false;
    }

    int GetLevels() const { return nlevels_; }
    float GetScaleFactor() const { return scaleFactor_; }
    std::vector<float> GetScaleFactors() const { return mvScaleFactor; }
    std::vector<float> GetInverseScaleFactors() const { return mvInvScaleFactor; }
    std::vector<float> GetScaleSigmaSquares() const { return mvLevelSigma2; }
    std::vector<float> GetInverseScaleSigmaSquares() const { return mvInvLevelSigma2; }

    // The public mvImagePyramid member (include/ORBextractor.h:85), fetched lazily from HBM.
    const std::vector<GrayImage>& ImagePyramid()
    {
        if (!pyramid_valid_) {
            pyramid_.assign(nlevels_, GrayImage{});
            for (int l = 0; l < nlevels_; ++l) {
                GrayImage& g = pyramid_[l];
                const int rc = orbx_get_level(h_, l, &g.data, &g.rows, &g.cols, &g.step);
                if (rc != ORBX_OK) throw OrbxError("orbx_get_level", rc);
            }
            pyramid_valid_ = true;
        }
        return pyramid_;
    }

    orbx_handle* handle() { return h_; }

private:
    orbx_handle* h_ = nullptr;
    int nfeatures_;
    float scaleFactor_;
    int nlevels_;
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
    std::vector<GrayImage> pyramid_;
    bool pyramid_valid_ = false;
};

struct ORBmatcher {
    static const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;   // src/ORBmatcher.cc:37-39
    // ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1728-1744)
    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orbm_descriptor_distance(a, b); }
};

}  // namespace ORB_SLAM2_AMD
