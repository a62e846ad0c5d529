// Example / test driver for the C++ mirror: reads a raw 8-bit image
// (rows x cols bytes), runs ORBextractor::operator() on the MI355X and writes
// keypoints (28 B each) then descriptors (32 B each) to the output file,
// preceded by the int32 keypoint count.
//   extract_example in.raw rows cols nfeatures out.bin
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ORBextractor.hpp"

int main(int argc, char** argv)
{
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s in.raw rows cols nfeatures out.bin\n", argv[0]);
        return 2;
    }
    const int rows = std::atoi(argv[2]), cols = std::atoi(argv[3]), nfeat = std::atoi(argv[4]);
    std::vector<uint8_t> img((size_t)rows * cols);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(img.data(), 1, img.size(), f) != img.size()) return 3;
    std::fclose(f);
    try {
        ORB_SLAM2_AMD::ORBextractor ex(nfeat, 1.2f, 8, 20, 7);
        std::vector<ORB_SLAM2_AMD::KeyPoint> kps;
        ORB_SLAM2_AMD::Descriptors desc;
        ORB_SLAM2_AMD::GrayImage im{img.data(), rows, cols, (size_t)cols};
        ex(im, ORB_SLAM2_AMD::GrayImage{}, kps, desc);
        const auto& pyr = ex.ImagePyramid();
        FILE* o = std::fopen(argv[5], "wb");
        const int n = (int)kps.size();
        std::fwrite(&n, 4, 1, o);
        std::fwrite(kps.data(), sizeof(ORB_SLAM2_AMD::KeyPoint), kps.size(), o);
        std::fwrite(desc.data.data(), 1, desc.data.size(), o);
        std::fclose(o);
        std::printf("%d keypoints, %d levels, level 7 %dx%d\n", n, ex.GetLevels(), pyr[7].cols, pyr[7].rows);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
