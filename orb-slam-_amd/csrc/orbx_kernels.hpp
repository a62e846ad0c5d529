// Internal kernel interface of liborbx (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/orbx.h"
#include "orbx_geom.hpp"

namespace orbx {

// Where the levels of frame f live.  Level 0 is the caller's image (no copy);
// levels >= 1 are in the handle's pyramid block.
struct FramePtrs {
    const uint8_t* in;
    size_t in_fstride;
    int in_pitch;
    uint8_t* pyr;
    size_t pyr_fstride;
};

struct ExtractBufs {
    const Geometry* geom;       // device copy
    const Cell* cells;          // device cell table
    const int2* xtab;           // resize tables (levels >= 1)
    const int2* ytab;
    const int4* pyr_bands;      // K1 small-batch band tables (Geometry::pg)
    uint32_t* slots;            // [B][slots_per_frame] FAST candidates
    int* cell_counts;           // [B][ncells]
    uint32_t* spill;            // [B][spill_per_frame] quadtree overflow (packed kp)
    uint32_t* spill_node;       // [B][spill_per_frame]
    uint8_t* qt_nodes;          // [B][qtg_per_frame] K3 node arrays of the levels whose list outgrows LDS
    uint32_t* qt_out;           // [B][out_per_frame] retained keypoints (level coords)
    int* qt_cnt;                // [B][nlevels]
    int* status;                // device error word (bit flags)
    int resize_mode;            // ORBX_RESIZE_* (orbx_set_cv_modes): K1's vertical pass
    int blur_mode;              // ORBX_BLUR_*: K4's GaussianBlur column pass and kernel
};

// OpenCV x86 builds run cv::resize INTER_LINEAR's vertical pass as VResizeLinearVec_32s8u (SSE2) over a dst row's
// first rz_simd_end(w) bytes: 16 at a time while x <= w - 16, then 4 at a time while x < w - 4; the scalar loop
// finishes the 0..4-byte tail (imgproc/src/resize.cpp)
inline int rz_simd_end(int w)
{
    int x = 0;
    while (x <= w - 16) x += 16;
    while (x < w - 4) x += 4;
    return x;
}

// XCD-aware workgroup order.  The dispatcher hands flat workgroup id b to XCD b % 8;
// each XCD has its own 4 MiB L2.  xcd_block maps b to a logical id so that every
// XCD owns one contiguous range of logical ids (whole frames, in order), so the
// overlapping reads of neighbouring cells / keypoint patches hit that XCD's L2.
constexpr int kXcds = 8;
__device__ __forceinline__ int xcd_block(int b, int nblocks)
{
    const int q = nblocks / kXcds, r = nblocks - q * kXcds;
    const int x = b % kXcds, k = b / kXcds;
    return x * q + min(x, r) + k;
}

enum : int {
    kStatusListOverflow = 1,
    kStatusOutOverflow = 2,
    kStatusCapOverflow = 4,
};

// K3 launch plan: runs of consecutive levels sharing a kernel configuration.  glob: the node arrays
// live in global memory (ExtractBufs::qt_nodes) because lcap nodes need more LDS than a workgroup has.
struct QtGroup {
    int l0, nl, nt, kpt, glob, lcap, cellcap;
};
constexpr int kQtMaxGroups = kMaxLevels + 1;
int qt_plan(const Geometry& g, int batch, QtGroup* out);   // returns the group count
// host: decides qt_glob per level and lays out the per-frame global node block (qtg_*); false if a
// level cannot be run at all
bool qt_prepare(Geometry& g);
// quadtree workgroup size and keypoints held in registers per thread at level l (the rest spill
// to global): level 0 holds most candidates, levels >= 2 a few hundred
// (level 0: 16 per thread, or 24 for frames above kQtBigArea pixels, whose level-0 candidates
// would otherwise mostly spill; the 24-wide kernel's 178 VGPRs crowd co-running waves, so
// smaller frames keep 16)
constexpr long long kQtBigArea = 1000000;
constexpr int kQtMergedMaxBatch = 8;   // batches up to this size run all levels in one launch
constexpr int kLatencyMaxBatch = 8;    // batches up to this size: FAST one cell per wave, describe one keypoint per wave
// FAST cells per wave above kLatencyMaxBatch.  Every level's cell list is padded with empty cells to a
// multiple of it, so a wave's cells share one level and its candidates land in that level's slot region.
#ifndef ORBX_FAST_CPW
#define ORBX_FAST_CPW 3
#endif
constexpr int kCellsPerWave = ORBX_FAST_CPW;
// cell_counts flag: the cell's candidates start at its own slot base (it did not fit its wave's output buffer).
// Otherwise they follow the wave's earlier cells' in one run from the slot base of the wave's first cell
// (kCellsPerWave consecutive cells of the level above kLatencyMaxBatch frames, one cell below), so a cell's
// first slot is that base plus the counts of the wave's cells before it (orbx_extract.hip cell_slot_word).
constexpr uint32_t kCellDirect = 0x80000000u;
__host__ __device__ inline int fast_cells_per_wave(int batch) { return batch <= kLatencyMaxBatch ? 1 : kCellsPerWave; }
// Workgroup size and keypoints per thread of level l's quadtree: level 0 holds most candidates
// (KITTI ~6,800), level 1 ~2,700, levels >= 2 a few hundred.  Measured per launch (KITTI, 192 frames):
// fewer waves per workgroup on the small levels does not shorten them (one wave for levels 3-7:
// 70 us against 84 us for 256 threads on levels 2-7 together, plus a separate level-2 launch), since
// a split round is a chain of dependent LDS steps whatever the workgroup size.
// Levels whose node list runs from global memory (LevelGeom::qt_glob) take one configuration.
constexpr int kQtGlobNT = 512, kQtGlobKPT = 8;
__host__ __device__ inline int qt_nt(const Geometry& g, int l)
{
    return g.lv[l].qt_glob ? kQtGlobNT : (l >= 2 ? 256 : 512);
}
__host__ __device__ inline int qt_kpt(const Geometry& g, int l)
{
    return g.lv[l].qt_glob ? kQtGlobKPT : (l == 0 ? g.qt_kpt0 : (l == 1 ? 8 : 4));
}
__host__ __device__ inline int qt_regcap(const Geometry& g, int l) { return qt_nt(g, l) * qt_kpt(g, l); }

// host: K1 small-batch launch groups and their band tables (Geometry::pg) from the resize row tables
bool pyr_plan(Geometry& g, const int2* yt, std::vector<int4>& bands);
void launch_pyramid(const Geometry& g, const ExtractBufs& b, const FramePtrs& p, int batch, hipStream_t s);
size_t pyr_level_lds(const Geometry& g, int l);   // k_pyramid_level's dynamic LDS for level l (>= 1)
void fast_groups(Geometry& g);   // host: FAST launch groups (cell ranges, LDS sizes)
void launch_fast(const Geometry& g, const ExtractBufs& b, const FramePtrs& p, int batch, hipStream_t s);
void launch_quadtree(const Geometry& g, const ExtractBufs& b, int* frame_counts, int batch, hipStream_t s);
void launch_describe(const Geometry& g, const ExtractBufs& b, const FramePtrs& p, orbx_keypoint* kps,
                     uint8_t* desc, int cap, int batch, hipStream_t s);

void launch_allpairs_top2(const uint8_t* q, int nq, const uint8_t* t, int nt, int* bi, int* b1, int* b2,
                          int* part, int nsplit, hipStream_t s);
void launch_best2_csr(const uint8_t* q, int nq, const uint8_t* t, const int* ptr, const int* idx, int tie_last,
                      int* bi, int* b1, int* b2, hipStream_t s);
void launch_allpairs_full(const uint8_t* q, int nq, const uint8_t* t, int nt, uint16_t* out, hipStream_t s);
size_t search_init_scratch_bytes(int nframes, int npairs, int cap);
// prev: [npairs][cap] float2 vbPrevMatched (window centres in, matched F2 positions out) or NULL
void launch_search_init(const orbx_keypoint* kps, const uint8_t* desc, const int* counts, int nframes, int cap,
                        const int* pa, const int* pb, int npairs, const orbm_grid& G, int window, float nnratio,
                        int check_ori, float* prev, void* scratch, int* m12, int* nm, hipStream_t s);

size_t stereo_match_smem(const Geometry& g, int cap);
void launch_stereo(const Geometry& g, const Geometry* d_geom, const FramePtrs& PL, const FramePtrs& PR,
                   const orbx_keypoint* kps, const uint8_t* desc, const int* counts, int cap, const int* fl,
                   const int* fr, int npairs, float bf, float maxD, int rband, float* uright, float* depth, int* sad,
                   int* ngood, hipStream_t s);
constexpr int kStMaxLevels = 32;
struct StBandArgs {
    float scale[kStMaxLevels];   // per-octave scale factor, padded with the last level's
    int nlevels, rows, rband;
    float minD, maxD;
};
size_t stereo_band_smem(int rows, int cap);
void launch_stereo_band(const StBandArgs& a, const orbx_keypoint* kps, const uint8_t* desc, const int* counts, int cap,
                        const int* fl, const int* fr, int npairs, int* best_idx, int* best_dist, hipStream_t s);

void launch_bow(int mode, const orbm_bow_view* v1, const orbm_bow_view* v2, const orbm_triang_params* tp,
                int npairs, int max_nodes1, float nnratio, int check_ori, int* match, int* bins, int stride,
                int* nmatches, hipStream_t s);

size_t proj_scratch_bytes(int nframes, int cap, int pcap);
void launch_proj(const orbx_keypoint* kps, const uint8_t* desc, const float* uright, const uint8_t* claimed,
                 const int* counts, int nframes, int cap, const orbm_proj_point* pts, const uint8_t* pdesc,
                 const int* npts, int pcap, const orbm_proj_params& P, void* scratch, int* match, int* nmatches,
                 hipStream_t s);

void launch_ingest(const uint8_t* src, int batch, int rows, int cols, int channels, int rgb, size_t sstep,
                   size_t sfs, const float* mx, const float* my, int nmaps, int drows, int dcols, uint8_t* dst,
                   size_t dstep, size_t dfs, hipStream_t s);
void launch_depth(const void* src, int depth_type, int batch, int rows, int cols, size_t sstep, size_t sfs,
                  float factor, float* dst, size_t dstep, size_t dfs, hipStream_t s);

size_t pose_scratch_bytes(int nframes, int cap, int pcap);
void launch_pose_search(int mode, const orbx_keypoint* kps, const uint8_t* desc, const float* uright,
                        const uint8_t* claimed, const int* counts, int nframes, int cap, const float* pose,
                        const orbm_map_point* pts, const uint8_t* pdesc, const int* npts, int pcap,
                        const orbm_pose_params& P, void* scratch, int* match, int* nmatches, hipStream_t s);

}  // namespace orbx
