// Frame geometry computed once per (params, rows, cols) on the host and read by
// every kernel.  All of it restates ORB-SLAM2 integer/float geometry:
//   level sizes          src/ORBextractor.cc:1347-1348
//   FAST cell grid        src/ORBextractor.cc:932-972
//   quadtree roots        src/ORBextractor.cc:650-675
//   per-level budgets     src/ORBextractor.cc:496-510
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "orbx_math.hpp"

namespace orbx {

constexpr int kMaxLevels = 16;
constexpr int kEdge = 19;                 // EDGE_THRESHOLD, src/ORBextractor.cc:74
constexpr int kMinBorder = kEdge - 3;     // minBorderX/Y, src/ORBextractor.cc:932
constexpr int kKpCoordBits = 24;          // packed keypoint: x (kp_xbits) | y (24 - kp_xbits) | score (8)

// One FAST cell ROI (src/ORBextractor.cc:952-976), level coordinates.
struct Cell {
    int16_t level, roi_w, roi_h, pad;
    int32_t roi_x0, roi_y0;
    int32_t slot_base;   // first candidate slot of this cell (frame-relative)
    int32_t slot_cap;    // ceil(dw/2)*ceil(dh/2): max strict-NMS survivors
};

struct LevelGeom {
    int w, h, pitch;          // pitch: device row pitch (levels >= 1)
    long long pyr_off;        // byte offset inside a frame's pyramid block (levels >= 1)
    int xtab_off, ytab_off;   // offsets of the resize coefficient tables (levels >= 1)
    int ncells, cell_begin;   // cells of this level in the cell table
    int slot_begin, slot_cap; // candidate slots of this level (frame-relative)
    int nfeat;                // N_l
    int cap;                  // max retained keypoints: max(N_l + 2, 4 * nIni)
    int out_off;              // first output slot of this level (frame-relative)
    int nIni;                 // quadtree root count
    float hX;                 // quadtree root width
    int qw, qh;               // maxX-minX, maxY-minY (quadtree frame)
    float scale;              // mvScaleFactor[l]
    float inv_scale;          // mvInvScaleFactor[l]
    float patch_size;         // (float)(int)(PATCH_SIZE * scale)
    int roi_mw, roi_mh;       // largest FAST cell ROI of this level
    int pyr_win;              // 1: every 4-column group's taps lie in 8 bytes from its first tap (K1 window path)
    int rz_simd_end;          // ORBX_RESIZE_SSE2: columns [0, rz_simd_end) take VResizeLinearVec_32s8u's vertical pass
    // K3 node arrays: in LDS (qt_glob 0), or, for budgets whose node list outgrows a workgroup's LDS,
    // in a per-(frame, level) global region of qtg_bytes at qtg_off inside the frame's node block
    int qt_glob;
    long long qtg_off, qtg_bytes;
};

// K1 small-batch launch group: levels s+1 .. s+n resized from level s in one launch (k_pyramid_fused).  A
// block makes `rows` rows of level s+n and every row of the levels before it that those need; its band-table
// entries (n + 1 int4 per band from bt_off: {first, last, own first, own last} for levels s .. s+n) say which.
struct PyrGroup {
    int s, n, rows, nbands;
    int bt_off;
    int lds_x, lds_y;   // LDS bytes of the two row buffers (levels s, s+2, ... / s+1, s+3, ...)
    int nt;             // threads per block
    int split;          // narrow levels: threads past the first row chunk take further chunks
};

struct Geometry {
    int rows, cols, nlevels;
    int ini_th, min_th;
    int ncells;               // cells over all levels (per frame)
    int slots_per_frame;      // candidate slots per frame
    int out_per_frame;        // sum of level caps
    int spill_per_frame;      // quadtree register-overflow keypoints per frame
    int max_cells_level;      // largest per-level cell count
    int max_roi_w, max_roi_h; // largest FAST cell ROI
    // FAST launches: cells [fast_cb[i], fast_cb[i + 1]) with per-wave LDS sized from that
    // group's largest ROI (fast_rw/rh).  The short, tall cells of the coarse levels get their
    // own launch so they do not lower the occupancy of the fine levels' launch.
    int fast_groups;
    int fast_cb[3], fast_rw[2], fast_rh[2];
    int lcap;                 // quadtree list capacity (max level cap + slack)
    int qt_kpt0;              // level-0 quadtree keypoints per thread (16, or 24 for large frames)
    int kp_xbits;             // packed keypoint x width (pack_kp): 12, or more for images wider than 4096 px
    long long pyr_bytes;      // bytes per frame for levels 1..L-1
    long long qtg_per_frame;  // K3 global node block per frame (0: every level's node list fits LDS)
    int pyr_ngroups;          // K1 small-batch launches (0: per-level launches for every batch)
    PyrGroup pg[kMaxLevels];
    int umax[16];
    LevelGeom lv[kMaxLevels];
};

// Packed candidate / retained keypoint: x (xb bits) | y (24 - xb bits) << xb | score << 24.  xb =
// Geometry::kp_xbits: 12 up to 4096 x 4096, wider images trade y bits for x bits (any image whose sides' bit
// widths sum to 24 or less, e.g. 8192 x 2048)
ORBX_HD uint32_t pack_kp(uint32_t x, uint32_t y, uint32_t s, uint32_t xb)
{
    return x | (y << xb) | (s << 24);
}
ORBX_HD uint32_t kp_x(uint32_t k, uint32_t xb) { return k & ((1u << xb) - 1u); }
ORBX_HD uint32_t kp_y(uint32_t k, uint32_t xb) { return (k >> xb) & ((1u << (kKpCoordBits - xb)) - 1u); }

}  // namespace orbx
