// liborbx C ABI (include/orbx.h): handle, geometry, workspace and launch
// sequencing.  Host code; the kernels are in orbx_extract.hip / orbx_match.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/orbx.h"
#include "orbx_host.hpp"
#include "orbx_kernels.hpp"

using namespace orbx;

namespace {

inline int cv_round(float v) { return (int)std::lrint(v); }
inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
inline int cv_ceil(float v) { int i = (int)v; return i + (i < v); }

struct Tables {
    int nlevels = 0;
    float scale[kMaxLevels], inv_scale[kMaxLevels], sigma2[kMaxLevels], inv_sigma2[kMaxLevels];
    int nfeat[kMaxLevels];
    int umax[16];
};

// ORBextractor::ORBextractor, src/ORBextractor.cc:466-540
bool make_tables(const orbx_params& p, Tables& t)
{
    if (p.nlevels < 1 || p.nlevels > kMaxLevels || p.nfeatures < 0 || !(p.scale_factor > 1.0f)) return false;
    t.nlevels = p.nlevels;
    const double sf = (double)p.scale_factor;
    t.scale[0] = 1.0f;
    t.sigma2[0] = 1.0f;
    for (int i = 1; i < p.nlevels; i++) {
        t.scale[i] = (float)((double)t.scale[i - 1] * sf);
        t.sigma2[i] = t.scale[i] * t.scale[i];
    }
    for (int i = 0; i < p.nlevels; i++) {
        t.inv_scale[i] = 1.0f / t.scale[i];
        t.inv_sigma2[i] = 1.0f / t.sigma2[i];
    }
    const float factor = (float)(1.0f / sf);
    float desired = (float)p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)p.nlevels));
    int sum = 0;
    for (int l = 0; l < p.nlevels - 1; l++) {
        t.nfeat[l] = cv_round(desired);
        sum += t.nfeat[l];
        desired *= factor;
    }
    t.nfeat[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);
    const int vmax = cv_floor(15 * std::sqrt(2.f) / 2 + 1);
    const int vmin = cv_ceil(15 * std::sqrt(2.f) / 2);
    const double hp2 = 15 * 15;
    for (int v = 0; v <= vmax; ++v) t.umax[v] = (int)std::lrint(std::sqrt(hp2 - v * v));
    for (int v = 15, v0 = 0; v >= vmin; --v) {
        while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
        t.umax[v] = v0;
        ++v0;
    }
    return true;
}

short sat_s16(float v)
{
    const int i = cv_round(v);
    return (short)std::min(std::max(i, -32768), 32767);
}

// cv::resize INTER_LINEAR coefficient tables: x: {x0 | x1<<16, a0 | a1<<16},
// y: {y0 | y1<<16, b0 | b1<<16}
void resize_tables(int sw, int sh, int dw, int dh, std::vector<int2>& xt, std::vector<int2>& yt)
{
    const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        const int x1 = sx + 1 < sw ? sx + 1 : sw - 1;
        const int a0 = sat_s16((1.f - fx) * 2048), a1 = sat_s16(fx * 2048);
        xt.push_back(make_int2(sx | (x1 << 16), (a0 & 0xFFFF) | (a1 << 16)));
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        const int b0 = sat_s16((1.f - fy) * 2048), b1 = sat_s16(fy * 2048);
        const int y0 = std::min(std::max(sy, 0), sh - 1), y1 = std::min(std::max(sy + 1, 0), sh - 1);
        yt.push_back(make_int2(y0 | (y1 << 16), (b0 & 0xFFFF) | (b1 << 16)));
    }
}

template <class T>
void dfree(T*& p)
{
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

}  // namespace

struct orbx_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    orbx_params params{};
    Tables tab;
    int resize_mode = ORBX_RESIZE_SCALAR;   // orbx_set_cv_modes
    int blur_mode = ORBX_BLUR_SCALAR;

    // geometry (per rows x cols): the current size's host copy and device tables
    bool geom_ok = false;
    int grows = -1, gcols = -1;
    Geometry geom{};
    std::vector<Cell> cells;
    Geometry* d_geom = nullptr;
    Cell* d_cells = nullptr;
    int2* d_xtab = nullptr;
    int2* d_ytab = nullptr;
    int4* d_pyrbt = nullptr;   // K1 small-batch band tables
    // Every size seen keeps its own immutable device tables: a size switch selects another block
    // instead of rewriting the tables that kernels of an earlier call (still queued on the caller's
    // stream) are reading.  Bounded by the number of distinct image sizes.
    struct GeomBlock {
        int rows, cols;
        Geometry geom;
        std::vector<Cell> cells;
        Geometry* d_geom;
        Cell* d_cells;
        int2* d_xtab;
        int2* d_ytab;
        int4* d_pyrbt;
    };
    std::vector<GeomBlock> geom_blocks;

    // batch workspace
    int batch_cap = 0;
    uint8_t* d_pyr = nullptr;
    uint32_t* d_slots = nullptr;
    int* d_cell_counts = nullptr;
    uint32_t* d_spill = nullptr;
    uint32_t* d_spill_node = nullptr;
    uint8_t* d_qt_nodes = nullptr;
    uint32_t* d_qt_out = nullptr;
    int* d_qt_cnt = nullptr;
    int* d_status = nullptr;

    // host-image path
    uint8_t* d_img = nullptr;
    size_t img_bytes = 0;
    int img_pitch = 0;
    uint8_t* d_out = nullptr;   // [keypoints ocap (64-byte rounded)][descriptors ocap x 32], one D2H copy
    int single_cap = 0;
    uint8_t* h_pin = nullptr;   // pinned staging: image in, count + keypoints + descriptors out
    int* h_status = nullptr;    // pinned status word (a pageable D2H copy can stall on other streams' work)
    size_t pin_bytes = 0;
    // the host path's stream work (H2D image, the extraction kernels, D2H results and status) as one
    // captured hipGraph, replayed while the buffers it was captured with stay the same
    hipGraphExec_t host_graph = nullptr;
    std::vector<const void*> graph_key;
    bool graph_failed = false;

    // The handle's device work is ordered across streams: its workspace (pyramid, candidate slots,
    // quadtree buffers) is shared by every call, so a call on another stream than the last one waits
    // for that call's completion event first (a host extract while a batch is still queued on the
    // caller's stream, or batches of one handle on alternating streams).
    hipEvent_t done_ev = nullptr;
    hipStream_t done_stream = nullptr;
    bool done_pending = false;

    // last batch (for pyramid / debug readback)
    FramePtrs last{};
    int last_batch = 0;
    std::vector<std::vector<uint8_t>> h_levels;
    std::vector<bool> level_cached;

    // timing: one set of 5 events per timed extract call (stage boundaries)
    bool timing = false;
    std::vector<hipEvent_t> ev;
    int ev_used = 0;
    // stage-split extractions (orbx_extract_stage_device): one (start, end) event pair per timed stage
    // call, on that stage's own stream
    std::vector<hipEvent_t> sev;
    std::vector<int> sev_stage;
    int sev_used = 0;

    // Buffers only grow, and an outgrown one is retired until orbx_destroy rather than freed:
    // hipFree / hipHostFree wait for the whole device, which would stall every other stream of the
    // process (the other extractor and matcher threads).  Capacities (bytes) per live buffer.
    std::vector<std::pair<const void*, size_t>> caps;
    std::vector<void*> retired_dev, retired_pin;
};

namespace {

size_t& cap_of(orbx_handle* h, const void* p)
{
    for (auto& c : h->caps)
        if (c.first == p) return c.second;
    h->caps.emplace_back(p, 0);
    return h->caps.back().second;
}

// p holds at least `count` T afterwards (contents not kept); grows geometrically, never frees
template <class T>
bool dalloc(orbx_handle* h, T*& p, size_t count)
{
    const size_t bytes = sizeof(T) * (count ? count : 1);
    if (p && cap_of(h, p) >= bytes) return true;
    if (p) h->retired_dev.push_back((void*)p);
    const size_t want = std::max(bytes, p ? cap_of(h, p) + cap_of(h, p) / 2 : bytes);
    p = nullptr;
    if (hipMalloc((void**)&p, want) != hipSuccess) {
        p = nullptr;
        return false;
    }
    cap_of(h, p) = want;
    return true;
}

// The handle's own stream serves the synchronous host paths only.  It is created on
// first use: device-batch users bring their own streams, and every idle stream would
// still take one of the process's few hardware queues (GPU_MAX_HW_QUEUES).  HIP maps streams
// onto those queues round-robin, and streams that share a queue run in order, so a host call
// could wait behind an unrelated kernel of the application's.  High-priority streams get
// queues of their own, apart from the application's default-priority streams (measured:
// tests/test_gpu_threads.py); the host matchers' streams are high-priority too (orbx_host.hip).
hipStream_t own_stream(orbx_handle* h)
{
    if (!h->stream) {
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
        hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, hi);
    }
    return h->stream;
}

void select_geometry(orbx_handle* h, const orbx_handle::GeomBlock& b)
{
    h->geom = b.geom;
    h->cells = b.cells;
    h->d_geom = b.d_geom;
    h->d_cells = b.d_cells;
    h->d_xtab = b.d_xtab;
    h->d_ytab = b.d_ytab;
    h->d_pyrbt = b.d_pyrbt;
    h->grows = b.rows;
    h->gcols = b.cols;
    h->geom_ok = true;
    h->batch_cap = 0;   // re-size the workspace for this geometry (buffers only grow)
    h->single_cap = 0;
}

template <class T>
bool dalloc_exact(T*& p, size_t count)
{
    p = nullptr;
    if (hipMalloc((void**)&p, sizeof(T) * (count ? count : 1)) != hipSuccess) {
        p = nullptr;
        return false;
    }
    return true;
}

orbx_status ensure_geometry(orbx_handle* h, int rows, int cols)
{
    if (h->geom_ok && h->grows == rows && h->gcols == cols) return ORBX_OK;
    // packed keypoint coordinates (pack_kp): x and y share 24 bits, 12 / 12 up to 4096 x 4096
    auto bits = [](int v) { int b = 0; while ((1 << b) < v) ++b; return b; };
    if (rows <= 0 || cols <= 0 || bits(cols) + bits(rows) > kKpCoordBits) return ORBX_EINVAL;
    const int kp_xbits = std::max(bits(cols), std::min(12, kKpCoordBits - bits(rows)));
    for (const auto& b : h->geom_blocks)
        if (b.rows == rows && b.cols == cols) {
            select_geometry(h, b);
            return ORBX_OK;
        }
    const Tables& t = h->tab;
    Geometry g{};
    g.rows = rows;
    g.cols = cols;
    g.nlevels = t.nlevels;
    g.kp_xbits = kp_xbits;
    g.ini_th = std::min(std::max(h->params.ini_th_fast, 0), 255);
    g.min_th = std::min(std::max(h->params.min_th_fast, 0), 255);
    std::memcpy(g.umax, t.umax, sizeof(g.umax));
    std::vector<Cell> cells;
    std::vector<int2> xt, yt;
    long long pyr = 0;
    int slot = 0, out = 0, maxcells = 1, lcap = 8;
    int prev_w = cols, prev_h = rows;
    for (int l = 0; l < t.nlevels; ++l) {
        LevelGeom& L = g.lv[l];
        // src/ORBextractor.cc:1347-1348
        L.w = cv_round((float)cols * t.inv_scale[l]);
        L.h = cv_round((float)rows * t.inv_scale[l]);
        L.pitch = (L.w + 63) & ~63;
        if (l > 0) {
            L.pyr_off = pyr;
            pyr += (long long)L.pitch * L.h;
            L.xtab_off = (int)xt.size();
            L.ytab_off = (int)yt.size();
            resize_tables(prev_w, prev_h, L.w, L.h, xt, yt);
            L.rz_simd_end = rz_simd_end(L.w);
            L.pyr_win = 1;
            for (int g0 = 0; g0 < L.w; g0 += 4) {   // k_pyramid_level's byte window per 4-column group
                const int first = xt[L.xtab_off + g0].x & 0xFFFF;
                for (int k = 0; k < 4; ++k) {
                    const int x = xt[L.xtab_off + std::min(g0 + k, L.w - 1)].x;
                    if ((x & 0xFFFF) < first || (x >> 16) - first > 7) L.pyr_win = 0;
                }
            }
            // the window path's x4 vertical sums: 4 * 255 * sum(a) * sum(b) + 2^23 < 2^32 (then every
            // result is <= 255 as well); OpenCV's coefficient pairs sum to 2048, give or take a rounding
            long long sa = 0, sb = 0;
            for (int i = L.xtab_off; i < (int)xt.size(); ++i)
                sa = std::max(sa, (long long)(xt[i].y & 0xFFFF) + ((unsigned)xt[i].y >> 16));
            for (int i = L.ytab_off; i < (int)yt.size(); ++i)
                sb = std::max(sb, (long long)(yt[i].y & 0xFFFF) + ((unsigned)yt[i].y >> 16));
            if (4LL * 255 * sa * sb + (1LL << 23) >= (1LL << 32)) L.pyr_win = 0;
        }
        prev_w = L.w;
        prev_h = L.h;
        // FAST cell grid, src/ORBextractor.cc:932-972
        const int minB = kMinBorder;
        const int maxBX = L.w - kEdge + 3, maxBY = L.h - kEdge + 3;
        const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
        const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
        if (nCols <= 0 || nRows <= 0) return ORBX_EINVAL;
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        L.cell_begin = (int)cells.size();
        L.slot_begin = slot;
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(minB + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBY - 3) continue;
            if (maxY > maxBY) maxY = (float)maxBY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minB + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBX - 6) continue;
                if (maxX > maxBX) maxX = (float)maxBX;
                Cell c{};
                c.level = (int16_t)l;
                c.roi_x0 = (int)iniX;
                c.roi_y0 = (int)iniY;
                c.roi_w = (int16_t)((int)maxX - (int)iniX);
                c.roi_h = (int16_t)((int)maxY - (int)iniY);
                if (c.roi_w > 66 || c.roi_h > 66) return ORBX_EINVAL;
                g.max_roi_w = std::max(g.max_roi_w, (int)c.roi_w);
                g.max_roi_h = std::max(g.max_roi_h, (int)c.roi_h);
                L.roi_mw = std::max(L.roi_mw, (int)c.roi_w);
                L.roi_mh = std::max(L.roi_mh, (int)c.roi_h);
                const int dw = c.roi_w - 6, dh = c.roi_h - 6;
                // a FAST wave's cells (kCellsPerWave consecutive cells of the level) write one run from the
                // first one's slot base: it starts on a 128-byte line, so the quadtree's gather reads whole lines
                if (((int)cells.size() - L.cell_begin) % kCellsPerWave == 0) slot = (slot + 31) & ~31;
                c.slot_base = slot;
                c.slot_cap = (dw > 0 && dh > 0) ? ((dw + 1) / 2) * ((dh + 1) / 2) : 0;
                slot += c.slot_cap;
                cells.push_back(c);
            }
        }
        // empty cells up to a whole number of FAST waves (kCellsPerWave): no wave spans two levels
        while (((int)cells.size() - L.cell_begin) % kCellsPerWave) {
            Cell c{};
            c.level = (int16_t)l;
            c.slot_base = slot;
            cells.push_back(c);
        }
        L.ncells = (int)cells.size() - L.cell_begin;
        L.slot_cap = slot - L.slot_begin;
        maxcells = std::max(maxcells, L.ncells);
        // DistributeOctTree roots, src/ORBextractor.cc:650-653
        L.qw = L.w - 2 * kMinBorder;
        L.qh = L.h - 2 * kMinBorder;
        L.nIni = (int)std::round((float)L.qw / L.qh);
        if (L.nIni <= 0) return ORBX_EINVAL;
        L.hX = (float)L.qw / L.nIni;
        L.nfeat = t.nfeat[l];
        L.cap = std::max(L.nfeat + 2, 4 * L.nIni);
        L.out_off = out;
        out += L.cap;
        lcap = std::max(lcap, L.cap + 4);
        L.scale = t.scale[l];
        L.inv_scale = t.inv_scale[l];
        L.patch_size = (float)(int)(31 * t.scale[l]);   // :1013
    }
    g.ncells = (int)cells.size();
    for (int l = 1; l < t.nlevels; ++l)   // a per-level pyramid launch stages its source rows in one workgroup's LDS
        if (pyr_level_lds(g, l) > 160 * 1024) return ORBX_EINVAL;
    std::vector<int4> pyrbt;
    if (!pyr_plan(g, yt.data(), pyrbt)) return ORBX_EINVAL;
    fast_groups(g);
    g.slots_per_frame = (slot + 31) & ~31;   // frames' slot blocks start on 128-byte lines
    g.out_per_frame = out;
    g.max_cells_level = maxcells;
    g.lcap = lcap;
    g.pyr_bytes = (pyr + 255) & ~255LL;
    int spill = 0;
    g.qt_kpt0 = (long long)rows * cols > kQtBigArea ? 24 : 16;
    // node lists too large for a workgroup's LDS run from global memory (any budget the reference takes)
    if (!qt_prepare(g)) return ORBX_EINVAL;
    for (int l = 0; l < t.nlevels; ++l) spill += std::max(0, g.lv[l].slot_cap - qt_regcap(g, l));
    g.spill_per_frame = std::max(spill, 1);

    // once per image size, into fresh buffers that nothing queued can be reading
    orbx_handle::GeomBlock b{rows, cols, g, std::move(cells), nullptr, nullptr, nullptr, nullptr, nullptr};
    auto release = [&b] {
        dfree(b.d_geom);
        dfree(b.d_cells);
        dfree(b.d_xtab);
        dfree(b.d_ytab);
        dfree(b.d_pyrbt);
    };
    if (!dalloc_exact(b.d_geom, 1) || !dalloc_exact(b.d_cells, b.cells.size()) || !dalloc_exact(b.d_xtab, xt.size()) ||
        !dalloc_exact(b.d_ytab, yt.size()) || !dalloc_exact(b.d_pyrbt, pyrbt.size())) {
        release();
        return ORBX_ENOMEM;
    }
    // on a pooled host-call stream (high priority, orbx_host.hip), so that a handle used only through
    // orbx_extract_batch_device never creates a stream of its own (each takes one of the process's
    // few hardware queues); the copies are complete before any later launch on any stream
    {
        HostCall c(h->device);
        hipStream_t s = c.stream();
        if (!s) {
            release();
            return ORBX_EDEVICE;
        }
        hipMemcpyAsync(b.d_geom, &b.geom, sizeof(Geometry), hipMemcpyHostToDevice, s);
        hipMemcpyAsync(b.d_cells, b.cells.data(), sizeof(Cell) * b.cells.size(), hipMemcpyHostToDevice, s);
        if (!xt.empty()) hipMemcpyAsync(b.d_xtab, xt.data(), sizeof(int2) * xt.size(), hipMemcpyHostToDevice, s);
        if (!yt.empty()) hipMemcpyAsync(b.d_ytab, yt.data(), sizeof(int2) * yt.size(), hipMemcpyHostToDevice, s);
        if (!pyrbt.empty())
            hipMemcpyAsync(b.d_pyrbt, pyrbt.data(), sizeof(int4) * pyrbt.size(), hipMemcpyHostToDevice, s);
        if (hipStreamSynchronize(s) != hipSuccess) {
            release();
            return ORBX_EDEVICE;
        }
    }
    h->geom_blocks.push_back(std::move(b));
    select_geometry(h, h->geom_blocks.back());
    return ORBX_OK;
}

orbx_status ensure_batch(orbx_handle* h, int batch)
{
    if (batch <= h->batch_cap) return ORBX_OK;
    const Geometry& g = h->geom;
    const size_t B = (size_t)batch;
    if (!dalloc(h, h->d_pyr, (size_t)g.pyr_bytes * B) || !dalloc(h, h->d_slots, (size_t)g.slots_per_frame * B) ||
        !dalloc(h, h->d_cell_counts, (size_t)g.ncells * B) || !dalloc(h, h->d_spill, (size_t)g.spill_per_frame * B) ||
        !dalloc(h, h->d_spill_node, (size_t)g.spill_per_frame * B) || !dalloc(h, h->d_qt_out, (size_t)g.out_per_frame * B) ||
        !dalloc(h, h->d_qt_cnt, (size_t)g.nlevels * B) || !dalloc(h, h->d_status, 16) ||
        !dalloc(h, h->d_qt_nodes, (size_t)g.qtg_per_frame * B)) {
        h->batch_cap = 0;
        return ORBX_ENOMEM;
    }
    h->batch_cap = batch;
    return ORBX_OK;
}

ExtractBufs bufs(orbx_handle* h)
{
    ExtractBufs b;
    b.geom = h->d_geom;
    b.cells = h->d_cells;
    b.xtab = h->d_xtab;
    b.ytab = h->d_ytab;
    b.pyr_bands = h->d_pyrbt;
    b.slots = h->d_slots;
    b.cell_counts = h->d_cell_counts;
    b.spill = h->d_spill;
    b.spill_node = h->d_spill_node;
    b.qt_nodes = h->d_qt_nodes;
    b.qt_out = h->d_qt_out;
    b.qt_cnt = h->d_qt_cnt;
    b.status = h->d_status;
    b.resize_mode = h->resize_mode;
    b.blur_mode = h->blur_mode;
    return b;
}

// stream s waits for the handle's last device call when that call was queued on another stream
void order_after_last(orbx_handle* h, hipStream_t s)
{
    if (h->done_pending && h->done_stream != s) hipStreamWaitEvent(s, h->done_ev, 0);
}

// the handle's latest device work is the work queued so far on s
void mark_last(orbx_handle* h, hipStream_t s)
{
    if (!h->done_ev && hipEventCreateWithFlags(&h->done_ev, hipEventDisableTiming) != hipSuccess) {
        h->done_ev = nullptr;
        return;
    }
    hipEventRecord(h->done_ev, s);
    h->done_stream = s;
    h->done_pending = true;
}

// the next set of 5 stage-boundary events of a timed handle (orbx_set_timing)
const hipEvent_t* next_stage_events(orbx_handle* h)
{
    if ((size_t)(h->ev_used + 1) * 5 > h->ev.size()) {
        const size_t old = h->ev.size();
        h->ev.resize(old + 5 * 64);
        for (size_t i = old; i < h->ev.size(); ++i) hipEventCreate(&h->ev[i]);
    }
    return &h->ev[(size_t)(h->ev_used++) * 5];
}

// the extraction's stream work alone (no host state): also what the host path's graph captures;
// ev (timed handles): events recorded at the 5 stage boundaries
void enqueue_pipeline(orbx_handle* h, const FramePtrs& P, int batch, orbx_keypoint* kps, uint8_t* desc, int* counts,
                      int cap, hipStream_t s, const hipEvent_t* ev = nullptr)
{
    const Geometry& g = h->geom;
    ExtractBufs b = bufs(h);
    if (counts == h->d_status + 1 && batch == 1) {   // the host path: status and count in one memset
        hipMemsetAsync(h->d_status, 0, 2 * sizeof(int), s);
    } else {
        hipMemsetAsync(counts, 0, sizeof(int) * batch, s);
        hipMemsetAsync(h->d_status, 0, sizeof(int), s);
    }
    if (ev) hipEventRecord(ev[0], s);
    launch_pyramid(g, b, P, batch, s);
    if (ev) hipEventRecord(ev[1], s);
    launch_fast(g, b, P, batch, s);
    if (ev) hipEventRecord(ev[2], s);
    launch_quadtree(g, b, counts, batch, s);
    if (ev) hipEventRecord(ev[3], s);
    launch_describe(g, b, P, kps, desc, cap, batch, s);
    if (ev) hipEventRecord(ev[4], s);
}

orbx_status run_pipeline(orbx_handle* h, const FramePtrs& P, int batch, orbx_keypoint* kps, uint8_t* desc,
                         int* counts, int cap, hipStream_t s)
{
    enqueue_pipeline(h, P, batch, kps, desc, counts, cap, s, h->timing ? next_stage_events(h) : nullptr);
    h->last = P;
    h->last_batch = batch;
    std::fill(h->level_cached.begin(), h->level_cached.end(), false);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

bool ensure_status_word(orbx_handle* h)
{
    if (!h->h_status && hipHostMalloc((void**)&h->h_status, 64, hipHostMallocDefault) != hipSuccess) {
        h->h_status = nullptr;
        return false;
    }
    return true;
}

orbx_status status_from_device(orbx_handle* h, hipStream_t s)
{
    if (!ensure_status_word(h)) return ORBX_ENOMEM;
    if (hipMemcpyAsync(h->h_status, h->d_status, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess)
        return ORBX_EDEVICE;
    if (hipStreamSynchronize(s) != hipSuccess) return ORBX_EDEVICE;
    const int st = *h->h_status;
    if (st & kStatusCapOverflow) return ORBX_ENOSPC;
    if (st) return ORBX_EDEVICE;
    return ORBX_OK;
}

}  // namespace

extern "C" {

orbx_status orbx_create(const orbx_params* params, int device, orbx_handle** out)
{
    if (!params || !out) return ORBX_EINVAL;
    *out = nullptr;
    orbx_handle* h = new (std::nothrow) orbx_handle();
    if (!h) return ORBX_ENOMEM;
    h->params = *params;
    if (!make_tables(*params, h->tab)) {
        delete h;
        return ORBX_EINVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        delete h;
        return ORBX_EDEVICE;
    }
    h->device = device;
    h->h_levels.resize(kMaxLevels);
    h->level_cached.assign(kMaxLevels, false);
    *out = h;
    return ORBX_OK;
}

void orbx_destroy(orbx_handle* h)
{
    if (!h) return;
    DeviceGuard guard(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    if (h->h_pin) hipHostFree(h->h_pin);
    if (h->h_status) hipHostFree(h->h_status);
    for (void* p : h->retired_pin) hipHostFree(p);
    for (void* p : h->retired_dev) (void)hipFree(p);
    for (auto& b : h->geom_blocks) {
        dfree(b.d_geom);
        dfree(b.d_cells);
        dfree(b.d_xtab);
        dfree(b.d_ytab);
        dfree(b.d_pyrbt);
    }
    dfree(h->d_pyr);
    dfree(h->d_slots);
    dfree(h->d_cell_counts);
    dfree(h->d_spill);
    dfree(h->d_spill_node);
    dfree(h->d_qt_nodes);
    dfree(h->d_qt_out);
    dfree(h->d_qt_cnt);
    dfree(h->d_status);
    dfree(h->d_img);
    dfree(h->d_out);
    for (auto& e : h->ev)
        if (e) hipEventDestroy(e);
    for (auto& e : h->sev)
        if (e) hipEventDestroy(e);
    if (h->host_graph) hipGraphExecDestroy(h->host_graph);
    if (h->done_ev) hipEventDestroy(h->done_ev);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
}

orbx_status orbx_set_cv_modes(orbx_handle* h, int resize_mode, int blur_mode)
{
    if (!h || (resize_mode != ORBX_RESIZE_SCALAR && resize_mode != ORBX_RESIZE_SSE2) ||
        (blur_mode != ORBX_BLUR_SCALAR && blur_mode != ORBX_BLUR_SSE2 && blur_mode != ORBX_BLUR_BITEXACT))
        return ORBX_EINVAL;
    h->resize_mode = resize_mode;
    h->blur_mode = blur_mode;
    std::fill(h->level_cached.begin(), h->level_cached.end(), false);
    return ORBX_OK;
}

orbx_status orbx_get_tables(const orbx_handle* h, int* nlevels, float* scale_factor, float* scale, float* inv_scale,
                            float* sigma2, float* inv_sigma2, int* features_per_level)
{
    if (!h) return ORBX_EINVAL;
    const Tables& t = h->tab;
    if (nlevels) *nlevels = t.nlevels;
    if (scale_factor) *scale_factor = h->params.scale_factor;
    for (int l = 0; l < t.nlevels; ++l) {
        if (scale) scale[l] = t.scale[l];
        if (inv_scale) inv_scale[l] = t.inv_scale[l];
        if (sigma2) sigma2[l] = t.sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = t.inv_sigma2[l];
        if (features_per_level) features_per_level[l] = t.nfeat[l];
    }
    return ORBX_OK;
}

int orbx_capacity(const orbx_handle* h, int rows, int cols)
{
    if (!h) return -1;
    orbx_handle* m = const_cast<orbx_handle*>(h);
    DeviceGuard guard(m->device);
    if (ensure_geometry(m, rows, cols) != ORBX_OK) return -1;
    return m->geom.out_per_frame;
}

orbx_status orbx_debug_launches(orbx_handle* h, int rows, int cols, int batch, int* counts, int n)
{
    if (!h || !counts || n < 1 || batch < 1) return ORBX_EINVAL;
    DeviceGuard guard(h->device);
    const orbx_status st = ensure_geometry(h, rows, cols);
    if (st != ORBX_OK) return st;
    const Geometry& g = h->geom;
    int fast = 0;
    for (int i = 0; i < g.fast_groups; ++i) fast += g.fast_cb[i + 1] > g.fast_cb[i];
    if (batch <= kLatencyMaxBatch) fast = std::min(fast, 1);   // launch_fast: one launch for small batches
    QtGroup grp[kQtMaxGroups];
    // the pyramid's launches each read one level (counts[4]: bit mask): one launch per level from the one
    // before it
    const bool fused = batch <= kLatencyMaxBatch && g.pyr_ngroups > 0;   // launch_pyramid's choice
    int srcmask = (1 << (g.nlevels - 1)) - 1;
    if (fused) {
        srcmask = 0;
        for (int i = 0; i < g.pyr_ngroups; ++i) srcmask |= 1 << g.pg[i].s;
    }
    const int c[5] = {fused ? g.pyr_ngroups : g.nlevels - 1, fast, qt_plan(g, batch, grp), 1, srcmask};
    for (int i = 0; i < n; ++i) counts[i] = i < 5 ? c[i] : 0;
    return ORBX_OK;
}

// Host-path copies between the pinned staging block and device memory as kernels on the extraction's own
// queue: an SDMA copy (hipMemcpy*Async) costs its own ~11 us for a 640x480 image plus ~11 us before the
// compute queue sees it has finished; a kernel reading or writing the mapped pinned block over PCIe needs
// neither.  Two (src, dst, 16-byte units) regions per launch.
__global__ __launch_bounds__(256) void k_host_copy(const uint4* __restrict__ s0, uint4* __restrict__ d0, size_t n0,
                                                   const uint4* __restrict__ s1, uint4* __restrict__ d1, size_t n1)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n0 + n1; i += stride) {
        if (i < n0) d0[i] = s0[i];
        else d1[i - n0] = s1[i - n0];
    }
}

orbx_status orbx_extract(orbx_handle* h, const uint8_t* img, int rows, int cols, size_t step, orbx_keypoint* kps,
                         int cap, uint8_t* desc, int* n_out)
{
    if (!h || !n_out) return ORBX_EINVAL;
    if (!img || rows <= 0 || cols <= 0) return ORBX_EMPTY;   // src/ORBextractor.cc:1252
    if (step < (size_t)cols || !kps || !desc || cap < 0) return ORBX_EINVAL;
    DeviceGuard guard(h->device);
    orbx_status st = ensure_geometry(h, rows, cols);
    if (st != ORBX_OK) return st;
    if ((st = ensure_batch(h, 1)) != ORBX_OK) return st;
    const int pitch = (cols + 63) & ~63;
    const size_t need = (size_t)pitch * rows;
    if (need > h->img_bytes) {
        if (!dalloc(h, h->d_img, need)) return ORBX_ENOMEM;
        h->img_bytes = need;
    }
    const int ocap = h->geom.out_per_frame;
    // device results [keypoints ocap][descriptors ocap x 32] mirror the pinned block from kp_off, and the
    // frame's count sits in the status block's second word: two D2H copies (status + count, results)
    const size_t kp_b = ((size_t)ocap * sizeof(orbx_keypoint) + 63) & ~(size_t)63;
    if (ocap > h->single_cap) {
        if (!dalloc(h, h->d_out, kp_b + (size_t)ocap * 32)) return ORBX_ENOMEM;
        h->single_cap = ocap;
    }
    // pinned staging: [image rows x pitch][status, count (16 bytes)][keypoints ocap][descriptors ocap x 32]
    const size_t img_b = need;   // pitch * rows, a multiple of 64
    const size_t kp_off = img_b + 64, ds_off = kp_off + kp_b;
    const size_t pin_need = ds_off + (size_t)ocap * 32;
    if (pin_need > h->pin_bytes) {   // retired, not freed (see orbx_handle::caps)
        if (h->h_pin) h->retired_pin.push_back(h->h_pin);
        h->h_pin = nullptr;
        const size_t want = std::max(pin_need, h->pin_bytes + h->pin_bytes / 2);
        h->pin_bytes = 0;
        if (hipHostMalloc((void**)&h->h_pin, want, hipHostMallocDefault) != hipSuccess) return ORBX_ENOMEM;
        h->pin_bytes = want;
    }
    for (int r = 0; r < rows; ++r) std::memcpy(h->h_pin + (size_t)r * pitch, img + (size_t)r * step, (size_t)cols);
    hipStream_t s = own_stream(h);
    order_after_last(h, s);
    FramePtrs P{h->d_img, need, pitch, h->d_pyr, (size_t)h->geom.pyr_bytes};
    int* phdr = (int*)(h->h_pin + img_b);   // [0] status, [1] count
    int* d_count = h->d_status + 1;
    orbx_keypoint* d_kps = (orbx_keypoint*)h->d_out;
    uint8_t* d_desc = h->d_out + kp_b;
    // H2D image, the kernels, then one round trip: status, count and the whole output capacity
    // a timed handle (orbx_set_timing) launches directly, recording the stage events
    const hipEvent_t* ev = h->timing ? next_stage_events(h) : nullptr;
    // the pinned block's device address (the same pointer under unified addressing)
    void* dpin = nullptr;
    if (hipHostGetDevicePointer(&dpin, h->h_pin, 0) != hipSuccess) dpin = nullptr;
    const bool kcopy = dpin != nullptr;   // else SDMA copies
    uint8_t* dp = (uint8_t*)dpin;
    const size_t out_b = kp_b + (size_t)ocap * 32;   // multiple of 32
    auto enqueue = [&]() {
        if (kcopy) {   // the image rows at the device pitch, so the copy is whole 16-byte units
            hipLaunchKernelGGL(k_host_copy, dim3(std::min<size_t>((need / 16 + 255) / 256, 1024)), dim3(256), 0, s,
                               (const uint4*)dp, (uint4*)h->d_img, need / 16, (const uint4*)nullptr, (uint4*)nullptr,
                               (size_t)0);
        } else {
            hipMemcpyAsync(h->d_img, h->h_pin, need, hipMemcpyHostToDevice, s);
        }
        enqueue_pipeline(h, P, 1, d_kps, d_desc, d_count, ocap, s, ev);
        if (kcopy) {   // status + count (the status block's first 16 bytes) and the whole output capacity
            hipLaunchKernelGGL(k_host_copy, dim3(std::min<size_t>((out_b / 16 + 1 + 255) / 256, 1024)), dim3(256), 0, s,
                               (const uint4*)h->d_status, (uint4*)(dp + img_b), (size_t)1, (const uint4*)h->d_out,
                               (uint4*)(dp + kp_off), out_b / 16);
        } else {
            hipMemcpyAsync(phdr, h->d_status, 2 * sizeof(int), hipMemcpyDeviceToHost, s);
            hipMemcpyAsync(h->h_pin + kp_off, h->d_out, out_b, hipMemcpyDeviceToHost, s);
        }
    };
    // Replayed as a hipGraph: one submission instead of ~17 (launch overhead is most of a 640x480 frame's
    // latency).  The graph is re-captured when any buffer or size it holds changes.
    const std::vector<const void*> key = {(const void*)h->h_pin, h->d_img, h->d_out, h->d_pyr, h->d_slots, h->d_cell_counts, h->d_spill,
                                          h->d_spill_node, h->d_qt_nodes, h->d_qt_out, h->d_qt_cnt, h->d_status, h->d_geom,
                                          h->d_cells, h->d_xtab, h->d_ytab, h->d_pyrbt, (const void*)(uintptr_t)rows,
                                          (const void*)(uintptr_t)cols, (const void*)(uintptr_t)ocap,
                                          (const void*)(uintptr_t)h->resize_mode, (const void*)(uintptr_t)h->blur_mode};
    bool launched = false;
    if (!ev && !h->graph_failed && !getenv("ORBX_NO_GRAPH")) {
        if (h->host_graph && h->graph_key != key) {
            hipGraphExecDestroy(h->host_graph);
            h->host_graph = nullptr;
        }
        if (!h->host_graph) {
            hipGraph_t graph = nullptr;
            bool ok = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess;
            if (ok) {
                enqueue();
                ok = hipStreamEndCapture(s, &graph) == hipSuccess && graph;
            }
            ok = ok && hipGraphInstantiate(&h->host_graph, graph, nullptr, nullptr, 0) == hipSuccess;
            if (graph) hipGraphDestroy(graph);
            if (!ok) {
                (void)hipGetLastError();
                h->host_graph = nullptr;
                h->graph_failed = true;   // direct launches from now on
            }
            h->graph_key = key;
        }
        launched = h->host_graph && hipGraphLaunch(h->host_graph, s) == hipSuccess;
    }
    if (!launched) enqueue();
    if (hipGetLastError() != hipSuccess) return ORBX_EDEVICE;
    h->last = P;
    h->last_batch = 1;
    std::fill(h->level_cached.begin(), h->level_cached.end(), false);
    if (hipStreamSynchronize(s) != hipSuccess) return ORBX_EDEVICE;
    h->done_pending = false;   // everything the handle queued has completed
    if (phdr[0] & kStatusCapOverflow) return ORBX_ENOSPC;
    if (phdr[0]) return ORBX_EDEVICE;
    const int n = phdr[1];
    if (n > cap) return ORBX_ENOSPC;
    if (n > 0) {
        std::memcpy(kps, h->h_pin + kp_off, sizeof(orbx_keypoint) * (size_t)n);
        std::memcpy(desc, h->h_pin + ds_off, (size_t)n * 32);
    }
    *n_out = n;
    return ORBX_OK;
}

orbx_status orbx_get_level(orbx_handle* h, int level, const uint8_t** data, int* rows, int* cols, size_t* step)
{
    if (!h || !h->geom_ok || h->last_batch <= 0 || level < 0 || level >= h->geom.nlevels) return ORBX_EINVAL;
    DeviceGuard guard(h->device);
    const LevelGeom& L = h->geom.lv[level];
    if (!h->level_cached[level]) {
        std::vector<uint8_t>& v = h->h_levels[level];
        v.resize((size_t)L.w * L.h);
        const uint8_t* src;
        size_t sp;
        if (level == 0) {
            src = h->last.in;
            sp = (size_t)h->last.in_pitch;
        } else {
            src = h->last.pyr + L.pyr_off;
            sp = (size_t)L.pitch;
        }
        order_after_last(h, own_stream(h));
        if (hipMemcpy2DAsync(v.data(), L.w, src, sp, L.w, L.h, hipMemcpyDeviceToHost, own_stream(h)) != hipSuccess ||
            hipStreamSynchronize(own_stream(h)) != hipSuccess)
            return ORBX_EDEVICE;
        h->level_cached[level] = true;
    }
    if (data) *data = h->h_levels[level].data();
    if (rows) *rows = L.h;
    if (cols) *cols = L.w;
    if (step) *step = (size_t)L.w;
    return ORBX_OK;
}

orbx_status orbx_extract_batch_device(orbx_handle* h, const uint8_t* d_imgs, int batch, int rows, int cols,
                                      size_t step, size_t frame_stride, orbx_keypoint* d_kps, uint8_t* d_desc,
                                      int* d_counts, int cap, void* stream)
{
    if (!h || !d_imgs || batch <= 0 || !d_kps || !d_desc || !d_counts || cap <= 0) return ORBX_EINVAL;
    if (step < (size_t)cols || (batch > 1 && frame_stride < step * (size_t)rows)) return ORBX_EINVAL;
    DeviceGuard guard(h->device);
    orbx_status st = ensure_geometry(h, rows, cols);
    if (st != ORBX_OK) return st;
    if ((st = ensure_batch(h, batch)) != ORBX_OK) return st;
    hipStream_t s = (hipStream_t)stream;   // taken literally: NULL is the HIP null stream
    order_after_last(h, s);
    FramePtrs P{d_imgs, frame_stride, (int)step, h->d_pyr, (size_t)h->geom.pyr_bytes};
    st = run_pipeline(h, P, batch, d_kps, d_desc, d_counts, cap, s);
    mark_last(h, s);
    return st;
}

orbx_status orbx_extract_stage_device(orbx_handle* h, int stage, const uint8_t* d_imgs, int batch, int rows, int cols,
                                      size_t step, size_t frame_stride, orbx_keypoint* d_kps, uint8_t* d_desc,
                                      int* d_counts, int cap, void* stream)
{
    if (!h || stage < 0 || stage > 3 || !d_imgs || batch <= 0 || !d_kps || !d_desc || !d_counts || cap <= 0)
        return ORBX_EINVAL;
    if (step < (size_t)cols || (batch > 1 && frame_stride < step * (size_t)rows)) return ORBX_EINVAL;
    DeviceGuard guard(h->device);
    orbx_status st;
    if (stage == 0) {   // sizes the geometry and workspace; later stages must match them
        if ((st = ensure_geometry(h, rows, cols)) != ORBX_OK) return st;
        if ((st = ensure_batch(h, batch)) != ORBX_OK) return st;
    } else if (!h->geom_ok || h->grows != rows || h->gcols != cols || batch > h->batch_cap) {
        return ORBX_EINVAL;
    }
    hipStream_t s = (hipStream_t)stream;
    const Geometry& g = h->geom;
    ExtractBufs b = bufs(h);
    FramePtrs P{d_imgs, frame_stride, (int)step, h->d_pyr, (size_t)g.pyr_bytes};
    hipEvent_t* tev = nullptr;   // a timed handle: this stage's (start, end) events
    if (h->timing) {
        if ((size_t)(h->sev_used + 1) * 2 > h->sev.size()) {
            const size_t old = h->sev.size();
            h->sev.resize(old + 2 * 64);
            h->sev_stage.resize(h->sev.size() / 2);
            for (size_t i = old; i < h->sev.size(); ++i) hipEventCreate(&h->sev[i]);
        }
        h->sev_stage[h->sev_used] = stage;
        tev = &h->sev[(size_t)(h->sev_used++) * 2];
    }
    // the previous batch's describe and any stereo search still reading its pyramids (the caller orders
    // the rest); before the start event, so the wait is not counted as pyramid time
    if (stage == 0) order_after_last(h, s);
    if (tev) hipEventRecord(tev[0], s);
    switch (stage) {
    case 0:
        hipMemsetAsync(d_counts, 0, sizeof(int) * batch, s);
        hipMemsetAsync(h->d_status, 0, sizeof(int), s);
        launch_pyramid(g, b, P, batch, s);
        break;
    case 1:
        launch_fast(g, b, P, batch, s);
        break;
    case 2:
        launch_quadtree(g, b, d_counts, batch, s);
        break;
    default:
        launch_describe(g, b, P, d_kps, d_desc, cap, batch, s);
        h->last = P;
        h->last_batch = batch;
        std::fill(h->level_cached.begin(), h->level_cached.end(), false);
        mark_last(h, s);
        break;
    }
    if (tev) hipEventRecord(tev[1], s);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbx_sync(orbx_handle* h, void* stream)
{
    if (!h) return ORBX_EINVAL;
    DeviceGuard guard(h->device);
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return ORBX_EDEVICE;
    if (!h->d_status) return ORBX_OK;
    return status_from_device(h, (hipStream_t)stream);
}

orbx_status orbx_set_timing(orbx_handle* h, int enable)
{
    if (!h) return ORBX_EINVAL;
    h->timing = enable != 0;
    h->ev_used = 0;   // (re)start accumulation
    h->sev_used = 0;
    return ORBX_OK;
}

orbx_status orbx_get_stage_times(orbx_handle* h, float* ms, int n)
{
    if (!h || !ms || (h->ev_used == 0 && h->sev_used == 0)) return ORBX_EINVAL;
    for (int i = 0; i < n && i < 4; ++i) ms[i] = 0.f;
    for (int c = 0; c < h->sev_used; ++c) {   // stage-split calls (their streams may differ)
        const hipEvent_t* e = &h->sev[(size_t)c * 2];
        float t = 0.f;
        if (hipEventSynchronize(e[1]) != hipSuccess) return ORBX_EDEVICE;
        hipEventElapsedTime(&t, e[0], e[1]);
        if (h->sev_stage[c] < n) ms[h->sev_stage[c]] += t;
    }
    if (h->ev_used > 0 && hipEventSynchronize(h->ev[(size_t)h->ev_used * 5 - 1]) != hipSuccess) return ORBX_EDEVICE;
    for (int c = 0; c < h->ev_used; ++c) {
        const hipEvent_t* e = &h->ev[(size_t)c * 5];
        for (int i = 0; i < n && i < 4; ++i) {
            float t = 0.f;
            hipEventElapsedTime(&t, e[i], e[i + 1]);
            ms[i] += t;
        }
    }
    return ORBX_OK;
}

orbx_status orbx_debug_pyramid(orbx_handle* h, int frame, uint8_t* out, size_t out_size)
{
    if (!h || !out || frame < 0 || frame >= h->last_batch) return ORBX_EINVAL;
    DeviceGuard guard(h->device);
    order_after_last(h, own_stream(h));
    size_t o = 0;
    for (int l = 0; l < h->geom.nlevels; ++l) {
        const LevelGeom& L = h->geom.lv[l];
        if (o + (size_t)L.w * L.h > out_size) return ORBX_ENOSPC;
        const uint8_t* src;
        size_t sp;
        if (l == 0) {
            src = h->last.in + (size_t)frame * h->last.in_fstride;
            sp = (size_t)h->last.in_pitch;
        } else {
            src = h->last.pyr + (size_t)frame * h->last.pyr_fstride + L.pyr_off;
            sp = (size_t)L.pitch;
        }
        hipMemcpy2DAsync(out + o, L.w, src, sp, L.w, L.h, hipMemcpyDeviceToHost, own_stream(h));
        o += (size_t)L.w * L.h;
    }
    return hipStreamSynchronize(own_stream(h)) == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbx_debug_candidates(orbx_handle* h, int frame, int level, int* xys, int cap, int* n)
{
    if (!h || !n || frame < 0 || frame >= h->last_batch || level < 0 || level >= h->geom.nlevels) return ORBX_EINVAL;
    DeviceGuard guard(h->device);
    order_after_last(h, own_stream(h));
    const Geometry& g = h->geom;
    std::vector<int> cnt(g.ncells);
    std::vector<uint32_t> sl(g.slots_per_frame);
    hipMemcpyAsync(cnt.data(), h->d_cell_counts + (size_t)frame * g.ncells, sizeof(int) * g.ncells,
                   hipMemcpyDeviceToHost, own_stream(h));
    hipMemcpyAsync(sl.data(), h->d_slots + (size_t)frame * g.slots_per_frame, sizeof(uint32_t) * g.slots_per_frame,
                   hipMemcpyDeviceToHost, own_stream(h));
    if (hipStreamSynchronize(own_stream(h)) != hipSuccess) return ORBX_EDEVICE;
    const LevelGeom& L = g.lv[level];
    // a cell's first slot: its own slot base if FAST wrote it directly (kCellDirect), else its wave's run
    // (the wave's first cell's slot base plus the wave's earlier cells' counts; orbx_kernels.hpp)
    const int cpw = fast_cells_per_wave(h->last_batch);
    int k = 0;
    uint32_t run = 0;
    for (int c = L.cell_begin; c < L.cell_begin + L.ncells; ++c) {
        const uint32_t raw = (uint32_t)cnt[c];
        const int n = (int)(raw & ~kCellDirect);
        if ((c - L.cell_begin) % cpw == 0) run = (uint32_t)h->cells[c].slot_base;
        const uint32_t a = (raw & kCellDirect) ? (uint32_t)h->cells[c].slot_base : run;
        run += (raw & kCellDirect) ? 0u : (uint32_t)n;
        for (int i = 0; i < n; ++i) {
            const uint32_t v = sl[a + i];
            if (k < cap && xys) {
                xys[3 * k] = (int)kp_x(v, (uint32_t)g.kp_xbits);
                xys[3 * k + 1] = (int)kp_y(v, (uint32_t)g.kp_xbits);
                xys[3 * k + 2] = (int)(v >> 24);
            }
            ++k;
        }
    }
    *n = k;
    return k > cap ? ORBX_ENOSPC : ORBX_OK;
}

}  // extern "C"

namespace {

// search limits of ComputeStereoMatches (src/Frame.cc:676-681, mb from :140) and the
// row-band half width that bounds every right keypoint's [floor(y-r), ceil(y+r)]
void stereo_limits(const orbx_handle* h, float bf, float fx, float* maxD, int* rband)
{
    const float mb = bf / fx;
    const float minZ = mb;
    *maxD = bf / minZ;
    float rmax = 0.f;
    for (int l = 0; l < h->tab.nlevels; ++l) rmax = std::max(rmax, 2.0f * h->tab.scale[l]);
    *rband = (int)std::ceil(rmax);
}

bool same_geometry(const orbx_handle* a, const orbx_handle* b)
{
    if (!a->geom_ok || !b->geom_ok || a->grows != b->grows || a->gcols != b->gcols) return false;
    if (a->tab.nlevels != b->tab.nlevels) return false;
    for (int l = 0; l < a->tab.nlevels; ++l)
        if (a->tab.scale[l] != b->tab.scale[l]) return false;
    return true;
}

}  // namespace

extern "C" {

orbx_status orbx_compute_stereo_matches(orbx_handle* left, orbx_handle* right, const orbx_keypoint* kps_l,
                                        const uint8_t* desc_l, int n_l, const orbx_keypoint* kps_r,
                                        const uint8_t* desc_r, int n_r, float bf, float fx, float* u_right,
                                        float* depth, int* n_good)
{
    if (!left || !right || !n_good || n_l < 0 || n_r < 0) return ORBX_EINVAL;
    *n_good = 0;
    if (n_l == 0) return ORBX_OK;   // Frame ctor returns before ComputeStereoMatches (src/Frame.cc:106-107)
    if (!kps_l || !desc_l || !u_right || !depth || (n_r > 0 && (!kps_r || !desc_r))) return ORBX_EINVAL;
    if (left->device != right->device || !same_geometry(left, right) || left->last_batch <= 0 ||
        right->last_batch <= 0 || !(fx != 0.f) || !(bf != 0.f))
        return ORBX_EINVAL;
    const int cap = std::max(n_l, n_r);
    if (cap > 32767) return ORBX_EINVAL;
    HostCall c(left->device);
    const int hmeta[5] = {n_l, n_r, 0, 1, 0};   // counts[2], fl, fr, ngood
    const size_t om = c.in(hmeta, sizeof(hmeta));
    // the kernels address frame f's keypoints at kps + f * cap: left rows at 0, right rows at cap
    const size_t ok = c.in(nullptr, sizeof(orbx_keypoint) * 2 * (size_t)cap);
    const size_t od = c.in(nullptr, (size_t)64 * cap);
    const size_t ou = c.out(sizeof(float) * (size_t)cap), oz = c.out(sizeof(float) * (size_t)cap);
    const size_t osad = c.out(sizeof(int) * (size_t)cap);
    orbx_status st = c.prepare();
    if (st != ORBX_OK) return st;
    uint8_t* hk = c.host(ok);
    uint8_t* hd = c.host(od);
    if (!hk || !hd) return ORBX_ENOMEM;
    std::memcpy(hk, kps_l, sizeof(orbx_keypoint) * (size_t)n_l);
    if (n_r > 0) std::memcpy(hk + sizeof(orbx_keypoint) * (size_t)cap, kps_r, sizeof(orbx_keypoint) * (size_t)n_r);
    std::memcpy(hd, desc_l, (size_t)32 * n_l);
    if (n_r > 0) std::memcpy(hd + (size_t)32 * cap, desc_r, (size_t)32 * n_r);
    if ((st = c.upload()) != ORBX_OK) return st;
    // the two images' pyramids: written by each handle's last extraction, on whatever stream it ran
    order_after_last(left, c.stream());
    if (right != left) order_after_last(right, c.stream());
    // single images: frame strides 0, so frame indices 0 / 1 both address the handle's image
    FramePtrs PL = left->last, PR = right->last;
    PL.in_fstride = PL.pyr_fstride = 0;
    PR.in_fstride = PR.pyr_fstride = 0;
    float maxD;
    int rband;
    stereo_limits(left, bf, fx, &maxD, &rband);
    int* meta = c.dev_as<int>(om);
    launch_stereo(left->geom, left->d_geom, PL, PR, c.dev_as<orbx_keypoint>(ok), c.dev(od), meta, cap, meta + 2,
                  meta + 3, 1, bf, maxD, rband, c.dev_as<float>(ou), c.dev_as<float>(oz), c.dev_as<int>(osad),
                  meta + 4, c.stream());
    if (hipGetLastError() != hipSuccess) return ORBX_EDEVICE;
    int ng = 0;
    c.fetch(ou, u_right, sizeof(float) * (size_t)n_l);
    c.fetch(oz, depth, sizeof(float) * (size_t)n_l);
    c.fetch(om + 16, &ng, sizeof(int));
    if ((st = c.finish()) != ORBX_OK) return st;
    *n_good = ng;
    return ORBX_OK;
}

orbx_status orbx_stereo_batch_device(orbx_handle* h, const orbx_keypoint* d_kps, const uint8_t* d_desc,
                                     const int* d_counts, int cap, const int* d_left, const int* d_right, int npairs,
                                     float bf, float fx, float* d_u_right, float* d_depth, int* d_n_good,
                                     void* stream)
{
    if (!h || !d_kps || !d_desc || !d_counts || cap <= 0 || cap > 32767 || npairs < 0 || !d_left || !d_right ||
        !d_u_right || !d_depth || !d_n_good || !(fx != 0.f) || !(bf != 0.f))
        return ORBX_EINVAL;
    if (!h->geom_ok || h->last_batch <= 0) return ORBX_EINVAL;
    if (npairs == 0) return ORBX_OK;
    DeviceGuard guard(h->device);
    hipStream_t s = (hipStream_t)stream;
    order_after_last(h, s);   // the batch's pyramids
    int* dsad = nullptr;
    if (hipMallocAsync((void**)&dsad, sizeof(int) * (size_t)npairs * cap, s) != hipSuccess) return ORBX_ENOMEM;
    float maxD;
    int rband;
    stereo_limits(h, bf, fx, &maxD, &rband);
    launch_stereo(h->geom, h->d_geom, h->last, h->last, d_kps, d_desc, d_counts, cap, d_left, d_right, npairs, bf,
                  maxD, rband, d_u_right, d_depth, dsad, d_n_good, s);
    hipFreeAsync(dsad, s);
    // the stereo kernels read the handle's pyramid workspace: the next extraction, which rewrites it, waits
    // for them (s already waited for the extraction, so this event covers both)
    mark_last(h, s);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbm_bow_search_device(int mode, const orbm_bow_view* d_view1, const orbm_bow_view* d_view2,
                                   const orbm_triang_params* d_tp, int npairs, int max_nodes1, float nnratio,
                                   int check_ori, int* d_match, int match_stride, int* d_nmatches, void* stream)
{
    if (mode < ORBM_BOW_KF_F || mode > ORBM_TRIANGULATION || !d_view1 || !d_view2 || npairs < 0 ||
        max_nodes1 < 0 || !d_match || match_stride <= 0 || !d_nmatches || (mode == ORBM_TRIANGULATION && !d_tp))
        return ORBX_EINVAL;
    if (npairs == 0) return ORBX_OK;
    hipStream_t s = (hipStream_t)stream;
    int* bins = nullptr;
    if (hipMallocAsync((void**)&bins, sizeof(int) * (size_t)npairs * match_stride, s) != hipSuccess)
        return ORBX_ENOMEM;
    launch_bow(mode, d_view1, d_view2, d_tp, npairs, max_nodes1, nnratio, check_ori, d_match, bins, match_stride,
               d_nmatches, s);
    hipFreeAsync(bins, s);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

}  // extern "C"

namespace {

bool bow_view_ok(const orbm_bow_view* v)
{
    if (!v || v->n < 0 || v->fv_nnodes < 0 || v->n > ORBM_MAX_FEATURES) return false;
    if (v->n > 0 && (!v->kps || !v->desc)) return false;
    if (v->fv_nnodes > 0 && (!v->fv_node || !v->fv_ptr || !v->fv_idx)) return false;
    for (int k = 0; k < v->fv_nnodes; ++k) {
        if (v->fv_ptr[k] > v->fv_ptr[k + 1] || (k > 0 && v->fv_node[k] <= v->fv_node[k - 1])) return false;
        for (int j = v->fv_ptr[k]; j < v->fv_ptr[k + 1]; ++j)
            if (v->fv_idx[j] < 0 || v->fv_idx[j] >= v->n) return false;
    }
    return v->fv_nnodes == 0 || v->fv_ptr[0] == 0;
}

// offsets of one staged view (device pointers are patched in after the buffers are sized)
struct BowOffs {
    size_t kps, desc, mp, ur, node, ptr, idx;
    bool has_mp, has_ur;
};

BowOffs bow_stage(HostCall& c, const orbm_bow_view* v)
{
    BowOffs o;
    o.kps = c.in(v->kps, sizeof(orbx_keypoint) * (size_t)v->n);
    o.desc = c.in(v->desc, (size_t)32 * v->n);
    o.has_mp = v->has_mp != nullptr;
    o.has_ur = v->u_right != nullptr;
    o.mp = o.has_mp ? c.in(v->has_mp, (size_t)v->n) : 0;
    o.ur = o.has_ur ? c.in(v->u_right, sizeof(float) * (size_t)v->n) : 0;
    o.node = c.in(v->fv_node, sizeof(int32_t) * (size_t)v->fv_nnodes);
    o.ptr = c.in(v->fv_ptr, sizeof(int32_t) * ((size_t)v->fv_nnodes + 1));
    o.idx = c.in(v->fv_idx, sizeof(int32_t) * (size_t)(v->fv_nnodes ? v->fv_ptr[v->fv_nnodes] : 0));
    return o;
}

orbm_bow_view bow_device_view(uint8_t* base, const BowOffs& o, const orbm_bow_view* v)
{
    orbm_bow_view d = *v;
    d.kps = (const orbx_keypoint*)(base + o.kps);
    d.desc = base + o.desc;
    d.has_mp = o.has_mp ? base + o.mp : nullptr;
    d.u_right = o.has_ur ? (const float*)(base + o.ur) : nullptr;
    d.fv_node = (const int32_t*)(base + o.node);
    d.fv_ptr = (const int32_t*)(base + o.ptr);
    d.fv_idx = (const int32_t*)(base + o.idx);
    return d;
}

}  // namespace

extern "C" {

orbx_status orbm_bow_search(int device, int mode, const orbm_bow_view* view1, const orbm_bow_view* view2,
                            const orbm_triang_params* tp, float nnratio, int check_ori, int* match, int* nmatches)
{
    if (mode < ORBM_BOW_KF_F || mode > ORBM_TRIANGULATION || !bow_view_ok(view1) || !bow_view_ok(view2) ||
        !nmatches || (mode == ORBM_TRIANGULATION && !tp))
        return ORBX_EINVAL;
    const int nout = mode == ORBM_BOW_KF_F ? view2->n : view1->n;
    if (nout > 0 && !match) return ORBX_EINVAL;
    *nmatches = 0;
    if (nout == 0) return ORBX_OK;
    HostCall c(device);
    // the two device view structs (+ tp) first: they are patched after the buffers are sized
    const size_t ov = c.in(nullptr, 2 * sizeof(orbm_bow_view) + sizeof(orbm_triang_params));
    const BowOffs o1 = bow_stage(c, view1), o2 = bow_stage(c, view2);
    const size_t om = c.out(sizeof(int) * ((size_t)nout + 1));
    orbx_status rc = c.prepare();
    if (rc != ORBX_OK) return rc;
    uint8_t* base = c.dev(0);
    orbm_bow_view dv[2] = {bow_device_view(base, o1, view1), bow_device_view(base, o2, view2)};
    std::memcpy(c.host(ov), dv, sizeof(dv));
    if (tp) std::memcpy(c.host(ov) + sizeof(dv), tp, sizeof(*tp));
    if ((rc = c.upload()) != ORBX_OK) return rc;
    const orbm_bow_view* d1 = c.dev_as<const orbm_bow_view>(ov);
    const orbm_triang_params* dtp = (const orbm_triang_params*)(c.dev(ov) + sizeof(dv));
    int* dm = c.dev_as<int>(om);
    rc = orbm_bow_search_device(mode, d1, d1 + 1, dtp, 1, view1->fv_nnodes, nnratio, check_ori, dm + 1, nout, dm,
                                c.stream());
    if (rc != ORBX_OK) return rc;
    c.fetch(om + sizeof(int), match, sizeof(int) * (size_t)nout);
    c.fetch(om, nmatches, sizeof(int));
    return c.finish();
}

orbx_status orbm_search_by_projection_device(const orbx_keypoint* d_kps, const uint8_t* d_desc, const float* d_uright,
                                             const uint8_t* d_claimed, const int* d_counts, int nframes, int cap,
                                             const orbm_proj_point* d_pts, const uint8_t* d_pdesc, const int* d_npts,
                                             int pcap, const orbm_proj_params* params, int* d_match,
                                             int* d_nmatches, void* stream)
{
    if (!d_kps || !d_desc || !d_uright || !d_claimed || !d_counts || nframes < 0 || cap <= 0 || cap > ORBM_MAX_FEATURES ||
        !d_pts || !d_pdesc || !d_npts || pcap <= 0 || !params || !d_match || !d_nmatches)
        return ORBX_EINVAL;
    if (nframes == 0) return ORBX_OK;
    hipStream_t s = (hipStream_t)stream;
    void* scratch = nullptr;
    if (hipMallocAsync(&scratch, proj_scratch_bytes(nframes, cap, pcap), s) != hipSuccess) return ORBX_ENOMEM;
    launch_proj(d_kps, d_desc, d_uright, d_claimed, d_counts, nframes, cap, d_pts, d_pdesc, d_npts, pcap, *params,
                scratch, d_match, d_nmatches, s);
    hipFreeAsync(scratch, s);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbm_search_by_projection(int device, const orbx_keypoint* kps, const uint8_t* desc, const float* uright,
                                      const uint8_t* claimed, int n, const orbm_proj_point* pts, const uint8_t* pdesc,
                                      int np, const orbm_proj_params* params, int* match, int* nmatches)
{
    if (n < 0 || n > ORBM_MAX_FEATURES || np < 0 || !params || !nmatches) return ORBX_EINVAL;
    *nmatches = 0;
    if (n == 0) return ORBX_OK;
    if (!kps || !desc || !uright || !claimed || !match || (np > 0 && (!pts || !pdesc))) return ORBX_EINVAL;
    for (int i = 0; i < np; ++i)
        if ((pts[i].flags & 1) && (pts[i].level < 0 || pts[i].level >= 16)) return ORBX_EINVAL;
    for (int i = 0; i < n; ++i) match[i] = -1;
    if (np == 0) return ORBX_OK;
    HostCall c(device);
    const int cn[2] = {n, np};
    const size_t ocn = c.in(cn, sizeof(cn));
    const size_t ok = c.in(kps, sizeof(orbx_keypoint) * (size_t)n);
    const size_t od = c.in(desc, (size_t)32 * n);
    const size_t ou = c.in(uright, sizeof(float) * (size_t)n);
    const size_t oc = c.in(claimed, (size_t)n);
    const size_t op = c.in(pts, sizeof(orbm_proj_point) * (size_t)np);
    const size_t opd = c.in(pdesc, (size_t)32 * np);
    const size_t om = c.out(sizeof(int) * ((size_t)n + 1));
    orbx_status rc = c.prepare();
    if (rc == ORBX_OK) rc = c.upload();
    if (rc != ORBX_OK) return rc;
    int* dm = c.dev_as<int>(om);
    const int* dcn = c.dev_as<const int>(ocn);
    rc = orbm_search_by_projection_device(c.dev_as<const orbx_keypoint>(ok), c.dev(od), c.dev_as<const float>(ou),
                                          c.dev(oc), dcn, 1, n, c.dev_as<const orbm_proj_point>(op), c.dev(opd),
                                          dcn + 1, np, params, dm + 1, dm, c.stream());
    if (rc != ORBX_OK) return rc;
    c.fetch(om + sizeof(int), match, sizeof(int) * (size_t)n);
    c.fetch(om, nmatches, sizeof(int));
    return c.finish();
}

orbx_status orbm_project_search_device(int mode, const orbx_keypoint* d_kps, const uint8_t* d_desc,
                                       const float* d_uright, const uint8_t* d_claimed, const int* d_counts,
                                       int nframes, int cap, const float* d_pose, const orbm_map_point* d_pts,
                                       const uint8_t* d_pdesc, const int* d_npts, int pcap,
                                       const orbm_pose_params* params, int* d_match, int* d_nmatches, void* stream)
{
    if (mode < ORBM_PROJ_LAST_FRAME || mode > ORBM_FUSE_SIM3 || !d_kps || !d_desc || !d_uright || !d_claimed ||
        !d_counts || nframes < 0 || cap <= 0 || cap > ORBM_MAX_FEATURES || !d_pose || !d_pts || !d_pdesc || !d_npts ||
        pcap <= 0 || !params || !d_match || !d_nmatches || params->nlevels < 1 || params->nlevels > 16)
        return ORBX_EINVAL;
    if (nframes == 0) return ORBX_OK;
    hipStream_t s = (hipStream_t)stream;
    void* scratch = nullptr;
    if (hipMallocAsync(&scratch, pose_scratch_bytes(nframes, cap, pcap), s) != hipSuccess) return ORBX_ENOMEM;
    launch_pose_search(mode, d_kps, d_desc, d_uright, d_claimed, d_counts, nframes, cap, d_pose, d_pts, d_pdesc,
                       d_npts, pcap, *params, scratch, d_match, d_nmatches, s);
    hipFreeAsync(scratch, s);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbm_project_search(int device, int mode, const orbx_keypoint* kps, const uint8_t* desc,
                                const float* uright, const uint8_t* claimed, int n, const float* pose,
                                const orbm_map_point* pts, const uint8_t* pdesc, int np,
                                const orbm_pose_params* params, int* match, int* nmatches)
{
    if (mode < ORBM_PROJ_LAST_FRAME || mode > ORBM_FUSE_SIM3 || n < 0 || n > ORBM_MAX_FEATURES || np < 0 || !params ||
        !nmatches || !pose || params->nlevels < 1 || params->nlevels > 16)
        return ORBX_EINVAL;
    const bool search = mode <= ORBM_PROJ_SIM3;
    const int nout = search ? n : np;
    *nmatches = 0;
    if (nout > 0 && !match) return ORBX_EINVAL;
    if ((n > 0 && (!kps || !desc || !uright || (search && !claimed))) || (np > 0 && (!pts || !pdesc)))
        return ORBX_EINVAL;
    for (int i = 0; i < n; ++i)
        if (kps[i].octave < 0 || kps[i].octave >= 16) return ORBX_EINVAL;
    if (mode == ORBM_PROJ_LAST_FRAME)
        for (int i = 0; i < np; ++i)
            if ((pts[i].flags & 1) && (pts[i].octave < 0 || pts[i].octave >= 16)) return ORBX_EINVAL;
    for (int i = 0; i < nout; ++i) match[i] = -1;
    if (n == 0 || np == 0) return ORBX_OK;
    HostCall c(device);
    const int cn[2] = {n, np};
    const size_t ocn = c.in(cn, sizeof(cn));
    const size_t opo = c.in(pose, sizeof(float) * 24);
    const size_t ok = c.in(kps, sizeof(orbx_keypoint) * (size_t)n);
    const size_t od = c.in(desc, (size_t)32 * n);
    const size_t ou = c.in(uright, sizeof(float) * (size_t)n);
    const size_t oc = c.in(search ? claimed : nullptr, (size_t)n);
    const size_t op = c.in(pts, sizeof(orbm_map_point) * (size_t)np);
    const size_t opd = c.in(pdesc, (size_t)32 * np);
    const size_t om = c.out(sizeof(int) * ((size_t)nout + 1));
    orbx_status rc = c.prepare();
    if (rc == ORBX_OK) rc = c.upload();
    if (rc != ORBX_OK) return rc;
    int* dm = c.dev_as<int>(om);
    const int* dcn = c.dev_as<const int>(ocn);
    rc = orbm_project_search_device(mode, c.dev_as<const orbx_keypoint>(ok), c.dev(od), c.dev_as<const float>(ou),
                                    c.dev(oc), dcn, 1, n, c.dev_as<const float>(opo),
                                    c.dev_as<const orbm_map_point>(op), c.dev(opd), dcn + 1, np, params, dm + 1, dm,
                                    c.stream());
    if (rc != ORBX_OK) return rc;
    c.fetch(om + sizeof(int), match, sizeof(int) * (size_t)nout);
    c.fetch(om, nmatches, sizeof(int));
    return c.finish();
}

orbx_status orbx_ingest_batch_device(const uint8_t* d_src, int batch, int rows, int cols, int channels, int rgb,
                                     size_t src_step, size_t src_frame_stride, const float* d_map_x,
                                     const float* d_map_y, int nmaps, int dst_rows, int dst_cols, uint8_t* d_dst,
                                     size_t dst_step, size_t dst_frame_stride, void* stream)
{
    if (!d_src || !d_dst || batch < 0 || rows <= 0 || cols <= 0 || (channels != 1 && channels != 3 && channels != 4) ||
        src_step < (size_t)cols * channels || dst_rows <= 0 || dst_cols <= 0 || dst_step < (size_t)dst_cols ||
        (!d_map_x) != (!d_map_y) || rows > 32767 || cols > 32767)
        return ORBX_EINVAL;
    if (d_map_x && nmaps <= 0) return ORBX_EINVAL;
    if (!d_map_x && (dst_rows != rows || dst_cols != cols)) return ORBX_EINVAL;
    if (batch > 1 && (src_frame_stride < src_step * rows || dst_frame_stride < dst_step * dst_rows))
        return ORBX_EINVAL;
    if (batch == 0) return ORBX_OK;
    launch_ingest(d_src, batch, rows, cols, channels, rgb ? 1 : 0, src_step, src_frame_stride, d_map_x, d_map_y,
                  d_map_x ? nmaps : 1, dst_rows, dst_cols, d_dst, dst_step, dst_frame_stride, (hipStream_t)stream);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbx_depth_batch_device(const void* d_src, int depth_type, int batch, int rows, int cols,
                                    size_t src_step, size_t src_frame_stride, float factor, float* d_dst,
                                    size_t dst_step, size_t dst_frame_stride, void* stream)
{
    const size_t esz = depth_type == 0 ? 2 : 4;
    if (!d_src || !d_dst || (depth_type != 0 && depth_type != 1) || batch < 0 || rows <= 0 || cols <= 0 ||
        src_step < esz * cols || dst_step < 4 * (size_t)cols || src_step % esz || dst_step % 4 ||
        (batch > 1 && (src_frame_stride < src_step * rows || dst_frame_stride < dst_step * rows)))
        return ORBX_EINVAL;
    if (batch == 0) return ORBX_OK;
    launch_depth(d_src, depth_type, batch, rows, cols, src_step, src_frame_stride, factor, d_dst, dst_step,
                 dst_frame_stride, (hipStream_t)stream);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbm_best2_csr_device(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, const int* d_cand_ptr,
                                  const int* d_cand_idx, int tie_mode, int* d_best_idx, int* d_best, int* d_second,
                                  void* stream)
{
    if (nq < 0 || nt < 0 || (tie_mode != ORBM_TIE_FIRST && tie_mode != ORBM_TIE_LAST)) return ORBX_EINVAL;
    if (nq == 0) return ORBX_OK;
    if (!d_q || !d_cand_ptr || !d_best_idx || !d_best || !d_second || (nt > 0 && (!d_t || !d_cand_idx)))
        return ORBX_EINVAL;
    launch_best2_csr(d_q, nq, d_t, d_cand_ptr, d_cand_idx, tie_mode == ORBM_TIE_LAST, d_best_idx, d_best, d_second,
                     (hipStream_t)stream);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbm_best2_csr(int device, const uint8_t* q, int nq, const uint8_t* t, int nt, const int* cand_ptr,
                           const int* cand_idx, int tie_mode, int* best_idx, int* best, int* second)
{
    if (nq < 0 || nt < 0 || (tie_mode != ORBM_TIE_FIRST && tie_mode != ORBM_TIE_LAST)) return ORBX_EINVAL;
    if (nq == 0) return ORBX_OK;
    if (!q || !cand_ptr || !best_idx || !best || !second) return ORBX_EINVAL;
    const int ncand = cand_ptr[nq];
    if (cand_ptr[0] != 0 || ncand < 0 || (ncand > 0 && (!cand_idx || !t))) return ORBX_EINVAL;
    for (int i = 0; i < nq; ++i)
        if (cand_ptr[i + 1] < cand_ptr[i]) return ORBX_EINVAL;
    for (int k = 0; k < ncand; ++k)
        if (cand_idx[k] < 0 || cand_idx[k] >= nt) return ORBX_EINVAL;
    HostCall c(device);
    const size_t oq = c.in(q, (size_t)32 * nq);
    const size_t ot = c.in(t, (size_t)32 * nt);
    const size_t op = c.in(cand_ptr, sizeof(int) * ((size_t)nq + 1));
    const size_t oi = c.in(cand_idx, sizeof(int) * (size_t)ncand);
    const size_t oo = c.out(sizeof(int) * 3 * (size_t)nq);
    orbx_status rc = c.prepare();
    if (rc == ORBX_OK) rc = c.upload();
    if (rc != ORBX_OK) return rc;
    int* o = c.dev_as<int>(oo);
    rc = orbm_best2_csr_device(c.dev(oq), nq, c.dev(ot), nt, c.dev_as<const int>(op), c.dev_as<const int>(oi),
                               tie_mode, o, o + nq, o + 2 * nq, c.stream());
    if (rc != ORBX_OK) return rc;
    c.fetch(oo, best_idx, sizeof(int) * (size_t)nq);
    c.fetch(oo + sizeof(int) * (size_t)nq, best, sizeof(int) * (size_t)nq);
    c.fetch(oo + sizeof(int) * 2 * (size_t)nq, second, sizeof(int) * (size_t)nq);
    return c.finish();
}

orbx_status orbm_stereo_band_device(const orbx_keypoint* d_kps, const uint8_t* d_desc, const int* d_counts, int cap,
                                    const int* d_left, const int* d_right, int npairs, int rows, const float* scale,
                                    int nlevels, float min_d, float max_d, int* d_best_idx, int* d_best_dist,
                                    void* stream)
{
    if (npairs < 0 || cap < 1 || cap > 65535 || rows < 1 || nlevels < 1 || nlevels > kStMaxLevels || !scale)
        return ORBX_EINVAL;
    if (npairs == 0) return ORBX_OK;
    if (!d_kps || !d_desc || !d_counts || !d_left || !d_right || !d_best_idx || !d_best_dist) return ORBX_EINVAL;
    if (stereo_band_smem(rows, cap) > 160 * 1024) return ORBX_ENOSPC;
    StBandArgs a{};
    float rmax = 0.f;
    for (int l = 0; l < kStMaxLevels; ++l) {
        a.scale[l] = scale[std::min(l, nlevels - 1)];
        if (l < nlevels) rmax = std::max(rmax, 2.0f * scale[l]);
    }
    a.nlevels = nlevels;
    a.rows = rows;
    a.rband = (int)std::ceil(rmax);
    a.minD = min_d;
    a.maxD = max_d;
    launch_stereo_band(a, d_kps, d_desc, d_counts, cap, d_left, d_right, npairs, d_best_idx, d_best_dist,
                       (hipStream_t)stream);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbm_stereo_band(int device, const orbx_keypoint* kps_l, const uint8_t* desc_l, int n_l,
                             const orbx_keypoint* kps_r, const uint8_t* desc_r, int n_r, int rows, const float* scale,
                             int nlevels, float min_d, float max_d, int* best_idx, int* best_dist)
{
    if (n_l < 0 || n_r < 0 || n_l > 65535 || n_r > 65535 || rows < 1 || nlevels < 1 || nlevels > kStMaxLevels ||
        !scale)
        return ORBX_EINVAL;
    if (n_l == 0) return ORBX_OK;
    if (!kps_l || !desc_l || !best_idx || !best_dist || (n_r > 0 && (!kps_r || !desc_r))) return ORBX_EINVAL;
    for (int i = 0; i < n_r; ++i)
        if (kps_r[i].octave < 0 || kps_r[i].octave >= nlevels) return ORBX_EINVAL;
    const int cap = std::max(n_l, n_r);
    if (stereo_band_smem(rows, cap) > 160 * 1024) return ORBX_ENOSPC;
    HostCall c(device);
    const int meta[4] = {n_l, n_r, 0, 1};   // counts[2], left frame, right frame
    const size_t om = c.in(meta, sizeof(meta));
    const size_t ok = c.in(nullptr, sizeof(orbx_keypoint) * 2 * (size_t)cap);   // frame f at kps + f * cap
    const size_t od = c.in(nullptr, (size_t)64 * cap);
    const size_t oo = c.out(sizeof(int) * 2 * (size_t)cap);
    orbx_status rc = c.prepare();
    if (rc != ORBX_OK) return rc;
    uint8_t* hk = c.host(ok);
    uint8_t* hd = c.host(od);
    if (!hk || !hd) return ORBX_ENOMEM;
    std::memcpy(hk, kps_l, sizeof(orbx_keypoint) * (size_t)n_l);
    if (n_r) std::memcpy(hk + sizeof(orbx_keypoint) * (size_t)cap, kps_r, sizeof(orbx_keypoint) * (size_t)n_r);
    std::memcpy(hd, desc_l, (size_t)32 * n_l);
    if (n_r) std::memcpy(hd + (size_t)32 * cap, desc_r, (size_t)32 * n_r);
    if ((rc = c.upload()) != ORBX_OK) return rc;
    const int* m = c.dev_as<const int>(om);
    int* o = c.dev_as<int>(oo);
    rc = orbm_stereo_band_device(c.dev_as<const orbx_keypoint>(ok), c.dev(od), m, cap, m + 2, m + 3, 1, rows, scale,
                                 nlevels, min_d, max_d, o, o + cap, c.stream());
    if (rc != ORBX_OK) return rc;
    c.fetch(oo, best_idx, sizeof(int) * (size_t)n_l);
    c.fetch(oo + sizeof(int) * (size_t)cap, best_dist, sizeof(int) * (size_t)n_l);
    return c.finish();
}

int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b)
{
    int d = 0;
    for (int i = 0; i < 4; ++i) {
        uint64_t x, y;
        std::memcpy(&x, a + 8 * i, 8);
        std::memcpy(&y, b + 8 * i, 8);
        d += __builtin_popcountll(x ^ y);
    }
    return d;
}

orbx_status orbm_allpairs_device(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int mode, int* d_best_idx,
                                 int* d_best, int* d_second, uint16_t* d_full, void* stream)
{
    if (!d_q || !d_t || nq < 0 || nt < 0) return ORBX_EINVAL;
    if (nq == 0 || nt == 0) return ORBX_OK;
    hipStream_t s = (hipStream_t)stream;
    if (mode == ORBM_TOP2) {
        if (!d_best_idx || !d_best || !d_second) return ORBX_EINVAL;
        int nsplit = std::max(1, std::min(64, (256 * 4) / std::max(1, (nq + 255) / 256)));
        nsplit = std::min(nsplit, (nt + 255) / 256);
        int* part = nullptr;
        if (hipMallocAsync((void**)&part, sizeof(int) * 3 * (size_t)nq * nsplit, s) != hipSuccess) return ORBX_ENOMEM;
        launch_allpairs_top2(d_q, nq, d_t, nt, d_best_idx, d_best, d_second, part, nsplit, s);
        hipFreeAsync(part, s);
    } else if (mode == ORBM_FULL_U16) {
        if (!d_full) return ORBX_EINVAL;
        launch_allpairs_full(d_q, nq, d_t, nt, d_full, s);
    } else {
        return ORBX_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbm_allpairs(int device, const uint8_t* q, int nq, const uint8_t* t, int nt, int mode, int* best_idx,
                          int* best, int* second, uint16_t* full)
{
    if (nq < 0 || nt < 0 || (mode != ORBM_TOP2 && mode != ORBM_FULL_U16)) return ORBX_EINVAL;
    if (nq == 0) return ORBX_OK;
    if (!q || (nt > 0 && !t)) return ORBX_EINVAL;
    if (mode == ORBM_TOP2 && (!best_idx || !best || !second)) return ORBX_EINVAL;
    if (mode == ORBM_FULL_U16 && !full) return ORBX_EINVAL;
    if (nt == 0) {
        if (mode == ORBM_TOP2)
            for (int i = 0; i < nq; ++i) {
                best_idx[i] = -1;
                best[i] = second[i] = 256;
            }
        return ORBX_OK;
    }
    HostCall c(device);
    const size_t oq = c.in(q, (size_t)32 * nq);
    const size_t ot = c.in(t, (size_t)32 * nt);
    const size_t out_bytes = mode == ORBM_TOP2 ? sizeof(int) * 3 * (size_t)nq : sizeof(uint16_t) * (size_t)nq * nt;
    const size_t oo = c.out(out_bytes);
    orbx_status rc = c.prepare();
    if (rc == ORBX_OK) rc = c.upload();
    if (rc != ORBX_OK) return rc;
    int* o = c.dev_as<int>(oo);
    rc = orbm_allpairs_device(c.dev(oq), nq, c.dev(ot), nt, mode, o, o + nq, o + 2 * nq, (uint16_t*)o, c.stream());
    if (rc != ORBX_OK) return rc;
    if (mode == ORBM_TOP2) {
        c.fetch(oo, best_idx, sizeof(int) * (size_t)nq);
        c.fetch(oo + sizeof(int) * (size_t)nq, best, sizeof(int) * (size_t)nq);
        c.fetch(oo + sizeof(int) * 2 * (size_t)nq, second, sizeof(int) * (size_t)nq);
    } else {
        c.fetch(oo, full, out_bytes);
    }
    return c.finish();
}

orbx_status orbm_search_for_initialization_device(const orbx_keypoint* d_kps, const uint8_t* d_desc,
                                                  const int* d_counts, int nframes, int cap, const int* d_pair_a,
                                                  const int* d_pair_b, int npairs, const orbm_grid* grid,
                                                  int window, float nnratio, int check_ori, float* d_prev_matched,
                                                  int* d_matches12, int* d_nmatches, void* stream)
{
    if (!d_kps || !d_desc || !d_counts || nframes <= 0 || cap <= 0 || cap > 32767 || npairs < 0 || !grid)
        return ORBX_EINVAL;
    if (npairs == 0) return ORBX_OK;
    if (!d_pair_a || !d_pair_b || !d_matches12 || !d_nmatches) return ORBX_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    void* scratch = nullptr;
    if (hipMallocAsync(&scratch, search_init_scratch_bytes(nframes, npairs, cap), s) != hipSuccess)
        return ORBX_ENOMEM;
    launch_search_init(d_kps, d_desc, d_counts, nframes, cap, d_pair_a, d_pair_b, npairs, *grid, window, nnratio,
                       check_ori, d_prev_matched, scratch, d_matches12, d_nmatches, s);
    hipFreeAsync(scratch, s);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

orbx_status orbm_search_init_batch_device(const orbx_keypoint* d_kps, const uint8_t* d_desc, const int* d_counts,
                                          int nframes, int cap, const int* d_pair_a, const int* d_pair_b, int npairs,
                                          int rows, int cols, int window, float nnratio, int check_ori,
                                          int* d_matches12, int* d_nmatches, void* stream)
{
    if (rows <= 0 || cols <= 0) return ORBX_EINVAL;
    // Frame::ComputeImageBounds without distortion (src/Frame.cc:614-620) and the grid scale (:127-128)
    const orbm_grid g{0.0f, 0.0f, 64.0f / ((float)cols - 0.0f), 48.0f / ((float)rows - 0.0f)};
    return orbm_search_for_initialization_device(d_kps, d_desc, d_counts, nframes, cap, d_pair_a, d_pair_b, npairs,
                                                 &g, window, nnratio, check_ori, nullptr, d_matches12, d_nmatches,
                                                 stream);
}

orbx_status orbm_search_for_initialization(int device, const orbx_keypoint* kps1, const uint8_t* desc1, int n1,
                                           const orbx_keypoint* kps2, const uint8_t* desc2, int n2,
                                           const orbm_grid* grid, float* prev_matched, int window, float nnratio,
                                           int check_ori, int* matches12, int* nmatches)
{
    if (n1 < 0 || n2 < 0 || n1 > 32767 || n2 > 32767 || !grid || !nmatches) return ORBX_EINVAL;
    *nmatches = 0;
    if (n1 == 0) return ORBX_OK;   // vnMatches12 is empty
    if (!kps1 || !desc1 || !prev_matched || !matches12 || (n2 > 0 && (!kps2 || !desc2))) return ORBX_EINVAL;
    // extractor order (ORBextractor::operator() concatenates the levels, src/ORBextractor.cc:1290-1333): the
    // device finds level 0 as a prefix
    for (int i = 1; i < n1; ++i)
        if (kps1[i].octave < kps1[i - 1].octave) return ORBX_EINVAL;
    for (int i = 1; i < n2; ++i)
        if (kps2[i].octave < kps2[i - 1].octave) return ORBX_EINVAL;
    for (int i = 0; i < n1; ++i) matches12[i] = -1;
    if (n2 == 0) return ORBX_OK;   // every GetFeaturesInArea is empty
    const int cap = std::max(n1, n2);
    HostCall c(device);
    const int meta[4] = {n1, n2, 0, 1};   // counts[2], pair (0, 1)
    const size_t om = c.in(meta, sizeof(meta));
    const size_t ok = c.in(nullptr, sizeof(orbx_keypoint) * 2 * (size_t)cap);   // frame f at kps + f * cap
    const size_t od = c.in(nullptr, (size_t)64 * cap);
    const size_t opv = c.in(prev_matched, sizeof(float) * 2 * (size_t)n1);
    const size_t ores = c.out(sizeof(int) * ((size_t)cap + 1));
    const size_t osc = c.out(search_init_scratch_bytes(2, 1, cap));
    orbx_status rc = c.prepare();
    if (rc != ORBX_OK) return rc;
    uint8_t* hk = c.host(ok);
    uint8_t* hd = c.host(od);
    if (!hk || !hd) return ORBX_ENOMEM;
    std::memcpy(hk, kps1, sizeof(orbx_keypoint) * (size_t)n1);
    std::memcpy(hk + sizeof(orbx_keypoint) * (size_t)cap, kps2, sizeof(orbx_keypoint) * (size_t)n2);
    std::memcpy(hd, desc1, (size_t)32 * n1);
    std::memcpy(hd + (size_t)32 * cap, desc2, (size_t)32 * n2);
    if ((rc = c.upload()) != ORBX_OK) return rc;
    const int* m = c.dev_as<const int>(om);
    int* res = c.dev_as<int>(ores);
    launch_search_init(c.dev_as<const orbx_keypoint>(ok), c.dev(od), m, 2, cap, m + 2, m + 3, 1, *grid, window,
                       nnratio, check_ori, c.dev_as<float>(opv), c.dev(osc), res + 1, res, c.stream());
    if (hipGetLastError() != hipSuccess) return ORBX_EDEVICE;
    c.fetch(ores + sizeof(int), matches12, sizeof(int) * (size_t)n1);
    c.fetch(ores, nmatches, sizeof(int));
    c.fetch(opv, prev_matched, sizeof(float) * 2 * (size_t)n1);
    return c.finish();
}

}  // extern "C"
