/*
 * orbref.c — CPU parity oracle (TEST INFRASTRUCTURE ONLY, see orbref.h).
 *
 * Every function names the reference file:line it restates.  Compiled with
 * -ffp-contract=off; the two FMAs that GCC -O3 -march=native forms in the
 * reference's BRIEF sampling (re-checked on this host's g++ 11)
 * are written out with fmaf().
 */
#include "orbref.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

static const int kPattern[1024] = {
#include "../orb-slam-_amd/csrc/orb_pattern.inc"
};

enum { PATCH_SIZE = 31, HALF_PATCH_SIZE = 15, EDGE_THRESHOLD = 19 };

/* ---- OpenCV scalar helpers -------------------------------- */
static inline int cv_round_f(float v) { return (int)lrintf(v); }   /* cvtss2si, ties-to-even */
static inline int cv_round_d(double v) { return (int)lrint(v); }
static inline int cv_floor_f(float v) { int i = (int)v; return i - (i > v); }
static inline int cv_ceil_f(float v) { int i = (int)v; return i + (i < v); }
static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
static inline short sat_s16_f(float v) { int i = cv_round_f(v); return (short)clampi(i, SHRT_MIN, SHRT_MAX); }

/* ---- a1: tables, src/ORBextractor.cc:466-540 ---------------------------- */
int orbref_make_tables(const orbref_params* p, orbref_tables* t)
{
    if (!p || !t || p->nlevels < 1 || p->nlevels > ORBREF_MAX_LEVELS || p->nfeatures < 0 ||
        !(p->scale_factor > 1.0f))
        return -22;
    memset(t, 0, sizeof(*t));
    t->nlevels = p->nlevels;
    t->nfeatures = p->nfeatures;
    const double scaleFactor = (double)p->scale_factor; /* double member, include/ORBextractor.h:98 */
    t->scale[0] = 1.0f;
    t->sigma2[0] = 1.0f;
    for (int i = 1; i < p->nlevels; i++) {          /* :478-482 */
        t->scale[i] = (float)((double)t->scale[i - 1] * scaleFactor);
        t->sigma2[i] = t->scale[i] * t->scale[i];
    }
    for (int i = 0; i < p->nlevels; i++) {          /* :486-490 */
        t->inv_scale[i] = 1.0f / t->scale[i];
        t->inv_sigma2[i] = 1.0f / t->sigma2[i];
    }
    /* :497-510 per-level feature budget */
    const float factor = (float)(1.0f / scaleFactor);
    float desired = (float)p->nfeatures * (1 - factor) /
                    (1 - (float)pow((double)factor, (double)p->nlevels));
    int sum = 0;
    for (int l = 0; l < p->nlevels - 1; l++) {
        t->nfeat_level[l] = cv_round_f(desired);
        sum += t->nfeat_level[l];
        desired *= factor;
    }
    t->nfeat_level[p->nlevels - 1] = p->nfeatures - sum > 0 ? p->nfeatures - sum : 0;

    /* :522-539 umax */
    const int vmax = cv_floor_f(HALF_PATCH_SIZE * sqrtf(2.f) / 2 + 1);
    const int vmin = cv_ceil_f(HALF_PATCH_SIZE * sqrtf(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (int v = 0; v <= vmax; ++v) t->umax[v] = cv_round_d(sqrt(hp2 - v * v));
    for (int v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (t->umax[v0] == t->umax[v0 + 1]) ++v0;
        t->umax[v] = v0;
        ++v0;
    }
    return 0;
}

void orbref_level_size(const orbref_tables* t, int level, int cols, int rows, int* w, int* h)
{
    /* src/ORBextractor.cc:1347-1348 */
    const float s = t->inv_scale[level];
    *w = cv_round_f((float)cols * s);
    *h = cv_round_f((float)rows * s);
}

/* ---- a3: cv::resize INTER_LINEAR, u8, generic fixed-point path ---------- */
/* SURVEY A.2 alternative: how far OpenCV 3.x's x86 build takes VResizeLinearVec_32s8u (SSE2) over a dst row of
 * `width` bytes before the scalar VResizeLinear loop finishes it: 16 at a time while x <= width - 16, then 4 at a
 * time while x < width - 4 (imgproc/src/resize.cpp), leaving a 0..4-byte scalar tail. */
int orbref_resize_simd_end(int width)
{
    int x = 0;
    while (x <= width - 16) x += 16;
    while (x < width - 4) x += 4;
    return x;
}

/* Vertical pass of one dst pixel: mode 0 the generic FixedPtCast<int, uchar, 22>
 * (h0 b0 + h1 b1 + 2^21) >> 22; mode 1 the SSE2 VResizeLinearVec_32s8u form
 * ((mulhi16(h0 >> 4, b0) + mulhi16(h1 >> 4, b1) + 2) >> 2) (_mm_srai_epi32 by 4, _mm_packs_epi32, _mm_mulhi_epi16,
 * _mm_adds_epi16, _mm_srai_epi16 by 2, _mm_packus_epi16). */
static inline uint8_t resize_vpass(int h0, int h1, int b0, int b1, int simd)
{
    if (!simd) return sat_u8((h0 * b0 + h1 * b1 + (1 << 21)) >> 22);
    const int x0 = clampi(h0 >> 4, SHRT_MIN, SHRT_MAX), x1 = clampi(h1 >> 4, SHRT_MIN, SHRT_MAX);
    const int m = clampi(((x0 * (short)b0) >> 16) + ((x1 * (short)b1) >> 16), SHRT_MIN, SHRT_MAX);
    return sat_u8(clampi(m + 2, SHRT_MIN, SHRT_MAX) >> 2);
}

void orbref_resize_linear_mode(const uint8_t* src, int sw, int sh, size_t sstep,
                               uint8_t* dst, int dw, int dh, size_t dstep, int mode)
{
    const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    const int xs = mode == ORBREF_RESIZE_SSE2 ? orbref_resize_simd_end(dw) : 0;
    int* xofs = (int*)malloc(sizeof(int) * (size_t)dw);
    short* alpha = (short*)malloc(sizeof(short) * 2 * (size_t)dw);
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor_f(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        xofs[dx] = sx;
        alpha[2 * dx] = sat_s16_f((1.f - fx) * 2048);
        alpha[2 * dx + 1] = sat_s16_f(fx * 2048);
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor_f(fy);
        fy -= sy;
        const int b0 = sat_s16_f((1.f - fy) * 2048), b1 = sat_s16_f(fy * 2048);
        const int y0 = clampi(sy, 0, sh - 1), y1 = clampi(sy + 1, 0, sh - 1);
        const uint8_t* r0 = src + (size_t)y0 * sstep;
        const uint8_t* r1 = src + (size_t)y1 * sstep;
        uint8_t* d = dst + (size_t)dy * dstep;
        for (int dx = 0; dx < dw; dx++) {
            const int x0 = xofs[dx], x1 = x0 + 1 < sw ? x0 + 1 : sw - 1;
            const int a0 = alpha[2 * dx], a1 = alpha[2 * dx + 1];
            const int h0 = r0[x0] * a0 + r0[x1] * a1;
            const int h1 = r1[x0] * a0 + r1[x1] * a1;
            d[dx] = resize_vpass(h0, h1, b0, b1, dx < xs);
        }
    }
    free(xofs);
    free(alpha);
}

void orbref_resize_linear(const uint8_t* src, int sw, int sh, size_t sstep,
                          uint8_t* dst, int dw, int dh, size_t dstep)
{
    orbref_resize_linear_mode(src, sw, sh, sstep, dst, dw, dh, dstep, ORBREF_RESIZE_SCALAR);
}

/* ---- a5: cv::FAST TYPE_9_16 with NMS (FAST_t<16> + cornerScore<16>) ----- */
static const int kRingX[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
static const int kRingY[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

static int corner_score16(const uint8_t* ptr, const int* pixel, int threshold)
{
    const int K = 8, N = K * 3 + 1;
    int v = ptr[0];
    short d[25];
    for (int k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = d[k + 1] < d[k + 2] ? d[k + 1] : d[k + 2];
        if (d[k + 3] < a) a = d[k + 3];
        if (a <= a0) continue;
        for (int m = 4; m <= 8; m++) if (d[k + m] < a) a = d[k + m];
        int t0 = a < d[k] ? a : d[k];
        if (t0 > a0) a0 = t0;
        int t1 = a < d[k + 9] ? a : d[k + 9];
        if (t1 > a0) a0 = t1;
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = d[k + 1] > d[k + 2] ? d[k + 1] : d[k + 2];
        for (int m = 3; m <= 5; m++) if (d[k + m] > b) b = d[k + m];
        if (b >= b0) continue;
        for (int m = 6; m <= 8; m++) if (d[k + m] > b) b = d[k + m];
        int t0 = b > d[k] ? b : d[k];
        if (t0 < b0) b0 = t0;
        int t1 = b > d[k + 9] ? b : d[k + 9];
        if (t1 < b0) b0 = t1;
    }
    return -b0 - 1;
}

int orbref_fast(const uint8_t* img, size_t step, int rows, int cols, int threshold, int* out, int cap)
{
    const int K = 8, N = 16 + K + 1;
    int pixel[25];
    for (int k = 0; k < 16; k++) pixel[k] = kRingX[k] + kRingY[k] * (int)step;
    for (int k = 16; k < N; k++) pixel[k] = pixel[k - 16];
    threshold = clampi(threshold, 0, 255);
    uint8_t tab[512];
    for (int i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (rows < 7 || cols < 7) return 0;

    uint8_t* buf = (uint8_t*)calloc((size_t)cols * 3, 1);
    int* cp = (int*)malloc(sizeof(int) * 3 * ((size_t)cols + 1));
    int n = 0;
    for (int i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = img + (size_t)i * step + 3;
        uint8_t* curr = buf + (size_t)((i - 3) % 3) * cols;
        int* cornerpos = cp + (size_t)((i - 3) % 3) * (cols + 1) + 1;
        memset(curr, 0, (size_t)cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; j++, ptr++) {
                const int v = ptr[0];
                const uint8_t* t = tab - v + 255;
                int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
                d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
                d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
                d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
                d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
                d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
                if (d & 1) {
                    const int vt = v - threshold;
                    for (int k = 0, count = 0; k < N; k++) {
                        if (ptr[pixel[k]] < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else count = 0;
                    }
                }
                if (d & 2) {
                    const int vt = v + threshold;
                    for (int k = 0, count = 0; k < N; k++) {
                        if (ptr[pixel[k]] > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf + (size_t)((i - 4 + 3) % 3) * cols;
        const uint8_t* pprev = buf + (size_t)((i - 5 + 3) % 3) * cols;
        cornerpos = cp + (size_t)((i - 4 + 3) % 3) * (cols + 1) + 1;
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            const int j = cornerpos[k];
            const int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                score > curr[j] && score > curr[j + 1]) {
                if (n >= cap) { free(buf); free(cp); return -1; }
                out[3 * n] = j;
                out[3 * n + 1] = i - 1;
                out[3 * n + 2] = score;
                n++;
            }
        }
    }
    free(buf);
    free(cp);
    return n;
}

/* ---- a4: per-level cell loop, src/ORBextractor.cc:932-1002 --------------- */
int orbref_level_candidates(const uint8_t* level, size_t step, int w, int h, int ini_th, int min_th,
                            int* out, int cap)
{
    const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
    const int maxBorderX = w - EDGE_THRESHOLD + 3, maxBorderY = h - EDGE_THRESHOLD + 3;
    const float W = 30;
    const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    if (nCols <= 0 || nRows <= 0) return 0; /* reference divides by zero here */
    const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
    int n = 0;
    int* cell = (int*)malloc(sizeof(int) * 3 * 4096);
    for (int i = 0; i < nRows; i++) {
        const float iniY = (float)(minBorderY + i * hCell);
        float maxY = iniY + hCell + 6;
        if (iniY >= maxBorderY - 3) continue;
        if (maxY > maxBorderY) maxY = (float)maxBorderY;
        for (int j = 0; j < nCols; j++) {
            const float iniX = (float)(minBorderX + j * wCell);
            float maxX = iniX + wCell + 6;
            if (iniX >= maxBorderX - 6) continue;
            if (maxX > maxBorderX) maxX = (float)maxBorderX;
            const int y0 = (int)iniY, x0 = (int)iniX;
            const int rr = (int)maxY - y0, cc = (int)maxX - x0;
            const uint8_t* roi = level + (size_t)y0 * step + x0;
            int k = orbref_fast(roi, step, rr, cc, ini_th, cell, 4096);
            if (k == 0) k = orbref_fast(roi, step, rr, cc, min_th, cell, 4096);
            if (k < 0) { free(cell); return -1; }
            for (int q = 0; q < k; q++) {
                if (n >= cap) { free(cell); return -1; }
                out[3 * n] = cell[3 * q] + j * wCell;
                out[3 * n + 1] = cell[3 * q + 1] + i * hCell;
                out[3 * n + 2] = cell[3 * q + 2];
                n++;
            }
        }
    }
    free(cell);
    return n;
}

int orbref_level_cells(int w, int h)
{
    /* number of FAST cells ComputeKeyPointsOctTree scans on a w x h level (:941-972) */
    const int minB = EDGE_THRESHOLD - 3, maxBX = w - EDGE_THRESHOLD + 3, maxBY = h - EDGE_THRESHOLD + 3;
    const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
    const int nCols = (int)(width / 30), nRows = (int)(height / 30);
    if (nCols <= 0 || nRows <= 0) return 0;
    const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
    int n = 0;
    for (int i = 0; i < nRows; i++) {
        if ((float)(minB + i * hCell) >= maxBY - 3) continue;
        for (int j = 0; j < nCols; j++)
            if (!((float)(minB + j * wCell) >= maxBX - 6)) n++;
    }
    return n;
}

/* ---- a6: DistributeOctTree, src/ORBextractor.cc:569-907 ------------------ */
typedef struct {
    int x0, x1, y0, y1;       /* UL.x, UR.x, UL.y, BL.y */
    int* keys;                /* indices into the candidate array, reference order */
    int nkeys;
    int no_more;
    int prev, next;           /* std::list links */
    long seq;                 /* creation order: canonical tie-break for the size sort */
} qnode;

typedef struct {
    qnode* a;
    int n, cap, head, tail, size;
    long seq;
} qlist;

static int ql_new(qlist* L)
{
    if (L->n == L->cap) {
        L->cap = L->cap ? L->cap * 2 : 256;
        L->a = (qnode*)realloc(L->a, sizeof(qnode) * (size_t)L->cap);
    }
    qnode* q = &L->a[L->n];
    memset(q, 0, sizeof(*q));
    q->prev = q->next = -1;
    return L->n++;
}

static void ql_push_front(qlist* L, int i)
{
    L->a[i].prev = -1;
    L->a[i].next = L->head;
    if (L->head >= 0) L->a[L->head].prev = i; else L->tail = i;
    L->head = i;
    L->a[i].seq = L->seq++;
    L->size++;
}

static void ql_push_back(qlist* L, int i)
{
    L->a[i].next = -1;
    L->a[i].prev = L->tail;
    if (L->tail >= 0) L->a[L->tail].next = i; else L->head = i;
    L->tail = i;
    L->a[i].seq = L->seq++;
    L->size++;
}

static int ql_erase(qlist* L, int i)
{
    qnode* q = &L->a[i];
    const int nx = q->next;
    if (q->prev >= 0) L->a[q->prev].next = q->next; else L->head = q->next;
    if (q->next >= 0) L->a[q->next].prev = q->prev; else L->tail = q->prev;
    free(q->keys);
    q->keys = NULL;
    L->size--;
    return nx;
}

/* ExtractorNode::DivideNode, src/ORBextractor.cc:569-629.  Creates the four
 * children (not yet linked) and returns their indices in ch[0..3]. */
static void divide_node(qlist* L, int pi, const int* xys, int ch[4])
{
    for (int q = 0; q < 4; q++) ch[q] = ql_new(L);
    qnode* p = &L->a[pi];
    const int halfX = (int)ceilf((float)(p->x1 - p->x0) / 2);
    const int halfY = (int)ceilf((float)(p->y1 - p->y0) / 2);
    const int mx = p->x0 + halfX, my = p->y0 + halfY;
    const int rx0[4] = {p->x0, mx, p->x0, mx}, rx1[4] = {mx, p->x1, mx, p->x1};
    const int ry0[4] = {p->y0, p->y0, my, my}, ry1[4] = {my, my, p->y1, p->y1};
    for (int q = 0; q < 4; q++) {
        qnode* c = &L->a[ch[q]];
        c->x0 = rx0[q]; c->x1 = rx1[q]; c->y0 = ry0[q]; c->y1 = ry1[q];
        c->keys = (int*)malloc(sizeof(int) * (size_t)(p->nkeys > 0 ? p->nkeys : 1));
        c->nkeys = 0;
    }
    for (int k = 0; k < p->nkeys; k++) {
        const int id = p->keys[k];
        const float kx = (float)xys[3 * id], ky = (float)xys[3 * id + 1];
        int q;
        if (kx < (float)mx) q = ky < (float)my ? 0 : 2;
        else q = ky < (float)my ? 1 : 3;
        qnode* c = &L->a[ch[q]];
        c->keys[c->nkeys++] = id;
    }
    for (int q = 0; q < 4; q++)
        if (L->a[ch[q]].nkeys == 1) L->a[ch[q]].no_more = 1;
}

typedef struct { int size; long seq; int node; } size_node;

static int cmp_size_node(const void* A, const void* B)
{
    const size_node* a = (const size_node*)A;
    const size_node* b = (const size_node*)B;
    if (a->size != b->size) return a->size < b->size ? -1 : 1;
    return a->seq < b->seq ? -1 : (a->seq > b->seq);   /* canonical: creation order */
}

/* Link the non-empty children of a split node (push_front in n1..n4 order) and
 * record the expandable ones; returns how many had more than one key. */
static int link_children(qlist* L, const int ch[4], size_node** vec, int* nvec, int* capvec)
{
    int nexp = 0;
    for (int q = 0; q < 4; q++) {
        qnode* c = &L->a[ch[q]];
        if (c->nkeys > 0) {
            ql_push_front(L, ch[q]);
            if (L->a[ch[q]].nkeys > 1) {
                nexp++;
                if (*nvec == *capvec) {
                    *capvec = *capvec ? *capvec * 2 : 256;
                    *vec = (size_node*)realloc(*vec, sizeof(size_node) * (size_t)*capvec);
                }
                (*vec)[*nvec].size = L->a[ch[q]].nkeys;
                (*vec)[*nvec].seq = L->a[ch[q]].seq;
                (*vec)[*nvec].node = ch[q];
                (*nvec)++;
            }
        } else {
            free(c->keys);
            c->keys = NULL;
        }
    }
    return nexp;
}

int orbref_distribute(const int* xys, int n, int minX, int maxX, int minY, int maxY, int N,
                      int* out, int cap)
{
    /* :650-653 */
    const int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
    if (nIni <= 0) return -1;          /* reference divides by zero */
    const float hX = (float)(maxX - minX) / nIni;

    qlist L;
    memset(&L, 0, sizeof(L));
    L.head = L.tail = -1;
    int* ini = (int*)malloc(sizeof(int) * (size_t)nIni);
    for (int i = 0; i < nIni; i++) {   /* :663-675 */
        const int id = ql_new(&L);
        qnode* q = &L.a[id];
        q->x0 = (int)(hX * (float)i);
        q->x1 = (int)(hX * (float)(i + 1));
        q->y0 = 0;
        q->y1 = maxY - minY;
        q->keys = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
        ql_push_back(&L, id);
        ini[i] = id;
    }
    for (int k = 0; k < n; k++) {      /* :679-683 */
        size_t r = (size_t)((float)xys[3 * k] / hX);
        if (r >= (size_t)nIni) r = (size_t)nIni - 1;   /* unreachable for in-border keypoints */
        qnode* q = &L.a[ini[r]];
        q->keys[q->nkeys++] = k;
    }
    free(ini);
    for (int it = L.head; it >= 0;) {  /* :688-699 */
        if (L.a[it].nkeys == 1) { L.a[it].no_more = 1; it = L.a[it].next; }
        else if (L.a[it].nkeys == 0) it = ql_erase(&L, it);
        else it = L.a[it].next;
    }

    size_node* vec = NULL;
    int nvec = 0, capvec = 0;
    size_node* prevv = NULL;
    int capprev = 0;
    int finish = 0;
    while (!finish) {                  /* :710-876 */
        int prevSize = L.size;
        int nToExpand = 0;
        nvec = 0;
        for (int it = L.head; it >= 0;) {
            if (L.a[it].no_more) { it = L.a[it].next; continue; }
            int ch[4];
            divide_node(&L, it, xys, ch);
            nToExpand += link_children(&L, ch, &vec, &nvec, &capvec);
            it = ql_erase(&L, it);
        }
        if (L.size >= N || L.size == prevSize) {
            finish = 1;
        } else if (L.size + nToExpand * 3 > N) {
            while (!finish) {          /* :805-874 */
                prevSize = L.size;
                if (capprev < nvec) {
                    capprev = nvec;
                    prevv = (size_node*)realloc(prevv, sizeof(size_node) * (size_t)capprev);
                }
                const int nprev = nvec;
                if (nprev) memcpy(prevv, vec, sizeof(size_node) * (size_t)nprev);
                nvec = 0;
                qsort(prevv, (size_t)nprev, sizeof(size_node), cmp_size_node);
                for (int j = nprev - 1; j >= 0; j--) {
                    int ch[4];
                    divide_node(&L, prevv[j].node, xys, ch);
                    link_children(&L, ch, &vec, &nvec, &capvec);
                    ql_erase(&L, prevv[j].node);
                    if (L.size >= N) break;
                }
                if (L.size >= N || L.size == prevSize) finish = 1;
            }
        }
    }

    /* :882-906 retain the best keypoint per node (first max wins) */
    int m = 0, status = 0;
    for (int it = L.head; it >= 0; it = L.a[it].next) {
        const qnode* q = &L.a[it];
        int best = q->keys[0];
        int bestResp = xys[3 * best + 2];
        for (int k = 1; k < q->nkeys; k++) {
            const int id = q->keys[k];
            if (xys[3 * id + 2] > bestResp) { best = id; bestResp = xys[3 * id + 2]; }
        }
        if (m >= cap) { status = -1; break; }
        out[m++] = best;
    }
    for (int i = 0; i < L.n; i++) free(L.a[i].keys);
    free(L.a);
    free(vec);
    free(prevv);
    return status < 0 ? -1 : m;
}

/* ---- a7: IC_Angle + cv::fastAtan2 --------------------------------------- */
float orbref_fast_atan2(float y, float x)
{
    /* OpenCV 3.x mathfuncs atan_f32; float arithmetic, no FMA */
    static const float k180pi = (float)(180 / 3.1415926535897932384626433832795);
    const float p1 = 0.9997878412794807f * k180pi;
    const float p3 = -0.3258083974640975f * k180pi;
    const float p5 = 0.1555786518463281f * k180pi;
    const float p7 = -0.04432655554792128f * k180pi;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

float orbref_ic_angle(const uint8_t* img, size_t step, int cx, int cy, const int* umax)
{
    /* src/ORBextractor.cc:84-128 */
    const uint8_t* center = img + (size_t)cy * step + cx;
    const int s = (int)step;
    int m01 = 0, m10 = 0;
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m10 += u * center[u];
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int vsum = 0;
        const int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            const int vp = center[u + v * s], vm = center[u - v * s];
            vsum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * vsum;
    }
    return orbref_fast_atan2((float)m01, (float)m10);
}

/* ---- a8: GaussianBlur 7x7 sigma 2 BORDER_REFLECT_101, u8 integer path --- */
static inline int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

/* The 7 integer taps of GaussianBlur(7x7, sigma 2) on u8, per OpenCV build:
 *  ORBREF_BLUR_SCALAR / _SSE2: OpenCV <= 3.4.1 (and 2.4).  createSeparableLinearFilter converts the CV_32F
 *    getGaussianKernel(7, 2) to CV_32S at x256 (convertTo, cvRound): [18 34 49 55 49 34 18], sum 257.
 *  ORBREF_BLUR_BITEXACT: OpenCV >= 3.4.6 / 4.1 GaussianBlur 8U fixed point (smooth.cpp
 *    getGaussianKernelBitExact + getGaussianKernelFixedPoint_ED): the side taps are rounded at 8 fraction
 *    bits with the rounding error carried inwards, and the centre closes the sum to exactly 256. */
void orbref_blur_kernel(int mode, int k[7])
{
    if (mode != ORBREF_BLUR_BITEXACT) {
        static const int k0[7] = {18, 34, 49, 55, 49, 34, 18};
        memcpy(k, k0, sizeof(k0));
        return;
    }
    /* sigmaX = 2; scale2X = -0.125 / sigma^2; values[i] = exp(x*x*scale2X) for x = 1-n, 3-n, .. (step 2) */
    const int n = 7, n2 = 3;
    const double scale2X = -0.125 / (2.0 * 2.0);
    double values[3], sum = 0.0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        values[i] = exp((double)(x * x) * scale2X);
        sum += values[i];
    }
    sum *= 2.0;
    sum += 1.0;
    const double mul1 = 1.0 / sum;
    double err = 0.0;
    int side = 0;
    for (int i = 0; i < n2; i++) {
        const double adj = values[i] * mul1 * 256.0 + err;
        const int v0 = (int)lrint(adj);
        err = adj - (double)v0;
        k[i] = k[n - 1 - i] = v0;
        side += v0;
    }
    k[n2] = 256 - 2 * side;
}

/* The column pass of one pixel from its 7-tap sum T (in 2^-16 units of the output):
 *  scalar: FixedPtCastEx<int, uchar>(16): (T + 2^15) >> 16, saturated.
 *  SSE2 (SymmColumnVec_32s8u, OpenCV <= 3.4.1 x86, every column but the row's width % 4 tail): the taps as
 *    float k/2^16, s = S0*k0 + 0; s += (S+j + S-j)*kj, j = 1..3 (mul then add, no FMA), _mm_cvtps_epi32
 *    (round half to even), _mm_packs_epi32, _mm_packus_epi16. */
static inline uint8_t blur_col(const int* S /* rows y-3 .. y+3 */, const int* k, int simd)
{
    if (!simd) {
        int acc = 0;
        for (int j = 0; j < 7; j++) acc += k[j] * S[j];
        return sat_u8((acc + (1 << 15)) >> 16);
    }
    const float f0 = (float)k[3] * (1.0f / 65536.0f), f1 = (float)k[4] * (1.0f / 65536.0f),
                f2 = (float)k[5] * (1.0f / 65536.0f), f3 = (float)k[6] * (1.0f / 65536.0f);
    float s = (float)S[3] * f0 + 0.0f;
    s = s + (float)(S[4] + S[2]) * f1;
    s = s + (float)(S[5] + S[1]) * f2;
    s = s + (float)(S[6] + S[0]) * f3;
    const long v = lrintf(s);
    return sat_u8(v > SHRT_MAX ? SHRT_MAX : (v < SHRT_MIN ? SHRT_MIN : (int)v));
}

void orbref_gaussian_blur7_mode(const uint8_t* src, int w, int h, size_t sstep, uint8_t* dst, size_t dstep, int mode)
{
    int k[7];
    orbref_blur_kernel(mode, k);
    const int xs = mode == ORBREF_BLUR_SSE2 ? (w & ~3) : 0;   /* SymmColumnVec_32s8u: i <= width - 4, by 16 then 4 */
    int* rows = (int*)malloc(sizeof(int) * (size_t)w * (size_t)h);
    for (int y = 0; y < h; y++) {
        const uint8_t* s = src + (size_t)y * sstep;
        for (int x = 0; x < w; x++) {
            int acc = 0;
            for (int i = 0; i < 7; i++) acc += k[i] * s[reflect101(x + i - 3, w)];
            rows[(size_t)y * w + x] = acc;
        }
    }
    for (int y = 0; y < h; y++) {
        uint8_t* d = dst + (size_t)y * dstep;
        for (int x = 0; x < w; x++) {
            int S[7];
            for (int j = 0; j < 7; j++) S[j] = rows[(size_t)reflect101(y + j - 3, h) * w + x];
            d[x] = blur_col(S, k, x < xs);
        }
    }
    free(rows);
}

void orbref_gaussian_blur7(const uint8_t* src, int w, int h, size_t sstep, uint8_t* dst, size_t dstep)
{
    orbref_gaussian_blur7_mode(src, w, h, sstep, dst, dstep, ORBREF_BLUR_SCALAR);
}

/* ---- a9: computeOrbDescriptor, src/ORBextractor.cc:141-192 --------------- */
/* cos/sin of the BRIEF angle.  ORBREF_TRIG_GLIBC is the host libm's cosf / sinf (glibc 2.35, the
 * reference's own, < 1 ulp but not correctly rounded); ORBREF_TRIG_CR rounds the x87 80-bit cosl / sinl of the
 * same float once to float (correct rounding except where the long double result sits within 2^-64 relative of
 * a float midpoint; tests/test_cv_modes.py checks it against the double evaluation on every angle it meets). */
void orbref_brief_mode(const uint8_t* blur, size_t step, float kx, float ky, float angle_deg, uint8_t desc[32],
                       int trig_mode)
{
    const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
    const float angle = angle_deg * factorPI;
    const float a = trig_mode == ORBREF_TRIG_CR ? (float)cosl((long double)angle) : cosf(angle);
    const float b = trig_mode == ORBREF_TRIG_CR ? (float)sinl((long double)angle) : sinf(angle);
    const uint8_t* center = blur + (ptrdiff_t)cv_round_f(ky) * (ptrdiff_t)step + cv_round_f(kx);
    const int s = (int)step;
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int k = 0; k < 8; ++k) {
            const int* pr = &kPattern[4 * (8 * i + k)];
            int t[2];
            for (int e = 0; e < 2; e++) {
                const float px = (float)pr[2 * e], py = (float)pr[2 * e + 1];
                const int yy = cv_round_f(fmaf(px, b, py * a));
                const int xx = cv_round_f(fmaf(px, a, -(py * b)));
                t[e] = center[yy * s + xx];
            }
            val |= (t[0] < t[1]) << k;
        }
        desc[i] = (uint8_t)val;
    }
}

void orbref_brief(const uint8_t* blur, size_t step, float kx, float ky, float angle_deg, uint8_t desc[32])
{
    orbref_brief_mode(blur, step, kx, ky, angle_deg, desc, ORBREF_TRIG_GLIBC);
}

/* ---- a2: ORBextractor::operator(), src/ORBextractor.cc:1248-1334 --------- */
int orbref_extract_mode(const orbref_params* p, const orbref_cv_modes* m, const uint8_t* img, int rows, int cols,
                        size_t step, orbref_keypoint* kps, int cap, uint8_t* desc, int* n_out,
                        uint8_t* pyramid, int* level_counts, int* cand_counts)
{
    static const orbref_cv_modes canonical = {ORBREF_RESIZE_SCALAR, ORBREF_BLUR_SCALAR, ORBREF_TRIG_GLIBC};
    if (!m) m = &canonical;
    if (!p || !n_out) return -22;
    if (!img || rows <= 0 || cols <= 0) return 1; /* :1252 empty image: no-op */
    orbref_tables t;
    if (orbref_make_tables(p, &t) != 0) return -22;
    const int L = t.nlevels;

    /* a3 ComputePyramid :1342-1377 */
    int lw[ORBREF_MAX_LEVELS], lh[ORBREF_MAX_LEVELS];
    uint8_t* lev[ORBREF_MAX_LEVELS];
    for (int l = 0; l < L; l++) {
        orbref_level_size(&t, l, cols, rows, &lw[l], &lh[l]);
        if (lw[l] <= 0 || lh[l] <= 0) return -22;
        lev[l] = (uint8_t*)malloc((size_t)lw[l] * lh[l]);
        if (l == 0) {
            for (int y = 0; y < rows; y++) memcpy(lev[0] + (size_t)y * cols, img + (size_t)y * step, (size_t)cols);
        } else {
            orbref_resize_linear_mode(lev[l - 1], lw[l - 1], lh[l - 1], (size_t)lw[l - 1], lev[l], lw[l], lh[l],
                                      (size_t)lw[l], m->resize);
        }
    }

    /* a4/a6 ComputeKeyPointsOctTree :915-1026 */
    int* lvl_kx[ORBREF_MAX_LEVELS];
    int* lvl_ky[ORBREF_MAX_LEVELS];
    int* lvl_sc[ORBREF_MAX_LEVELS];
    int lvl_n[ORBREF_MAX_LEVELS];
    int status = 0;
    for (int l = 0; l < L; l++) {
        const int cap_c = lw[l] * lh[l] / 2 + 16;
        int* cand = (int*)malloc(sizeof(int) * 3 * (size_t)cap_c);
        int nc = orbref_level_candidates(lev[l], (size_t)lw[l], lw[l], lh[l], p->ini_th_fast, p->min_th_fast, cand, cap_c);
        if (cand_counts) cand_counts[l] = nc;
        const int minB = EDGE_THRESHOLD - 3;
        const int capd = nc + 4 * 64 + 8;
        int* idx = (int*)malloc(sizeof(int) * (size_t)capd);
        int nd = nc < 0 ? -1
                        : orbref_distribute(cand, nc, minB, lw[l] - EDGE_THRESHOLD + 3, minB,
                                            lh[l] - EDGE_THRESHOLD + 3, t.nfeat_level[l], idx, capd);
        if (nd < 0) { status = -22; nd = 0; }
        lvl_n[l] = nd;
        lvl_kx[l] = (int*)malloc(sizeof(int) * (size_t)(nd + 1));
        lvl_ky[l] = (int*)malloc(sizeof(int) * (size_t)(nd + 1));
        lvl_sc[l] = (int*)malloc(sizeof(int) * (size_t)(nd + 1));
        for (int i = 0; i < nd; i++) {   /* :1019-1025 add border */
            lvl_kx[l][i] = cand[3 * idx[i]] + minB;
            lvl_ky[l][i] = cand[3 * idx[i] + 1] + minB;
            lvl_sc[l][i] = cand[3 * idx[i] + 2];
        }
        free(cand);
        free(idx);
    }
    int total = 0;
    for (int l = 0; l < L; l++) total += lvl_n[l];
    if (status == 0 && total > cap) status = -28;

    if (status == 0) {
        int off = 0;
        for (int l = 0; l < L; l++) {
            if (level_counts) level_counts[l] = lvl_n[l];
            const int nl = lvl_n[l];
            if (nl == 0) continue;
            const float size = (float)(int)(PATCH_SIZE * t.scale[l]);   /* :1013 */
            uint8_t* blur = (uint8_t*)malloc((size_t)lw[l] * lh[l]);
            orbref_gaussian_blur7_mode(lev[l], lw[l], lh[l], (size_t)lw[l], blur, (size_t)lw[l], m->blur);   /* :1300-1306 */
            for (int i = 0; i < nl; i++) {
                orbref_keypoint* k = &kps[off + i];
                const float ang = orbref_ic_angle(lev[l], (size_t)lw[l], lvl_kx[l][i], lvl_ky[l][i], t.umax);  /* :1030-1033 */
                orbref_brief_mode(blur, (size_t)lw[l], (float)lvl_kx[l][i], (float)lvl_ky[l][i], ang,
                                  desc + 32 * (size_t)(off + i), m->trig);
                float x = (float)lvl_kx[l][i], y = (float)lvl_ky[l][i];
                if (l != 0) { x *= t.scale[l]; y *= t.scale[l]; }   /* :1322-1329 */
                k->x = x; k->y = y; k->size = size; k->angle = ang;
                k->response = (float)lvl_sc[l][i];
                k->octave = l; k->class_id = -1;
            }
            free(blur);
            off += nl;
        }
        *n_out = total;
    }
    if (pyramid) {
        size_t o = 0;
        for (int l = 0; l < L; l++) { memcpy(pyramid + o, lev[l], (size_t)lw[l] * lh[l]); o += (size_t)lw[l] * lh[l]; }
    }
    for (int l = 0; l < L; l++) { free(lev[l]); free(lvl_kx[l]); free(lvl_ky[l]); free(lvl_sc[l]); }
    return status;
}

int orbref_extract(const orbref_params* p, const uint8_t* img, int rows, int cols, size_t step,
                   orbref_keypoint* kps, int cap, uint8_t* desc, int* n_out,
                   uint8_t* pyramid, int* level_counts, int* cand_counts)
{
    return orbref_extract_mode(p, NULL, img, rows, cols, step, kps, cap, desc, n_out, pyramid, level_counts,
                               cand_counts);
}

/* ---- a11: DescriptorDistance, src/ORBmatcher.cc:1728-1744 ---------------- */
int orbref_descriptor_distance(const uint8_t* a, const uint8_t* b)
{
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t wa, wb;
        memcpy(&wa, a + 4 * i, 4);
        memcpy(&wb, b + 4 * i, 4);
        uint32_t v = wa ^ wb;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

/* ---- a14 + a16: SearchForInitialization over the Frame grid ------------- */
enum { GRID_COLS = 64, GRID_ROWS = 48, TH_LOW = 50, HISTO_LENGTH = 30 };

static void three_maxima(const int* hist, int* i1, int* i2, int* i3)
{
    /* src/ORBmatcher.cc:1679-1723 */
    int max1 = 0, max2 = 0, max3 = 0;
    *i1 = *i2 = *i3 = -1;
    for (int i = 0; i < HISTO_LENGTH; i++) {
        const int s = hist[i];
        if (s > max1) { max3 = max2; max2 = max1; max1 = s; *i3 = *i2; *i2 = *i1; *i1 = i; }
        else if (s > max2) { max3 = max2; max2 = s; *i3 = *i2; *i2 = i; }
        else if (s > max3) { max3 = s; *i3 = i; }
    }
    if ((float)max2 < 0.1f * (float)max1) { *i2 = -1; *i3 = -1; }
    else if ((float)max3 < 0.1f * (float)max1) { *i3 = -1; }
}

int orbref_search_for_initialization(const orbref_keypoint* k1, const uint8_t* d1, int n1,
                                     const orbref_keypoint* k2, const uint8_t* d2, int n2,
                                     float minX, float maxX, float minY, float maxY, float* prev_xy,
                                     int* matches12, int window, float nnratio, int check_ori)
{
    /* Frame's static image bounds (Frame::ComputeImageBounds, src/Frame.cc:563-621: 0..cols x 0..rows
       without distortion, the undistorted corners otherwise) and grid scale (src/Frame.cc:127-128) */
    const float invW = (float)GRID_COLS / (maxX - minX);
    const float invH = (float)GRID_ROWS / (maxY - minY);

    /* AssignFeaturesToGrid / PosInGrid, src/Frame.cc:292-311, 504-518 */
    int* cnt = (int*)calloc(GRID_COLS * GRID_ROWS + 1, sizeof(int));
    int* cellOf = (int*)malloc(sizeof(int) * (size_t)(n2 + 1));
    for (int i = 0; i < n2; i++) {
        const int px = (int)roundf((k2[i].x - minX) * invW);
        const int py = (int)roundf((k2[i].y - minY) * invH);
        cellOf[i] = (px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS) ? -1 : px * GRID_ROWS + py;
        if (cellOf[i] >= 0) cnt[cellOf[i] + 1]++;
    }
    for (int c = 0; c < GRID_COLS * GRID_ROWS; c++) cnt[c + 1] += cnt[c];
    int* cells = (int*)malloc(sizeof(int) * (size_t)(n2 + 1));
    int* fill = (int*)calloc(GRID_COLS * GRID_ROWS, sizeof(int));
    for (int i = 0; i < n2; i++)
        if (cellOf[i] >= 0) cells[cnt[cellOf[i]] + fill[cellOf[i]]++] = i;

    /* src/ORBmatcher.cc:417-588 */
    int nmatches = 0;
    for (int i = 0; i < n1; i++) matches12[i] = -1;
    int* matchedDist = (int*)malloc(sizeof(int) * (size_t)(n2 + 1));
    int* matches21 = (int*)malloc(sizeof(int) * (size_t)(n2 + 1));
    int* binOf = (int*)malloc(sizeof(int) * (size_t)(n1 + 1));
    for (int i = 0; i < n2; i++) { matchedDist[i] = INT_MAX; matches21[i] = -1; }
    int hist[HISTO_LENGTH] = {0};
    const float factor = 1.0f / HISTO_LENGTH;
    const float r = (float)window;

    for (int i1 = 0; i1 < n1; i1++) {
        binOf[i1] = -1;
        if (k1[i1].octave > 0) continue;
        const float x = prev_xy[2 * i1], y = prev_xy[2 * i1 + 1];
        /* Frame::GetFeaturesInArea(x, y, r, 0, 0), src/Frame.cc:410-495 */
        const int nMinCellX = (int)floorf((x - minX - r) * invW) > 0 ? (int)floorf((x - minX - r) * invW) : 0;
        if (nMinCellX >= GRID_COLS) continue;
        const int cxm = (int)ceilf((x - minX + r) * invW);
        const int nMaxCellX = cxm < GRID_COLS - 1 ? cxm : GRID_COLS - 1;
        if (nMaxCellX < 0) continue;
        const int nMinCellY = (int)floorf((y - minY - r) * invH) > 0 ? (int)floorf((y - minY - r) * invH) : 0;
        if (nMinCellY >= GRID_ROWS) continue;
        const int cym = (int)ceilf((y - minY + r) * invH);
        const int nMaxCellY = cym < GRID_ROWS - 1 ? cym : GRID_ROWS - 1;
        if (nMaxCellY < 0) continue;

        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1, any = 0;
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
                const int c = ix * GRID_ROWS + iy;
                for (int j = cnt[c]; j < cnt[c + 1]; j++) {
                    const int i2 = cells[j];
                    const orbref_keypoint* kp = &k2[i2];
                    if (kp->octave < 0 || kp->octave > 0) continue;
                    const float distx = kp->x - x, disty = kp->y - y;
                    if (!(fabsf(distx) < r && fabsf(disty) < r)) continue;
                    any = 1;
                    const int dist = orbref_descriptor_distance(d1 + 32 * (size_t)i1, d2 + 32 * (size_t)i2);
                    if (matchedDist[i2] <= dist) continue;
                    if (dist < bestDist) { bestDist2 = bestDist; bestDist = dist; bestIdx2 = i2; }
                    else if (dist < bestDist2) bestDist2 = dist;
                }
            }
        }
        if (!any) continue;
        if (bestDist <= TH_LOW && (float)bestDist < (float)bestDist2 * nnratio) {
            if (matches21[bestIdx2] >= 0) { matches12[matches21[bestIdx2]] = -1; nmatches--; }
            matches12[i1] = bestIdx2;
            matches21[bestIdx2] = i1;
            matchedDist[bestIdx2] = bestDist;
            nmatches++;
            if (check_ori) {
                float rot = k1[i1].angle - k2[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                binOf[i1] = bin;
                hist[bin]++;
            }
        }
    }
    if (check_ori) {
        int a, b, c;
        three_maxima(hist, &a, &b, &c);
        for (int i1 = 0; i1 < n1; i1++) {
            const int bin = binOf[i1];
            if (bin < 0 || bin == a || bin == b || bin == c) continue;
            if (matches12[i1] >= 0) { matches12[i1] = -1; nmatches--; }
        }
    }
    for (int i1 = 0; i1 < n1; i1++)
        if (matches12[i1] >= 0) { prev_xy[2 * i1] = k2[matches12[i1]].x; prev_xy[2 * i1 + 1] = k2[matches12[i1]].y; }
    free(cnt); free(cellOf); free(cells); free(fill); free(matchedDist); free(matches21); free(binOf);
    return nmatches;
}

void orbref_allpairs_top2(const uint8_t* q, int nq, const uint8_t* t, int nt,
                          int* best_idx, int* best_d, int* second_d)
{
    for (int i = 0; i < nq; i++) {
        int b1 = 256, b2 = 256, bi = -1;
        for (int j = 0; j < nt; j++) {
            const int d = orbref_descriptor_distance(q + 32 * (size_t)i, t + 32 * (size_t)j);
            if (d < b1) { b2 = b1; b1 = d; bi = j; }
            else if (d < b2) b2 = d;
        }
        best_idx[i] = bi; best_d[i] = b1; second_d[i] = b2;
    }
}

/* ---- a15: Frame::ComputeStereoMatches, src/Frame.cc:630-872 -------------- */
/* Level l of a concatenated pyramid dump (orbref_extract's `pyramid` layout). */
static const uint8_t* pyr_level(const uint8_t* pyr, const orbref_tables* t, int l, int cols, int rows, int* w, int* h)
{
    size_t o = 0;
    for (int q = 0; q < l; q++) {
        int qw, qh;
        orbref_level_size(t, q, cols, rows, &qw, &qh);
        o += (size_t)qw * qh;
    }
    orbref_level_size(t, l, cols, rows, w, h);
    return pyr + o;
}

static int cmp_dist_idx(const void* a, const void* b)
{
    const int* x = (const int*)a;
    const int* y = (const int*)b;
    if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;   /* std::pair<int,int> ordering */
    return x[1] < y[1] ? -1 : (x[1] > y[1]);
}

/* row table :645-673: vRowIndices[yi] lists iR in increasing order.  Rows outside
 * [0, nRows) are UB in the reference (never reached for kps >= 19 px from the edge);
 * they are dropped here.  rcnt[y]..rcnt[y+1] index ridx. */
static void stereo_row_table(const orbref_keypoint* kR, int nR, const float* scale, int nRows, int** rcnt_out,
                             int** ridx_out)
{
    int* rcnt = (int*)calloc((size_t)nRows + 1, sizeof(int));
    for (int iR = 0; iR < nR; iR++) {
        const float kpY = kR[iR].y;
        const float r = 2.0f * scale[kR[iR].octave];
        const int maxr = (int)ceilf(kpY + r);
        const int minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) rcnt[yi + 1]++;
    }
    for (int y = 0; y < nRows; y++) rcnt[y + 1] += rcnt[y];
    int* ridx = (int*)malloc(sizeof(int) * ((size_t)rcnt[nRows] + 1));
    int* rfill = (int*)calloc((size_t)nRows + 1, sizeof(int));
    for (int iR = 0; iR < nR; iR++) {
        const float kpY = kR[iR].y;
        const float r = 2.0f * scale[kR[iR].octave];
        const int maxr = (int)ceilf(kpY + r);
        const int minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) ridx[rcnt[yi] + rfill[yi]++] = iR;
    }
    free(rfill);
    *rcnt_out = rcnt;
    *ridx_out = ridx;
}

/* the coarse search of one left keypoint, :699-757: returns bestDist (TH_HIGH = 100 when no
 * candidate beats it, or when the keypoint is skipped) and sets *bestIdxR (first min, increasing iR) */
static int stereo_coarse(const orbref_keypoint* kpL, const uint8_t* dLi, const orbref_keypoint* kR, const uint8_t* dR,
                         const int* rcnt, const int* ridx, int nRows, float minD, float maxD, int* bestIdxR)
{
    const int levelL = kpL->octave;
    const float vL = kpL->y, uL = kpL->x;
    if (vL < 0) return 100;                              /* (size_t) of a negative float: UB, never reached */
    const size_t row = (size_t)vL;                       /* vRowIndices[vL], :699 */
    if (row >= (size_t)nRows) return 100;
    const int c0 = rcnt[row], c1 = rcnt[row + 1];
    if (c0 == c1) return 100;                            /* :702-703 */
    const float minU = uL - maxD, maxU = uL - minD;      /* :707-708 */
    if (maxU < 0) return 100;
    int bestDist = 100;                                  /* ORBmatcher::TH_HIGH */
    for (int c = c0; c < c1; c++) {                      /* :723-757 */
        const int iR = ridx[c];
        const orbref_keypoint* kpR = &kR[iR];
        if (kpR->octave < levelL - 1 || kpR->octave > levelL + 1) continue;
        const float uR = kpR->x;
        if (uR >= minU && uR <= maxU) {
            const int dist = orbref_descriptor_distance(dLi, dR + 32 * (size_t)iR);
            if (dist < bestDist) { bestDist = dist; *bestIdxR = iR; }
        }
    }
    return bestDist;
}

int orbref_compute_stereo_matches(const orbref_params* p, int rows, int cols, const uint8_t* pyrL,
                                  const uint8_t* pyrR, const orbref_keypoint* kL, const uint8_t* dL, int nL,
                                  const orbref_keypoint* kR, const uint8_t* dR, int nR, float bf, float fx,
                                  float* uRight, float* depth, int* sad_out)
{
    orbref_tables t;
    if (orbref_make_tables(p, &t) != 0) return -22;
    for (int i = 0; i < nL; i++) { uRight[i] = -1.0f; depth[i] = -1.0f; if (sad_out) sad_out[i] = -1; }  /* :633-634 */
    const int thOrbDist = (100 + TH_LOW) / 2;                                                             /* :638 */
    const int nRows = rows;                                                                               /* :641 */

    int *rcnt, *ridx;
    stereo_row_table(kR, nR, t.scale, nRows, &rcnt, &ridx);

    /* :676-681.  The reference reads the member mb before Frame's constructor assigns
     * it (src/Frame.cc:108 vs :140); the intended value mb = mbf/fx is used. */
    const float mb = bf / fx;
    const float minZ = mb;
    const float minD = 0;
    const float maxD = bf / minZ;

    int* vDistIdx = (int*)malloc(sizeof(int) * 2 * ((size_t)nL + 1));
    int nd = 0;
    for (int iL = 0; iL < nL; iL++) {
        const orbref_keypoint* kpL = &kL[iL];
        const int levelL = kpL->octave;
        const float uL = kpL->x;
        int bestIdxR = 0;
        const int bestDist = stereo_coarse(kpL, dL + 32 * (size_t)iL, kR, dR, rcnt, ridx, nRows, minD, maxD, &bestIdxR);
        if (bestDist >= thOrbDist) continue;                 /* :762 */

        /* sub-pixel match by correlation, :764-853 */
        const float uR0 = kR[bestIdxR].x;
        const float scaleFactor = t.inv_scale[levelL];
        const float scaleduL = roundf(kpL->x * scaleFactor);
        const float scaledvL = roundf(kpL->y * scaleFactor);
        const float scaleduR0 = roundf(uR0 * scaleFactor);
        const int w = 5, L = 5;
        int lw, lh, rw, rh;
        const uint8_t* IL0 = pyr_level(pyrL, &t, levelL, cols, rows, &lw, &lh);
        const uint8_t* IR0 = pyr_level(pyrR, &t, levelL, cols, rows, &rw, &rh);
        const float iniu = scaleduR0 + L - w;                /* quirk kept: +L, :795 */
        const float endu = scaleduR0 + L + w + 1;
        if (iniu < 0 || endu >= rw) continue;
        const int vy = (int)scaledvL, ux = (int)scaleduL, ur = (int)scaleduR0;
        /* windows read the level's 19-px BORDER_REFLECT_101 padding when they cross an
         * edge (ComputePyramid :1350-1373); beyond the padding the reference is UB */
        if (vy - w < -EDGE_THRESHOLD || vy + w >= lh + EDGE_THRESHOLD || ux - w < -EDGE_THRESHOLD ||
            ux + w >= lw + EDGE_THRESHOLD || ur - L - w < -EDGE_THRESHOLD)
            continue;
#define PADPX(img, W, H, X, Y) ((float)(img)[(size_t)reflect101((Y), (H)) * (W) + reflect101((X), (W))])
        const float cL = PADPX(IL0, lw, lh, ux, vy);
        float vDists[11];
        int bestDistS = INT_MAX, bestincR = 0;
        for (int incR = -L; incR <= L; incR++) {
            const float cR = PADPX(IR0, rw, rh, ur + incR, vy);
            double acc = 0.0;                                /* cv::norm(IL, IR, NORM_L1) */
            for (int y = -w; y <= w; y++)
                for (int x = -w; x <= w; x++) {
                    const float a = PADPX(IL0, lw, lh, ux + x, vy + y) - cL;
                    const float b = PADPX(IR0, rw, rh, ur + incR + x, vy + y) - cR;
                    acc += fabs((double)a - (double)b);
                }
            const float dist = (float)acc;
            if (dist < (float)bestDistS) { bestDistS = (int)dist; bestincR = incR; }
            vDists[L + incR] = dist;
        }
        if (bestincR == -L || bestincR == L) continue;       /* :816-817 */
        const float dist1 = vDists[L + bestincR - 1];
        const float dist2 = vDists[L + bestincR];
        const float dist3 = vDists[L + bestincR + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = t.scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
        float disparity = (uL - bestuR);
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
                disparity = (float)0.01;
                bestuR = (float)((double)uL - 0.01);
            }
            depth[iL] = bf / disparity;
            uRight[iL] = bestuR;
            if (sad_out) sad_out[iL] = bestDistS;
            vDistIdx[2 * nd] = bestDistS;
            vDistIdx[2 * nd + 1] = iL;
            nd++;
        }
    }
    /* median cut :857-871 (an empty vDistIdx is UB in the reference: nothing to cut) */
    int good = nd;
    if (nd > 0) {
        qsort(vDistIdx, (size_t)nd, 2 * sizeof(int), cmp_dist_idx);
        const float median = (float)vDistIdx[2 * (nd / 2)];
        const float thDist = 1.5f * 1.4f * median;
        for (int i = nd - 1; i >= 0; i--) {
            if ((float)vDistIdx[2 * i] < thDist) break;
            uRight[vDistIdx[2 * i + 1]] = -1;
            depth[vDistIdx[2 * i + 1]] = -1;
            good--;
        }
    }
#undef PADPX
    free(rcnt); free(ridx); free(vDistIdx);
    return good;
}

int orbref_stereo_band(const orbref_keypoint* kL, const uint8_t* dL, int nL, const orbref_keypoint* kR,
                       const uint8_t* dR, int nR, int rows, const float* scale, float minD, float maxD,
                       int* best_idx, int* best_dist)
{
    int *rcnt, *ridx;
    stereo_row_table(kR, nR, scale, rows, &rcnt, &ridx);
    for (int iL = 0; iL < nL; iL++) {
        int bestIdxR = 0;
        const int bestDist = stereo_coarse(&kL[iL], dL + 32 * (size_t)iL, kR, dR, rcnt, ridx, rows, minD, maxD,
                                           &bestIdxR);
        best_dist[iL] = bestDist;
        best_idx[iL] = bestDist < 100 ? bestIdxR : -1;
    }
    free(rcnt); free(ridx);
    return 0;
}

/* ---- a12 / a13: vocabulary-node candidate searches, src/ORBmatcher.cc ------
 * DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>) as CSR: node ids
 * ascending, ptr[k]..ptr[k+1] the feature indices of node k in insertion order.
 * The merge-join over the two maps (:175-257) visits the shared node ids in
 * ascending order. */
static int fv_find(const orbref_featvec* f, int node, int from)
{
    int lo = from, hi = f->nnodes;   /* lower_bound */
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (f->node[mid] < node) lo = mid + 1; else hi = mid;
    }
    return lo;
}

static int rot_bin(float a1, float a2)
{
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

/* rotation-consistency filter (:259-285 and twins): drop every match outside the three
 * largest histogram bins.  match[] is indexed like bins[]; returns the matches removed. */
static int rot_filter(const int* bins, int n, int* match)
{
    int hist[HISTO_LENGTH] = {0};
    for (int i = 0; i < n; i++)
        if (bins[i] >= 0) hist[bins[i]]++;
    int a, b, c, removed = 0;
    three_maxima(hist, &a, &b, &c);
    for (int i = 0; i < n; i++) {
        const int bin = bins[i];
        if (bin < 0 || bin == a || bin == b || bin == c) continue;
        match[i] = -1;
        removed++;
    }
    return removed;
}

int orbref_search_by_bow_kf_f(const orbref_keypoint* kkf, const uint8_t* dkf, const uint8_t* kf_has_mp, int nkf,
                              const orbref_featvec* fvkf, const orbref_keypoint* kf, const uint8_t* df, int nf,
                              const orbref_featvec* fvf, float nnratio, int check_ori, int* match_f)
{
    /* src/ORBmatcher.cc:159-288 */
    int* bins = (int*)malloc(sizeof(int) * ((size_t)nf + 1));
    for (int i = 0; i < nf; i++) { match_f[i] = -1; bins[i] = -1; }
    int nmatches = 0;
    int ik = 0, jf = 0;
    while (ik < fvkf->nnodes && jf < fvf->nnodes) {
        const int nk = fvkf->node[ik], nfn = fvf->node[jf];
        if (nk == nfn) {
            for (int a = fvkf->ptr[ik]; a < fvkf->ptr[ik + 1]; a++) {
                const int realIdxKF = fvkf->idx[a];
                if (!kf_has_mp[realIdxKF]) continue;   /* !pMP || pMP->isBad() */
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                for (int b = fvf->ptr[jf]; b < fvf->ptr[jf + 1]; b++) {
                    const int realIdxF = fvf->idx[b];
                    if (match_f[realIdxF] >= 0) continue;
                    const int dist = orbref_descriptor_distance(dkf + 32 * (size_t)realIdxKF, df + 32 * (size_t)realIdxF);
                    if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdxF = realIdxF; }
                    else if (dist < bestDist2) bestDist2 = dist;
                }
                if (bestDist1 <= TH_LOW && (float)bestDist1 < nnratio * (float)bestDist2) {
                    match_f[bestIdxF] = realIdxKF;
                    if (check_ori) bins[bestIdxF] = rot_bin(kkf[realIdxKF].angle, kf[bestIdxF].angle);
                    nmatches++;
                }
            }
            ik++;
            jf++;
        } else if (nk < nfn) {
            ik = fv_find(fvkf, nfn, ik);
        } else {
            jf = fv_find(fvf, nk, jf);
        }
    }
    if (check_ori) nmatches -= rot_filter(bins, nf, match_f);
    free(bins);
    return nmatches;
}

int orbref_search_by_bow_kf_kf(const orbref_keypoint* k1, const uint8_t* d1, const uint8_t* has_mp1, int n1,
                               const orbref_featvec* fv1, const orbref_keypoint* k2, const uint8_t* d2,
                               const uint8_t* has_mp2, int n2, const orbref_featvec* fv2, float nnratio,
                               int check_ori, int* match12)
{
    /* src/ORBmatcher.cc:590-723 */
    int* bins = (int*)malloc(sizeof(int) * ((size_t)n1 + 1));
    uint8_t* matched2 = (uint8_t*)calloc((size_t)n2 + 1, 1);
    for (int i = 0; i < n1; i++) { match12[i] = -1; bins[i] = -1; }
    int nmatches = 0;
    int i1 = 0, i2 = 0;
    while (i1 < fv1->nnodes && i2 < fv2->nnodes) {
        const int a1 = fv1->node[i1], a2 = fv2->node[i2];
        if (a1 == a2) {
            for (int a = fv1->ptr[i1]; a < fv1->ptr[i1 + 1]; a++) {
                const int idx1 = fv1->idx[a];
                if (!has_mp1[idx1]) continue;
                int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
                for (int b = fv2->ptr[i2]; b < fv2->ptr[i2 + 1]; b++) {
                    const int idx2 = fv2->idx[b];
                    if (matched2[idx2] || !has_mp2[idx2]) continue;
                    const int dist = orbref_descriptor_distance(d1 + 32 * (size_t)idx1, d2 + 32 * (size_t)idx2);
                    if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdx2 = idx2; }
                    else if (dist < bestDist2) bestDist2 = dist;
                }
                if (bestDist1 < TH_LOW && (float)bestDist1 < nnratio * (float)bestDist2) {   /* strict < (:666) */
                    match12[idx1] = bestIdx2;
                    matched2[bestIdx2] = 1;
                    if (check_ori) bins[idx1] = rot_bin(k1[idx1].angle, k2[bestIdx2].angle);
                    nmatches++;
                }
            }
            i1++;
            i2++;
        } else if (a1 < a2) {
            i1 = fv_find(fv1, a2, i1);
        } else {
            i2 = fv_find(fv2, a1, i2);
        }
    }
    if (check_ori) nmatches -= rot_filter(bins, n1, match12);
    free(bins);
    free(matched2);
    return nmatches;
}

/* CheckDistEpipolarLine (src/ORBmatcher.cc:140-157).  The reference is built with
 * -O3 -march=native; GCC 11 contracts these expressions into the FMAs written here
 * (verified on this host's g++ 11.4 at -march=x86-64-v3). */
static int check_epipolar(const orbref_keypoint* kp1, const orbref_keypoint* kp2, const float* F, const float* sigma2)
{
    const float a = fmaf(kp1->x, F[0], kp1->y * F[3]) + F[6];
    const float b = fmaf(kp1->x, F[1], kp1->y * F[4]) + F[7];
    const float c = fmaf(kp1->y, F[5], kp1->x * F[2]) + F[8];
    const float num = fmaf(b, kp2->y, a * kp2->x) + c;
    const float den = fmaf(a, a, b * b);
    if (den == 0) return 0;
    const float dsqr = num * num / den;
    return (double)dsqr < 3.84 * (double)sigma2[kp2->octave];
}

int orbref_search_for_triangulation(const orbref_keypoint* k1, const uint8_t* d1, const uint8_t* has_mp1,
                                    const float* uright1, int n1, const orbref_featvec* fv1,
                                    const orbref_keypoint* k2, const uint8_t* d2, const uint8_t* has_mp2,
                                    const float* uright2, int n2, const orbref_featvec* fv2, const float* F12,
                                    float ex, float ey, const float* scale2, const float* sigma2_2,
                                    int only_stereo, int check_ori, int* match12)
{
    /* src/ORBmatcher.cc:725-891; vbMatched2 is never set, so every idx1 is independent */
    int* bins = (int*)malloc(sizeof(int) * ((size_t)n1 + 1));
    for (int i = 0; i < n1; i++) { match12[i] = -1; bins[i] = -1; }
    int nmatches = 0;
    int i1 = 0, i2 = 0;
    while (i1 < fv1->nnodes && i2 < fv2->nnodes) {
        const int a1 = fv1->node[i1], a2 = fv2->node[i2];
        if (a1 == a2) {
            for (int a = fv1->ptr[i1]; a < fv1->ptr[i1 + 1]; a++) {
                const int idx1 = fv1->idx[a];
                if (has_mp1[idx1]) continue;
                const int bStereo1 = uright1[idx1] >= 0;
                if (only_stereo && !bStereo1) continue;
                const orbref_keypoint* kp1 = &k1[idx1];
                int bestDist = TH_LOW, bestIdx2 = -1;
                for (int b = fv2->ptr[i2]; b < fv2->ptr[i2 + 1]; b++) {
                    const int idx2 = fv2->idx[b];
                    if (has_mp2[idx2]) continue;   /* vbMatched2[idx2] is always false */
                    const int bStereo2 = uright2[idx2] >= 0;
                    if (only_stereo && !bStereo2) continue;
                    const int dist = orbref_descriptor_distance(d1 + 32 * (size_t)idx1, d2 + 32 * (size_t)idx2);
                    if (dist > TH_LOW || dist > bestDist) continue;
                    const orbref_keypoint* kp2 = &k2[idx2];
                    if (!bStereo1 && !bStereo2) {
                        const float distex = ex - kp2->x;
                        const float distey = ey - kp2->y;
                        if (fmaf(distex, distex, distey * distey) < 100 * scale2[kp2->octave]) continue;
                    }
                    if (check_epipolar(kp1, kp2, F12, sigma2_2)) { bestIdx2 = idx2; bestDist = dist; }
                }
                if (bestIdx2 >= 0) {
                    match12[idx1] = bestIdx2;
                    nmatches++;
                    if (check_ori) bins[idx1] = rot_bin(kp1->angle, k2[bestIdx2].angle);
                }
            }
            i1++;
            i2++;
        } else if (a1 < a2) {
            i1 = fv_find(fv1, a2, i1);
        } else {
            i2 = fv_find(fv2, a1, i2);
        }
    }
    if (check_ori) nmatches -= rot_filter(bins, n1, match12);
    free(bins);
    return nmatches;
}

/* ---- §8f row 2: DBoW2 TemplatedVocabulary::transform ---------------------
 * Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1259 (transform of a feature
 * set and of one feature), BowVector.cpp:34-84 (addWeight / addIfNotExist /
 * normalize), FeatureVector.cpp:31-45 (addFeature).  Nodes: node 0 is the root;
 * node i > 0 has parent[i], a file leaf flag and a weight; the children of a node
 * are the nodes naming it as parent, in id order (loadFromTextFile :1378-1386).
 * isLeaf() is "no children" (:328); word ids number the flagged leaves in id order. */
int orbref_voc_transform(int nnodes, const int* parent, const uint8_t* is_leaf_flag, const uint8_t* desc,
                         const double* weight, int L, int scoring, int weighting, const uint8_t* feats, int n,
                         int levelsup, int* bow_word, double* bow_weight, int* bow_n, int* fv_node, int* fv_ptr,
                         int* fv_idx, int* fv_nnodes)
{
    if (nnodes < 2) { *bow_n = 0; *fv_nnodes = 0; fv_ptr[0] = 0; return 0; }
    int* ccount = (int*)calloc((size_t)nnodes, sizeof(int));
    int* cbegin = (int*)calloc((size_t)nnodes + 1, sizeof(int));
    int* child = (int*)malloc(sizeof(int) * (size_t)nnodes);
    int* word_of = (int*)calloc((size_t)nnodes, sizeof(int));
    for (int i = 1; i < nnodes; i++) ccount[parent[i]]++;
    for (int i = 0; i < nnodes; i++) cbegin[i + 1] = cbegin[i] + ccount[i];
    int* fill = (int*)calloc((size_t)nnodes, sizeof(int));
    int nwords = 0;
    for (int i = 1; i < nnodes; i++) {
        child[cbegin[parent[i]] + fill[parent[i]]++] = i;
        if (is_leaf_flag[i]) word_of[i] = nwords++;
    }
    /* scoring -> mustNormalize (ScoringObject.h:74-89) */
    const int must = scoring != 5;               /* DOT_PRODUCT does not normalise */
    const int l2 = scoring == 1;                 /* L2_NORM; the others normalise with L1 */
    const int nid_level = L - levelsup;
    int* wid = (int*)malloc(sizeof(int) * ((size_t)n + 1));
    int* nid = (int*)malloc(sizeof(int) * ((size_t)n + 1));
    double* w = (double*)malloc(sizeof(double) * ((size_t)n + 1));
    for (int f = 0; f < n; f++) {
        const uint8_t* d = feats + 32 * (size_t)f;
        int final_id = 0, level = 0, nd = 0;
        do {   /* :1224-1248 */
            ++level;
            const int c0 = cbegin[final_id], c1 = cbegin[final_id + 1];
            final_id = child[c0];
            double best_d = (double)orbref_descriptor_distance(d, desc + 32 * (size_t)final_id);
            for (int c = c0 + 1; c < c1; c++) {
                const int id = child[c];
                const double dd = (double)orbref_descriptor_distance(d, desc + 32 * (size_t)id);
                if (dd < best_d) { best_d = dd; final_id = id; }
            }
            if (level == nid_level) nd = final_id;
        } while (ccount[final_id] > 0);
        if (nid_level <= 0) nd = 0;
        else if (level < nid_level) nd = final_id;   /* unset in the reference (leaf above nid_level) */
        wid[f] = word_of[final_id];
        w[f] = weight[final_id];
        nid[f] = nd;
    }
    /* BowVector (std::map by word id) and FeatureVector (std::map by node id) */
    int nb = 0, nf = 0;
    for (int f = 0; f < n; f++) {
        if (!(w[f] > 0)) continue;   /* stopped word */
        /* BowVector: lower_bound insert */
        int lo = 0, hi = nb;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (bow_word[mid] < wid[f]) lo = mid + 1; else hi = mid; }
        if (lo < nb && bow_word[lo] == wid[f]) {
            if (weighting == 0 || weighting == 1) bow_weight[lo] += w[f];   /* addWeight; IDF/BINARY: addIfNotExist */
        } else {
            memmove(bow_word + lo + 1, bow_word + lo, sizeof(int) * (size_t)(nb - lo));
            memmove(bow_weight + lo + 1, bow_weight + lo, sizeof(double) * (size_t)(nb - lo));
            bow_word[lo] = wid[f];
            bow_weight[lo] = w[f];
            nb++;
        }
        /* FeatureVector: node list, each with its features in insertion order */
        lo = 0; hi = nf;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (fv_node[mid] < nid[f]) lo = mid + 1; else hi = mid; }
        if (!(lo < nf && fv_node[lo] == nid[f])) {
            memmove(fv_node + lo + 1, fv_node + lo, sizeof(int) * (size_t)(nf - lo));
            fv_node[lo] = nid[f];
            nf++;
        }
    }
    /* CSR of the FeatureVector: features in index order within each node */
    for (int k = 0; k <= nf; k++) fv_ptr[k] = 0;
    for (int f = 0; f < n; f++) {
        if (!(w[f] > 0)) continue;
        int lo = 0, hi = nf;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (fv_node[mid] < nid[f]) lo = mid + 1; else hi = mid; }
        fv_ptr[lo + 1]++;
    }
    for (int k = 0; k < nf; k++) fv_ptr[k + 1] += fv_ptr[k];
    int* pos = (int*)calloc((size_t)nf + 1, sizeof(int));
    for (int f = 0; f < n; f++) {
        if (!(w[f] > 0)) continue;
        int lo = 0, hi = nf;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (fv_node[mid] < nid[f]) lo = mid + 1; else hi = mid; }
        fv_idx[fv_ptr[lo] + pos[lo]++] = f;
    }
    if (weighting == 0 || weighting == 1) {
        if (nb > 0 && !must) {   /* :1155-1161 */
            const double ndd = (double)nb;
            for (int i = 0; i < nb; i++) bow_weight[i] /= ndd;
        }
    }
    if (must) {   /* BowVector::normalize, BowVector.cpp:62-84 */
        double norm = 0.0;
        if (!l2) { for (int i = 0; i < nb; i++) norm += fabs(bow_weight[i]); }
        else { for (int i = 0; i < nb; i++) norm += bow_weight[i] * bow_weight[i]; norm = sqrt(norm); }
        if (norm > 0.0)
            for (int i = 0; i < nb; i++) bow_weight[i] /= norm;
    }
    *bow_n = nb;
    *fv_nnodes = nf;
    free(ccount); free(cbegin); free(child); free(word_of); free(fill); free(wid); free(nid); free(w); free(pos);
    return 0;
}

/* ---- §8f row 3: ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th) ----
 * src/ORBmatcher.cc:45-129 with Frame::GetFeaturesInArea (src/Frame.cc:410-495) over the
 * frame grid (AssignFeaturesToGrid / PosInGrid, :292-311, 504-518).  Per MapPoint the
 * caller supplies what Tracking::SearchLocalPoints leaves in it (mTrackProjX/Y/XR,
 * mTrackViewCos, mnTrackScaleLevel, mbTrackInView && !isBad, Observations() > 0) and its
 * descriptor.  claimed[i] = F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0 on
 * entry; match[i] = the MapPoint this call assigned to F feature i (the last one), -1. */
int orbref_search_by_projection(const orbref_keypoint* kps, const uint8_t* desc, const float* uright,
                                const uint8_t* claimed_in, int n, float min_x, float min_y, float grid_w_inv,
                                float grid_h_inv, const float* scale, const orbref_proj_point* pts,
                                const uint8_t* pdesc, int np, float th, float nnratio, int* match)
{
    int* cnt = (int*)calloc(GRID_COLS * GRID_ROWS + 1, sizeof(int));
    int* cellOf = (int*)malloc(sizeof(int) * ((size_t)n + 1));
    for (int i = 0; i < n; i++) {   /* PosInGrid */
        const int px = (int)roundf((kps[i].x - min_x) * grid_w_inv);
        const int py = (int)roundf((kps[i].y - min_y) * grid_h_inv);
        cellOf[i] = (px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS) ? -1 : px * GRID_ROWS + py;
        if (cellOf[i] >= 0) cnt[cellOf[i] + 1]++;
    }
    for (int c = 0; c < GRID_COLS * GRID_ROWS; c++) cnt[c + 1] += cnt[c];
    int* cells = (int*)malloc(sizeof(int) * ((size_t)n + 1));
    int* fill = (int*)calloc(GRID_COLS * GRID_ROWS, sizeof(int));
    for (int i = 0; i < n; i++)
        if (cellOf[i] >= 0) cells[cnt[cellOf[i]] + fill[cellOf[i]]++] = i;
    uint8_t* claimed = (uint8_t*)malloc((size_t)n + 1);
    for (int i = 0; i < n; i++) { claimed[i] = claimed_in[i]; match[i] = -1; }

    const int bFactor = th != 1.0;
    int nmatches = 0;
    for (int m = 0; m < np; m++) {
        const orbref_proj_point* P = &pts[m];
        if (!(P->flags & 1)) continue;                          /* !mbTrackInView || isBad() */
        const int level = P->level;
        float r = P->view_cos > 0.998 ? 2.5f : 4.0f;            /* RadiusByViewingCos, :130-136 */
        if (bFactor) r *= th;
        const float rr = r * scale[level];
        const float x = P->proj_x, y = P->proj_y;
        const int minLevel = level - 1, maxLevel = level;
        const int nMinCellX = (int)floorf((x - min_x - rr) * grid_w_inv) > 0 ? (int)floorf((x - min_x - rr) * grid_w_inv) : 0;
        if (nMinCellX >= GRID_COLS) continue;
        const int cxm = (int)ceilf((x - min_x + rr) * grid_w_inv);
        const int nMaxCellX = cxm < GRID_COLS - 1 ? cxm : GRID_COLS - 1;
        if (nMaxCellX < 0) continue;
        const int nMinCellY = (int)floorf((y - min_y - rr) * grid_h_inv) > 0 ? (int)floorf((y - min_y - rr) * grid_h_inv) : 0;
        if (nMinCellY >= GRID_ROWS) continue;
        const int cym = (int)ceilf((y - min_y + rr) * grid_h_inv);
        const int nMaxCellY = cym < GRID_ROWS - 1 ? cym : GRID_ROWS - 1;
        if (nMaxCellY < 0) continue;
        const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1, any = 0;
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
                const int c = ix * GRID_ROWS + iy;
                for (int j = cnt[c]; j < cnt[c + 1]; j++) {
                    const int idx = cells[j];
                    const orbref_keypoint* kp = &kps[idx];
                    if (bCheckLevels) {
                        if (kp->octave < minLevel) continue;
                        if (maxLevel >= 0 && kp->octave > maxLevel) continue;
                    }
                    const float distx = kp->x - x, disty = kp->y - y;
                    if (!(fabsf(distx) < rr && fabsf(disty) < rr)) continue;
                    any = 1;   /* in vIndices */
                    if (claimed[idx]) continue;                 /* :82-84 */
                    if (uright[idx] > 0) {                      /* :86-91 */
                        const float er = fabsf(P->proj_xr - uright[idx]);
                        if (er > r * scale[level]) continue;
                    }
                    const int dist = orbref_descriptor_distance(pdesc + 32 * (size_t)m, desc + 32 * (size_t)idx);
                    if (dist < bestDist) {
                        bestDist2 = bestDist; bestDist = dist;
                        bestLevel2 = bestLevel; bestLevel = kp->octave;
                        bestIdx = idx;
                    } else if (dist < bestDist2) {
                        bestLevel2 = kp->octave; bestDist2 = dist;
                    }
                }
            }
        }
        if (!any) continue;
        if (bestDist <= 100) {                                  /* TH_HIGH, :116-124 */
            if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) continue;
            match[bestIdx] = m;
            claimed[bestIdx] = (P->flags & 2) ? 1 : 0;          /* F.mvpMapPoints[bestIdx] = pMP */
            nmatches++;
        }
    }
    free(cnt); free(cellOf); free(cells); free(fill); free(claimed);
    return nmatches;
}

/* ---- §8f row 3: the pose-projection searches (SearchByProjection x3, Fuse x2) ----
 * Arithmetic conventions (DESIGN.md "Projection arithmetic"):
 *  - cv::Mat 3x3 * 3x1 (+ 3x1) follows OpenCV 3.x gemm's small-matrix path: float products
 *    summed left to right, then the added column; Mat / double is convertTo(alpha = 1./s);
 *    Mat::dot and cv::norm accumulate the float products in double.
 *  - the reference's own float expressions carry the FMAs GCC -O3 -march=native forms.
 *  - (int) conversions of doubles follow x86-64 cvttsd2si (NaN / out of range -> INT_MIN). */
static inline int x86_int(double v)
{
    return (v >= -2147483648.0 && v < 2147483648.0) ? (int)v : INT_MIN;
}

static inline float mat3_row(const float* r, int stride, float x, float y, float z)
{
    return (r[0] * x + r[stride] * y) + r[2 * stride] * z;
}

typedef struct {
    float R[9], t[3], Ow[3];
    int fwd, bwd;
} proj_cam;

static void proj_camera(int mode, const float* pose, const orbref_pose_params* P, proj_cam* c)
{
    if (mode == ORBREF_PROJ_SIM3 || mode == ORBREF_FUSE_SIM3) {   /* Decompose Scw, :298-303 / :1053-1058 */
        double d = 0.0;
        for (int k = 0; k < 3; k++) d += (double)pose[k] * pose[k];
        const float scw = (float)sqrt(d);
        const float s = (float)(1.0 / (double)scw);
        for (int r = 0; r < 3; r++) {
            for (int k = 0; k < 3; k++) c->R[3 * r + k] = pose[4 * r + k] * s + 0.0f;
            c->t[r] = pose[4 * r + 3] * s + 0.0f;
        }
    } else {
        for (int r = 0; r < 3; r++) {
            for (int k = 0; k < 3; k++) c->R[3 * r + k] = pose[4 * r + k];
            c->t[r] = pose[4 * r + 3];
        }
    }
    for (int r = 0; r < 3; r++)   /* Ow = -Rcw.t()*tcw (KeyFrame::SetPose forms GetCameraCenter alike) */
        c->Ow[r] = -mat3_row(c->R + r, 3, c->t[0], c->t[1], c->t[2]);
    c->fwd = c->bwd = 0;
    if (mode == ORBREF_PROJ_LAST_FRAME) {   /* :1406-1417: twc = Ow, tlc = Rlw*twc+tlw */
        const float* L = pose + 12;
        const float tlc2 = mat3_row(L + 8, 1, c->Ow[0], c->Ow[1], c->Ow[2]) + L[11];
        c->fwd = tlc2 > P->b && !P->mono;
        c->bwd = -tlc2 > P->b && !P->mono;
    }
}

/* MapPoint::PredictScale (src/MapPoint.cc:385-417) */
static int predict_scale(float max_dist, float dist, const orbref_pose_params* P)
{
    const float ratio = max_dist / dist;
    int n = x86_int(ceil(log((double)ratio) / (double)P->log_scale));
    if (n < 0) n = 0;
    else if (n >= P->nlevels) n = P->nlevels - 1;
    return n;
}

typedef struct {
    float u, v, r, ur;
    int minLevel, maxLevel;
} proj_win;

/* The per-MapPoint part before the area query; 0 where the reference `continue`s. */
static int proj_point(int mode, const proj_cam* c, const orbref_map_point* M, const orbref_pose_params* P,
                      proj_win* w)
{
    const float X = M->x, Y = M->y, Z = M->z;
    const float xc = mat3_row(c->R, 1, X, Y, Z) + c->t[0];
    const float yc = mat3_row(c->R + 3, 1, X, Y, Z) + c->t[1];
    const float zc = mat3_row(c->R + 6, 1, X, Y, Z) + c->t[2];
    float u, v;
    w->ur = 0.0f;
    if (mode == ORBREF_PROJ_LAST_FRAME || mode == ORBREF_PROJ_KEYFRAME) {
        const float invzc = (float)(1.0 / (double)zc);          /* :1433 / :1570 */
        if (mode == ORBREF_PROJ_LAST_FRAME && invzc < 0) return 0;
        u = fmaf(P->fx * xc, invzc, P->cx);                     /* fx*xc*invzc+cx */
        v = fmaf(P->fy * yc, invzc, P->cy);
        if (u < P->min_x || u > P->max_x) return 0;
        if (v < P->min_y || v > P->max_y) return 0;
        w->u = u;
        w->v = v;
        if (mode == ORBREF_PROJ_LAST_FRAME) {                  /* :1446-1458 */
            const int L = M->octave;
            w->r = P->th * P->scale[L];
            if (c->fwd) { w->minLevel = L; w->maxLevel = -1; }
            else if (c->bwd) { w->minLevel = 0; w->maxLevel = L; }
            else { w->minLevel = L - 1; w->maxLevel = L + 1; }
            w->ur = fmaf(-P->bf, invzc, u);                     /* u - mbf*invzc, :1477 */
            return 1;
        }
    } else {
        if (zc < 0.0f) return 0;
        const float invz = mode == ORBREF_FUSE_SIM3 ? (float)(1.0 / (double)zc) : 1.0f / zc;
        const float x = xc * invz, y = yc * invz;
        u = fmaf(P->fx, x, P->cx);
        v = fmaf(P->fy, y, P->cy);
        if (!(u >= P->min_x && u < P->max_x && v >= P->min_y && v < P->max_y)) return 0;   /* IsInImage */
        w->u = u;
        w->v = v;
        if (mode == ORBREF_FUSE) w->ur = fmaf(-P->bf, invz, u);   /* u-bf*invz, :938 */
    }
    const float maxD = 1.2f * M->max_dist, minD = 0.8f * M->min_dist;   /* Get{Max,Min}DistanceInvariance */
    const float PO[3] = {X - c->Ow[0], Y - c->Ow[1], Z - c->Ow[2]};
    double s = 0.0;
    for (int k = 0; k < 3; k++) s += (double)PO[k] * PO[k];
    const float dist = (float)sqrt(s);                          /* cv::norm(PO) */
    if (dist < minD || dist > maxD) return 0;
    if (mode != ORBREF_PROJ_KEYFRAME) {                        /* viewing angle < 60 deg */
        double dot = 0.0;
        dot += (double)PO[0] * M->nx;
        dot += (double)PO[1] * M->ny;
        dot += (double)PO[2] * M->nz;
        if (dot < 0.5 * dist) return 0;
    }
    const int L = predict_scale(M->max_dist, dist, P);
    w->r = P->th * P->scale[L];
    w->minLevel = L - 1;
    w->maxLevel = mode == ORBREF_PROJ_KEYFRAME ? L + 1 : L;
    return 1;
}

/* Per-candidate tests of each mode other than the claims (level window, area, stereo). */
static int proj_candidate_ok(int mode, const proj_win* w, const orbref_keypoint* kp, float ur,
                             const orbref_pose_params* P)
{
    if (kp->octave < w->minLevel) return 0;
    if (w->maxLevel >= 0 && kp->octave > w->maxLevel) return 0;
    const float distx = kp->x - w->u, disty = kp->y - w->v;
    if (!(fabsf(distx) < w->r && fabsf(disty) < w->r)) return 0;
    if (mode == ORBREF_PROJ_LAST_FRAME && ur > 0) {            /* :1475-1481 */
        const float er = fabsf(w->ur - ur);
        if (er > w->r) return 0;
    }
    if (mode == ORBREF_FUSE) {                                  /* :982-1006 */
        const float ex = w->u - kp->x, ey = w->v - kp->y;
        if (ur >= 0) {
            const float er = w->ur - ur;
            const float e2 = fmaf(er, er, fmaf(ex, ex, ey * ey));
            if ((double)(e2 * P->inv_sigma2[kp->octave]) > 7.8) return 0;
        } else {
            const float e2 = fmaf(ex, ex, ey * ey);
            if ((double)(e2 * P->inv_sigma2[kp->octave]) > 5.99) return 0;
        }
    }
    return 1;
}

int orbref_project_search(int mode, const orbref_keypoint* kps, const uint8_t* desc, const float* uright,
                          const uint8_t* claimed_in, int n, const float* pose, const orbref_map_point* pts,
                          const uint8_t* pdesc, int np, const orbref_pose_params* P, int* match)
{
    const int search = mode <= ORBREF_PROJ_SIM3;
    const int rot = P->check_ori && (mode == ORBREF_PROJ_LAST_FRAME || mode == ORBREF_PROJ_KEYFRAME);
    const int thr = mode == ORBREF_PROJ_LAST_FRAME ? 100 : (mode == ORBREF_PROJ_KEYFRAME ? P->orb_dist : TH_LOW);
    int* cnt = (int*)calloc(GRID_COLS * GRID_ROWS + 1, sizeof(int));   /* AssignFeaturesToGrid */
    int* cellOf = (int*)malloc(sizeof(int) * ((size_t)n + 1));
    for (int i = 0; i < n; i++) {
        const int px = (int)roundf((kps[i].x - P->min_x) * P->grid_w_inv);
        const int py = (int)roundf((kps[i].y - P->min_y) * P->grid_h_inv);
        cellOf[i] = (px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS) ? -1 : px * GRID_ROWS + py;
        if (cellOf[i] >= 0) cnt[cellOf[i] + 1]++;
    }
    for (int c = 0; c < GRID_COLS * GRID_ROWS; c++) cnt[c + 1] += cnt[c];
    int* cells = (int*)malloc(sizeof(int) * ((size_t)n + 1));
    int* fill = (int*)calloc(GRID_COLS * GRID_ROWS, sizeof(int));
    for (int i = 0; i < n; i++)
        if (cellOf[i] >= 0) cells[cnt[cellOf[i]] + fill[cellOf[i]]++] = i;
    uint8_t* claimed = (uint8_t*)calloc((size_t)n + 1, 1);
    if (search)
        for (int i = 0; i < n; i++) { claimed[i] = claimed_in ? claimed_in[i] : 0; match[i] = -1; }
    else
        for (int m = 0; m < np; m++) match[m] = -1;
    int* ent_idx = (int*)malloc(sizeof(int) * ((size_t)np + 1));   /* rotHist entries in push order */
    int* ent_bin = (int*)malloc(sizeof(int) * ((size_t)np + 1));
    int nent = 0, nmatches = 0;
    proj_cam cam;
    proj_camera(mode, pose, P, &cam);

    for (int m = 0; m < np; m++) {
        const orbref_map_point* M = &pts[m];
        if (!(M->flags & 1)) continue;
        proj_win w;
        if (!proj_point(mode, &cam, M, P, &w)) continue;
        /* GetFeaturesInArea cell range (Frame.cc:410-495 / KeyFrame.cc:569-608) */
        const int cx0 = x86_int(floorf((w.u - P->min_x - w.r) * P->grid_w_inv));
        const int nMinCellX = cx0 > 0 ? cx0 : 0;
        if (nMinCellX >= GRID_COLS) continue;
        const int cx1 = x86_int(ceilf((w.u - P->min_x + w.r) * P->grid_w_inv));
        const int nMaxCellX = cx1 < GRID_COLS - 1 ? cx1 : GRID_COLS - 1;
        if (nMaxCellX < 0) continue;
        const int cy0 = x86_int(floorf((w.v - P->min_y - w.r) * P->grid_h_inv));
        const int nMinCellY = cy0 > 0 ? cy0 : 0;
        if (nMinCellY >= GRID_ROWS) continue;
        const int cy1 = x86_int(ceilf((w.v - P->min_y + w.r) * P->grid_h_inv));
        const int nMaxCellY = cy1 < GRID_ROWS - 1 ? cy1 : GRID_ROWS - 1;
        if (nMaxCellY < 0) continue;
        int bestDist = 256, bestIdx = -1;
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
                const int c = ix * GRID_ROWS + iy;
                for (int j = cnt[c]; j < cnt[c + 1]; j++) {
                    const int idx = cells[j];
                    if (!proj_candidate_ok(mode, &w, &kps[idx], uright[idx], P)) continue;
                    if (search && claimed[idx]) continue;
                    const int dist = orbref_descriptor_distance(pdesc + 32 * (size_t)m, desc + 32 * (size_t)idx);
                    if (dist < bestDist) { bestDist = dist; bestIdx = idx; }
                }
            }
        }
        if (bestIdx < 0 || bestDist > thr) continue;
        nmatches++;
        if (!search) { match[m] = bestIdx; continue; }
        match[bestIdx] = m;                                     /* mvpMapPoints[bestIdx] = pMP */
        claimed[bestIdx] = mode != ORBREF_PROJ_LAST_FRAME || (M->flags & 2);
        if (rot) {
            ent_idx[nent] = bestIdx;
            ent_bin[nent] = rot_bin(M->angle, kps[bestIdx].angle);
            nent++;
        }
    }
    if (rot) {   /* :1515-1535 / :1645-1664 */
        int hist[HISTO_LENGTH] = {0};
        for (int e = 0; e < nent; e++) hist[ent_bin[e]]++;
        int a, b, c;
        three_maxima(hist, &a, &b, &c);
        for (int e = 0; e < nent; e++) {
            const int bin = ent_bin[e];
            if (bin == a || bin == b || bin == c) continue;
            match[ent_idx[e]] = -2;                             /* mvpMapPoints[...] = NULL */
            nmatches--;
        }
    }
    free(cnt); free(cellOf); free(cells); free(fill); free(claimed); free(ent_idx); free(ent_bin);
    return nmatches;
}

/* ---- §8f row 4: image ingest (remap INTER_LINEAR + cvtColor to gray, depth convertTo) ---- */

/* cvRound(float) on x86-64 (cvtss2si): ties to even; NaN and out of range give INT_MIN */
static inline int cv_round_x86(float v)
{
    return (v >= -2147483648.0f && v < 2147483648.0f) ? (int)lrintf(v) : INT_MIN;
}

static inline int sat_short(int v) { return v < SHRT_MIN ? SHRT_MIN : (v > SHRT_MAX ? SHRT_MAX : v); }

void orbref_ingest(const uint8_t* src, int rows, int cols, int channels, int rgb, size_t src_step,
                   const float* map_x, const float* map_y, int dst_rows, int dst_cols, uint8_t* dst,
                   size_t dst_step)
{
    /* RGB2Gray<uchar> (color.cpp): tab[src[0]] + tab[src[1]+256] + tab[src[2]+512], the rounding
     * constant folded into the third table; blueIdx 0 (BGR) weights src[0] with B2Y */
    const int w0 = rgb ? 4899 : 1868, w1 = 9617, w2 = rgb ? 1868 : 4899;
    if (!map_x) { dst_rows = rows; dst_cols = cols; }
    for (int y = 0; y < dst_rows; y++) {
        for (int x = 0; x < dst_cols; x++) {
            int val[4] = {0, 0, 0, 0};
            if (map_x) {   /* RemapInvoker: XY = cvRound(m*INTER_TAB_SIZE) >> INTER_BITS, A = fractions */
                const int sx32 = cv_round_x86(map_x[(size_t)y * dst_cols + x] * 32.0f);
                const int sy32 = cv_round_x86(map_y[(size_t)y * dst_cols + x] * 32.0f);
                const int fx = sx32 & 31, fy = sy32 & 31;
                const int sx = sat_short(sx32 >> 5), sy = sat_short(sy32 >> 5);
                /* BilinearTab_i: (1-fy, fy) x (1-fx, fx) in 1/32 steps, scaled by 2^15.  The (0,0) entry
                 * saturates to 32767 in OpenCV; for u8 sources that cannot change a result. */
                const int w00 = (32 - fx) * (32 - fy) * 32, w01 = fx * (32 - fy) * 32;
                const int w10 = (32 - fx) * fy * 32, w11 = fx * fy * 32;
                const int in_x0 = sx >= 0 && sx < cols, in_x1 = sx + 1 >= 0 && sx + 1 < cols;
                const int in_y0 = sy >= 0 && sy < rows, in_y1 = sy + 1 >= 0 && sy + 1 < rows;
                for (int k = 0; k < channels; k++) {   /* remapBilinear, BORDER_CONSTANT cval 0 */
                    const int v00 = in_x0 && in_y0 ? src[(size_t)sy * src_step + (size_t)sx * channels + k] : 0;
                    const int v01 = in_x1 && in_y0 ? src[(size_t)sy * src_step + (size_t)(sx + 1) * channels + k] : 0;
                    const int v10 = in_x0 && in_y1 ? src[(size_t)(sy + 1) * src_step + (size_t)sx * channels + k] : 0;
                    const int v11 = in_x1 && in_y1 ? src[(size_t)(sy + 1) * src_step + (size_t)(sx + 1) * channels + k] : 0;
                    const int s = v00 * w00 + v01 * w01 + v10 * w10 + v11 * w11;
                    val[k] = sat_u8((s + (1 << 14)) >> 15);
                }
            } else {
                for (int k = 0; k < channels; k++) val[k] = src[(size_t)y * src_step + (size_t)x * channels + k];
            }
            const int g = channels == 1 ? val[0] : (val[0] * w0 + val[1] * w1 + val[2] * w2 + (1 << 13)) >> 14;
            dst[(size_t)y * dst_step + x] = (uint8_t)g;
        }
    }
}

void orbref_depth_convert(const void* src, int depth_type, int rows, int cols, size_t src_step, float factor,
                          float* dst, size_t dst_step)
{
    for (int y = 0; y < rows; y++)
        for (int x = 0; x < cols; x++) {
            const uint8_t* row = (const uint8_t*)src + (size_t)y * src_step;
            const float v = depth_type == 0 ? (float)((const uint16_t*)row)[x] : ((const float*)row)[x];
            ((float*)((uint8_t*)dst + (size_t)y * dst_step))[x] = v * factor + 0.0f;   /* cvtScale_, WT = float */
        }
}

/* ---- SURVEY.md 8b orbm_best2_csr: the shared best / second loop over a candidate list ---- */
void orbref_best2_csr(const uint8_t* q, int nq, const uint8_t* t, const int* cand_ptr, const int* cand_idx,
                      int tie_last, int* best_idx, int* best, int* second)
{
    for (int i = 0; i < nq; i++) {
        int bestDist = 256, bestDist2 = 256, bestIdx = -1;
        for (int c = cand_ptr[i]; c < cand_ptr[i + 1]; c++) {
            const int j = cand_idx[c];
            const int dist = orbref_descriptor_distance(q + 32 * (size_t)i, t + 32 * (size_t)j);
            if (dist < bestDist) {                      /* e.g. src/ORBmatcher.cc:214-224 */
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx = j;
            } else {
                if (tie_last && dist == bestDist) bestIdx = j;   /* :806-823 keeps the last <= */
                if (dist < bestDist2) bestDist2 = dist;
            }
        }
        best_idx[i] = bestIdx;
        best[i] = bestDist;
        second[i] = bestDist2;
    }
}
