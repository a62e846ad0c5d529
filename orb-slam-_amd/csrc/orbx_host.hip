// Pooled per-call resources of the synchronous host entry points (see orbx_host.hpp).
#include "orbx_host.hpp"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>

namespace orbx {

namespace {

constexpr size_t kAlign = 64;
constexpr size_t kPinnedMax = (size_t)64 << 20;   // larger layouts copy their tail blocks directly

size_t round_up(size_t v) { return (v + kAlign - 1) & ~(kAlign - 1); }

size_t grow_to(size_t need)
{
    size_t s = (size_t)1 << 16;
    while (s < need) s <<= 1;
    return s;
}

}  // namespace

struct HostCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t* pinned = nullptr;
    size_t pinned_size = 0;
    uint8_t* dbuf = nullptr;
    size_t dbuf_size = 0;
};

namespace {

// Contexts live for the whole process: they are never destroyed, so no HIP call runs during
// exit-time teardown.  The pool grows to the largest number of concurrent host calls.
std::mutex g_pool_mu;
std::vector<HostCtx*>* g_pool = nullptr;
// Pinned buffers a context outgrew.  hipHostFree waits for the whole device (every stream), so a
// growing host call would stall the other threads' work; the buffers are kept until the process
// ends instead (geometric growth: together less than the final buffer).
std::vector<uint8_t*>* g_retired = nullptr;

HostCtx* acquire(int device)
{
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (!g_pool) g_pool = new std::vector<HostCtx*>();
        for (size_t i = g_pool->size(); i-- > 0;) {
            HostCtx* c = (*g_pool)[i];
            if (c->device == device) {
                g_pool->erase(g_pool->begin() + (std::ptrdiff_t)i);
                return c;
            }
        }
    }
    HostCtx* c = new (std::nothrow) HostCtx();
    if (!c) return nullptr;
    c->device = device;
    // high priority: HIP gives these streams hardware queues apart from the application's
    // default-priority streams, so a host call never queues behind the application's kernels
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
    if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi) != hipSuccess) {
        delete c;
        return nullptr;
    }
    return c;
}

void release(HostCtx* c)
{
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool->push_back(c);
}

}  // namespace

bool device_ok(int device)
{
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && device >= 0 && device < n;
}

HostCall::HostCall(int device) : guard_(device)
{
    if (!device_ok(device)) {
        st_ = ORBX_EDEVICE;
        return;
    }
    ctx_ = acquire(device);
    if (!ctx_) st_ = ORBX_EDEVICE;
}

HostCall::~HostCall()
{
    if (!ctx_) return;
    if (queued_) hipStreamSynchronize(ctx_->stream);   // an error path left work queued: drain before reuse
    release(ctx_);
}

hipStream_t HostCall::stream() const { return ctx_ ? ctx_->stream : nullptr; }

size_t HostCall::in(const void* src, size_t bytes)
{
    // inputs come first so that one copy uploads them all
    if (outs_started_) st_ = ORBX_EINVAL;
    const size_t off = end_;
    ins_.push_back({off, bytes, src, -1});
    end_ = round_up(off + bytes);
    in_end_ = end_;
    return off;
}

size_t HostCall::out(size_t bytes)
{
    outs_started_ = true;
    const size_t off = end_;
    end_ = round_up(off + bytes);
    return off;
}

orbx_status HostCall::prepare()
{
    if (st_ != ORBX_OK) return st_;
    const size_t total = std::max(end_, kAlign);
    pin_ = std::min(total, kPinnedMax);
    if (ctx_->pinned_size < pin_) {
        if (ctx_->pinned) {   // rare: the context only grows; retired, never freed (see g_retired)
            std::lock_guard<std::mutex> lk(g_pool_mu);
            if (!g_retired) g_retired = new std::vector<uint8_t*>();
            g_retired->push_back(ctx_->pinned);
        }
        ctx_->pinned = nullptr;
        ctx_->pinned_size = 0;
        const size_t s = grow_to(pin_);
        if (hipHostMalloc((void**)&ctx_->pinned, s, hipHostMallocDefault) != hipSuccess) return st_ = ORBX_ENOMEM;
        ctx_->pinned_size = s;
    }
    if (ctx_->dbuf_size < total) {
        if (ctx_->dbuf) hipFreeAsync(ctx_->dbuf, ctx_->stream);   // stream-ordered: no device-wide sync
        ctx_->dbuf = nullptr;
        ctx_->dbuf_size = 0;
        const size_t s = grow_to(total);
        if (hipMallocAsync((void**)&ctx_->dbuf, s, ctx_->stream) != hipSuccess) return st_ = ORBX_ENOMEM;
        ctx_->dbuf_size = s;
        queued_ = true;
    }
    for (Block& b : ins_) {
        if (b.src && b.bytes && b.off + b.bytes <= pin_) std::memcpy(ctx_->pinned + b.off, b.src, b.bytes);
        if (!b.src && b.bytes && b.off + b.bytes > pin_) {   // filled through host(): its own staging copy
            b.stage = (int)staged_.size();
            staged_.emplace_back(b.bytes);
        }
    }
    return ORBX_OK;
}

uint8_t* HostCall::host(size_t off)
{
    if (!ctx_ || st_ != ORBX_OK) return nullptr;
    for (const Block& b : ins_) {
        if (b.off != off) continue;
        if (b.off + b.bytes <= pin_) return ctx_->pinned + off;
        return b.stage >= 0 ? staged_[(size_t)b.stage].data() : nullptr;
    }
    return nullptr;
}

uint8_t* HostCall::dev(size_t off) const { return ctx_ ? ctx_->dbuf + off : nullptr; }

orbx_status HostCall::upload()
{
    if (st_ != ORBX_OK) return st_;
    const size_t head = std::min(in_end_, pin_);
    queued_ = true;
    if (head && hipMemcpyAsync(ctx_->dbuf, ctx_->pinned, head, hipMemcpyHostToDevice, ctx_->stream) != hipSuccess)
        return st_ = ORBX_EDEVICE;
    for (const Block& b : ins_) {   // blocks past the pinned window: straight from the caller's memory
        const void* from = b.src ? b.src : b.stage >= 0 ? (const void*)staged_[(size_t)b.stage].data() : nullptr;
        if (from && b.bytes && b.off + b.bytes > pin_ &&
            hipMemcpyAsync(ctx_->dbuf + b.off, from, b.bytes, hipMemcpyHostToDevice, ctx_->stream) != hipSuccess)
            return st_ = ORBX_EDEVICE;
    }
    return ORBX_OK;
}

void HostCall::fetch(size_t off, void* dst, size_t bytes)
{
    if (bytes && dst) fetches_.push_back({off, bytes, dst});
}

orbx_status HostCall::finish()
{
    if (st_ != ORBX_OK) return st_;
    queued_ = true;
    for (const Fetch& f : fetches_) {
        void* to = f.off + f.bytes <= pin_ ? (void*)(ctx_->pinned + f.off) : f.dst;
        if (hipMemcpyAsync(to, ctx_->dbuf + f.off, f.bytes, hipMemcpyDeviceToHost, ctx_->stream) != hipSuccess)
            return st_ = ORBX_EDEVICE;
    }
    if (hipStreamSynchronize(ctx_->stream) != hipSuccess) return st_ = ORBX_EDEVICE;
    queued_ = false;
    for (const Fetch& f : fetches_)
        if (f.off + f.bytes <= pin_) std::memcpy(f.dst, ctx_->pinned + f.off, f.bytes);
    fetches_.clear();
    return ORBX_OK;
}

}  // namespace orbx
