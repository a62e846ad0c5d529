// Resources of the synchronous host entry points (orbx.h's orbm_* / orbv_transform / stereo host
// calls).  Internal, not part of the C ABI.
//
// The reference calls ORBmatcher concurrently from Tracking, LocalMapping and LoopClosing, next to
// the two extractor threads (src/Frame.cc:94-103, src/LocalMapping.cc:215,268,
// src/LoopClosing.cc:265).  A host call therefore must not stall the other threads' streams: no
// hipMalloc / hipFree / hipDeviceSynchronize per call, no legacy null stream, and the caller's
// current device is restored on return.  Each call checks a context out of a process-wide pool
// (a non-blocking stream, a pinned staging buffer and a device buffer that only grow) and hands
// it back on return, so concurrent callers never share a stream and a warm pool allocates nothing.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "../../include/orbx.h"

namespace orbx {

// Valid HIP ordinal?
bool device_ok(int device);

// Switches the calling thread to `device` for one call and restores its current device after
// (an invalid ordinal switches nothing; the call reports ORBX_EDEVICE itself).
class DeviceGuard {
public:
    explicit DeviceGuard(int device)
    {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != device && device_ok(device) && hipSetDevice(device) == hipSuccess)
            prev_ = cur;
    }
    ~DeviceGuard()
    {
        if (prev_ >= 0) hipSetDevice(prev_);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;

private:
    int prev_ = -1;
};

struct HostCtx;

// One synchronous host call.  Usage:
//   HostCall c(device);                      // check a context out of the pool
//   size_t a = c.in(src, bytes) ...;         // input blocks (copied at prepare())
//   size_t o = c.out(bytes) ...;             // device-only blocks (outputs, scratch), after the inputs
//   c.prepare();                             // size the buffers, fill the pinned inputs
//   c.host(a) ...                            // optional: fill or patch an input block (src NULL or not)
//   c.upload();                              // H2D of the input prefix on the call's stream
//   launch ...(c.dev(o), c.stream())
//   c.fetch(o, dst, bytes) ...; c.finish();  // D2H, stream sync, copy out
// Blocks are 64-byte aligned.  Blocks inside the pinned window go through pinned memory; larger
// layouts copy their tail blocks directly from / to the caller's memory, or, for an input block
// without a source (filled through host()), from a host-side staging copy of its own.
// A context's pinned buffer only grows; a replaced one is retired, not freed (hipHostFree waits for
// the whole device, which would stall every other thread's stream).
class HostCall {
public:
    explicit HostCall(int device);
    ~HostCall();
    HostCall(const HostCall&) = delete;
    HostCall& operator=(const HostCall&) = delete;

    orbx_status status() const { return st_; }
    hipStream_t stream() const;

    size_t in(const void* src, size_t bytes);
    size_t out(size_t bytes);
    orbx_status prepare();
    uint8_t* host(size_t off);         // staged copy of the input block at off (prepare() first)
    orbx_status upload();
    uint8_t* dev(size_t off) const;
    template <class T>
    T* dev_as(size_t off) const { return reinterpret_cast<T*>(dev(off)); }
    void fetch(size_t off, void* dst, size_t bytes);
    orbx_status finish();

private:
    struct Block {
        size_t off, bytes;
        const void* src;
        int stage;   // index into staged_ for a source-less block past the pinned window, else -1
    };
    struct Fetch {
        size_t off, bytes;
        void* dst;
    };
    DeviceGuard guard_;
    HostCtx* ctx_ = nullptr;
    orbx_status st_ = ORBX_OK;
    size_t end_ = 0, in_end_ = 0;
    bool outs_started_ = false;
    std::vector<Block> ins_;
    std::vector<Fetch> fetches_;
    std::vector<std::vector<uint8_t>> staged_;
    size_t pin_ = 0;   // pinned window: blocks ending at or below it are staged through pinned memory
    bool queued_ = false;
};

}  // namespace orbx
