"""Sweep tools/probes/libhbm_copy.so over launch shapes and buffer sizes (one GPU); prints GB/s per shape."""
import ctypes, os, sys, json
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "probes", "libhbm_copy.so"))
lib.hbm_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                         ctypes.c_void_p]
dev = torch.device("cuda", 0)
st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
res = []
for nbytes in (1 << 30, 4 << 30):
    a = torch.ones(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for blocks in (0, 1024, 2048, 4096, 8192, 16384):
        for unroll in (1, 2, 4, 8):
            for nt in (0, 1):
                f = lambda: lib.hbm_copy(b.data_ptr(), a.data_ptr(), nbytes // 16, blocks, unroll, nt, st)
                f(); torch.cuda.synchronize()
                best = 0
                for rep in range(3):
                    e0.record()
                    for _ in range(10): f()
                    e1.record(); torch.cuda.synchronize()
                    best = max(best, 2.0 * nbytes * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9)
                res.append((round(best), nbytes >> 20, blocks, unroll, nt))
                print(res[-1], flush=True)
    del a, b
res.sort(reverse=True)
print(json.dumps(res[:10]))
