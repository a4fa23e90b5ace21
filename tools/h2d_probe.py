"""H2D upload A/B: the bench's raw-frame upload -- one
4K I420 frame (12.4 MB) per copy from pinned host memory -- issued three ways,
GB/s for each:
  torch   : tensor.copy_(pinned, non_blocking=True) on a side stream (bench.py)
  hip     : hipMemcpyAsync(HostToDevice) on a non-blocking stream
  hip_sdma: hipMemcpyAsync with the copy marked for the DMA engine
            (hipMemcpyDeviceToDeviceNoCU is D2D only; for H2D the engine is
            chosen by the runtime -- see the rocprof kernel trace for blit
            dispatches)
Usage: python3 tools/h2d_probe.py [NCOPIES]
Run under `rocprofv3 --kernel-trace --stats` to count the blit kernels."""
import ctypes as C
import sys
import time

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
FS = 3840 * 2160 * 3 // 2
dev = torch.device("cuda", 0)
host = torch.empty((8, FS), dtype=torch.uint8).pin_memory()
host.random_(0, 255)
dst = torch.empty((N, FS), dtype=torch.uint8, device=dev)
hip = C.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]


def run_torch():
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        for i in range(N):
            dst[i].copy_(host[i % 8], non_blocking=True)
    s.synchronize()


st = C.c_void_p()
assert hip.hipStreamCreateWithFlags(C.byref(st), 1) == 0


def run_hip():
    for i in range(N):
        rc = hip.hipMemcpyAsync(dst[i].data_ptr(), host[i % 8].data_ptr(), FS, 1, st)
        assert rc == 0, rc
    assert hip.hipStreamSynchronize(st) == 0


for name, fn in (("torch", run_torch), ("hip", run_hip)):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    print("%-6s %d x %.1f MB: %.2f ms, %.1f GB/s" % (name, N, FS / 1e6, dt * 1e3, N * FS / dt / 1e9), flush=True)
ok = bool((dst[N - 1].cpu() == host[(N - 1) % 8]).all())
print("content ok:", ok)
