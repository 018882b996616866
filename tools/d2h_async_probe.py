"""Does hipMemcpyAsync D2H into PAGEABLE host memory block the calling thread (HIP stages
pageable copies)? And what do hipHostRegister / hipHostUnregister of a 200 MB array cost?"""
import ctypes as C
import time

import numpy as np
import torch

hip = C.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
NB = 199065600
dev = torch.empty(NB, dtype=torch.uint8, device="cuda").fill_(1)
a = torch.randn(8192, 8192, device="cuda")
host = np.zeros(NB, dtype=np.uint8)
st = torch.cuda.current_stream().cuda_stream
for trial in range(3):
    for _ in range(20):  # ~ tens of ms of GPU work queued ahead of the copy
        a = a @ a * 1e-4
    t0 = time.perf_counter()
    rc = hip.hipMemcpyAsync(host.ctypes.data, dev.data_ptr(), NB, 2, st)
    t1 = time.perf_counter()
    hip.hipStreamSynchronize(st)
    t2 = time.perf_counter()
    print(f"pageable async D2H rc={rc}: call returned after {1e3 * (t1 - t0):.2f} ms, done after {1e3 * (t2 - t0):.2f} ms")
t0 = time.perf_counter()
rc = hip.hipHostRegister(host.ctypes.data, NB, 0)
t1 = time.perf_counter()
print(f"hipHostRegister 199 MB rc={rc}: {1e3 * (t1 - t0):.2f} ms")
for trial in range(2):
    for _ in range(20):
        a = a @ a * 1e-4
    t0 = time.perf_counter()
    rc = hip.hipMemcpyAsync(host.ctypes.data, dev.data_ptr(), NB, 2, st)
    t1 = time.perf_counter()
    hip.hipStreamSynchronize(st)
    t2 = time.perf_counter()
    print(f"registered async D2H rc={rc}: call returned after {1e3 * (t1 - t0):.2f} ms, done after {1e3 * (t2 - t0):.2f} ms")
torch.cuda.synchronize()
t0 = time.perf_counter()
hip.hipMemcpyAsync(host.ctypes.data, dev.data_ptr(), NB, 2, st)
hip.hipStreamSynchronize(st)
print(f"registered D2H alone: {1e3 * (time.perf_counter() - t0):.2f} ms")
t0 = time.perf_counter()
rc = hip.hipHostUnregister(host.ctypes.data)
print(f"hipHostUnregister rc={rc}: {1e3 * (time.perf_counter() - t0):.2f} ms")
torch.cuda.synchronize()
t0 = time.perf_counter()
hip.hipMemcpyAsync(host.ctypes.data, dev.data_ptr(), NB, 2, st)
hip.hipStreamSynchronize(st)
print(f"pageable D2H alone: {1e3 * (time.perf_counter() - t0):.2f} ms")
