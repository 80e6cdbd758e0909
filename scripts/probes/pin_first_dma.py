#!/usr/bin/env python3
"""First-DMA cost of freshly allocated pinned host memory (orcg_host_alloc:
anonymous THP mapping + hipHostRegister): times a 320 MB D2H into a new
buffer twice, then into another new buffer after a sparse 'touch' (one small
D2H per 2 MB), and the same for H2D. One JSON line."""
import ctypes
import json
import time

import orc_amd

L = orc_amd._lib.load()
L.orcg_host_alloc.restype = ctypes.c_void_p
L.orcg_host_alloc.argtypes = [ctypes.c_uint64]
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipDeviceSynchronize.argtypes = []
N = 320 << 20
d = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(d), N) == 0
out = {}


def t(dst, src, n, kind):
    t0 = time.perf_counter()
    assert hip.hipMemcpy(dst, src, n, kind) == 0
    return round((time.perf_counter() - t0) * 1e3, 2)


for name, kind in (("d2h", 2), ("h2d", 1)):
    a = L.orcg_host_alloc(N + (32 << 20))
    dst, src = (a, d.value) if kind == 2 else (d.value, a)
    out[name + "_first_ms"] = t(dst, src, N, kind)
    out[name + "_second_ms"] = t(dst, src, N, kind)
    c = L.orcg_host_alloc(N + (32 << 20))
    dst, src = (c, d.value) if kind == 2 else (d.value, c)
    out[name + "_fresh_no_touch_ms"] = t(dst, src, N, kind)
    out[name + "_fresh_no_touch_second_ms"] = t(dst, src, N, kind)
    b = L.orcg_host_alloc(N + (32 << 20))
    t0 = time.perf_counter()
    for off in range(0, N, 2 << 20):
        if kind == 2:
            hip.hipMemcpy(b + off, d.value, 4096, 2)
        else:
            hip.hipMemcpy(d.value, b + off, 4096, 1)
    out[name + "_touch_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    dst, src = (b, d.value) if kind == 2 else (d.value, b)
    out[name + "_after_touch_ms"] = t(dst, src, N, kind)
print(json.dumps(out))
