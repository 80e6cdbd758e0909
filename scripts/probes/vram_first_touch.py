#!/usr/bin/env python3
"""First-touch cost of fresh device memory (hipMalloc) under host<->device
copies: H2D into a fresh buffer twice, H2D into a fresh buffer cleared first
by hipMemset, and D2H out of a fresh buffer that kernels wrote. One JSON
line (ms)."""
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
hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
hip.hipDeviceSynchronize.argtypes = []
N = 256 << 20
h = L.orcg_host_alloc(N)
out = {}


def fresh():
    d = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(d), N) == 0
    return d.value


def t(fn):
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    fn()
    hip.hipDeviceSynchronize()
    return round((time.perf_counter() - t0) * 1e3, 2)


w = fresh()
out["warmup_h2d_ms"] = t(lambda: hip.hipMemcpy(w, h, N, 1))
d1 = fresh()
out["h2d_fresh_ms"] = t(lambda: hip.hipMemcpy(d1, h, N, 1))
out["h2d_again_ms"] = t(lambda: hip.hipMemcpy(d1, h, N, 1))
d2 = fresh()
out["memset_fresh_ms"] = t(lambda: hip.hipMemset(d2, 0, N))
out["h2d_after_memset_ms"] = t(lambda: hip.hipMemcpy(d2, h, N, 1))
d3 = fresh()
out["d2h_fresh_unwritten_ms"] = t(lambda: hip.hipMemcpy(h, d3, N, 2))
out["d2h_again_ms"] = t(lambda: hip.hipMemcpy(h, d3, N, 2))
print(json.dumps(out))
