#!/usr/bin/env python3
"""Host read bandwidth of pinned (orcg_host_alloc = hipHostMalloc) vs pageable
memory: the RowReader's batches are copied out of a pinned host slab, so a
slow CPU read path there would bound RowReader::next."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bw(src, dst, reps=20):
    np.copyto(dst, src)
    t = time.perf_counter()
    for _ in range(reps):
        np.copyto(dst, src)
    return src.nbytes * reps / (time.perf_counter() - t) / 1e9


def main():
    import torch  # noqa: F401  (HIP runtime first)

    import orc_amd

    L = orc_amd._lib.load()
    n = 256 << 20
    p = L.orcg_host_alloc(n)
    pinned = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p))
    pinned[:] = 7
    page = np.full(n, 7, dtype=np.uint8)
    dst = np.empty(n, dtype=np.uint8)
    small = 128 << 10
    out = {"pinned_to_pageable_GBps": round(bw(pinned, dst, 5), 2), "pageable_to_pageable_GBps": round(bw(page, dst, 5), 2)}
    # batch-sized copies walking through the buffer (the RowReader pattern)
    for name, src in (("pinned", pinned), ("pageable", page)):
        d = np.empty(small, dtype=np.uint8)
        t = time.perf_counter()
        k = 0
        for off in range(0, n - small, small):
            np.copyto(d, src[off:off + small])
            k += 1
        out["%s_128KB_batches_GBps" % name] = round(k * small / (time.perf_counter() - t) / 1e9, 2)
    L.orcg_host_free(ctypes.c_void_p(p))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
