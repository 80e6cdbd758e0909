"""CPU-only tests of liborcgpu's host logic: the C ABI exports, the writer-side
encoder (checked by decoding with the oracle) and the host run planner.
No GPU calls are made here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from oracle import oracle
from orc_amd import _lib
import orc_amd

HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include")))
           if h.endswith(".h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(orcg_\w+)\s*\(", text))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    declared = declared_functions()
    assert len(declared) >= 25
    bound = {name for name, _, _ in _lib.SIGNATURES}
    for name in declared:
        assert hasattr(L, name), "liborcgpu.so does not export %s" % name
        assert name in bound, "orc_amd._lib has no signature for %s" % name


def test_device_count_never_aborts():
    # No GPU in the build container: must return 0 rather than crash.
    assert _lib.load().orcg_device_count() >= 0


def test_no_cpu_fallback_without_device():
    if _lib.load().orcg_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(orc_amd.DeviceError):
        orc_amd.Context(0)


@pytest.mark.parametrize("signed", [True, False])
@pytest.mark.parametrize("bits,aligned", [(1, False), (3, False), (13, False), (13, True), (28, False),
                                          (41, True), (64, True), (64, False)])
def test_encode_direct_roundtrip_via_oracle(signed, bits, aligned):
    rng = np.random.default_rng(bits * 7 + signed)
    n = 5000
    hi = (1 << (bits - 1)) if signed else (1 << bits) - 1
    if bits == 64:
        v = rng.integers(-(1 << 63), (1 << 63) - 1, size=n, dtype=np.int64, endpoint=True)
        if not signed:
            v = v  # any 64-bit pattern
    elif signed:
        v = rng.integers(-hi, hi, size=n, dtype=np.int64)
    else:
        v = rng.integers(0, hi, size=n, dtype=np.int64, endpoint=True)
    data, pos = orc_amd.encode_direct(v, signed, aligned=aligned, rows_per_group=1000)
    got = oracle.rlev2_decode(data.tobytes(), n, signed)
    np.testing.assert_array_equal(got, v)
    # positions behave like RleDecoderV2::seek (RleDecoderV2.cc:109-117)
    for g in range(pos.shape[0]):
        d = oracle.RleDecoderV2(data.tobytes(), signed)
        d.seek(int(pos[g, 0]), int(pos[g, 1]))
        np.testing.assert_array_equal(d.next(10), v[g * 1000: g * 1000 + 10])


def _mixed_stream(rng, signed, nruns=200):
    vals, kinds, lens = [], [], []
    for _ in range(nruns):
        k = rng.integers(0, 4)
        if k == 0:
            L = int(rng.integers(3, 11))
            x = int(rng.integers(-1000, 1000)) if signed else int(rng.integers(0, 1 << 40))
            vals += [x] * L
        elif k == 1:
            L = int(rng.integers(1, 513))
            w = int(rng.integers(1, 63))
            lo = -(1 << (w - 1)) if signed else 0
            vals += list(rng.integers(lo, 1 << (w - 1), size=L))
        elif k == 2:
            L = int(rng.integers(20, 513))
            base = int(rng.integers(-5000, 5000)) if signed else int(rng.integers(0, 5000))
            x = base + rng.integers(0, 200, size=L)
            npatch = int(rng.integers(1, 6))
            idx = rng.choice(L, size=npatch, replace=False)
            x[idx] += rng.integers(1 << 20, 1 << 30, size=npatch)
            vals += list(x)
        else:
            L = int(rng.integers(1, 513))
            start = int(rng.integers(-10 ** 6, 10 ** 6)) if signed else int(rng.integers(0, 10 ** 6))
            if rng.integers(0, 2):
                step = int(rng.integers(-50, 50))
                x = start + step * np.arange(L)
            else:
                d = rng.integers(0, 1000, size=L)
                d[0] = 0
                x = start + np.cumsum(d) * (1 if rng.integers(0, 2) else -1)
                if L > 1 and x[1] == x[0]:
                    x[1:] += 1 if (L < 3 or x[2] >= x[1]) else -1
            vals += list(x)
        kinds.append(int(k))
        lens.append(L)
    return np.array(vals, dtype=np.int64), kinds, lens


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("signed", [True, False])
def test_encode_runs_roundtrip_via_oracle(seed, signed):
    rng = np.random.default_rng(seed)
    for _ in range(20):
        v, kinds, lens = _mixed_stream(rng, signed)
        try:
            data, offs = orc_amd.encode_runs(v, signed, kinds, lens)
        except orc_amd.OrcError:
            continue  # an unrepresentable random draw; try again
        got = oracle.rlev2_decode(data.tobytes(), v.size, signed)
        np.testing.assert_array_equal(got, v)
        return
    pytest.fail("no representable stream drawn")


def test_plan_matches_oracle_count_and_segments():
    rng = np.random.default_rng(3)
    v, kinds, lens = _mixed_stream(rng, True, nruns=400)
    data, offs = orc_amd.encode_runs(v, True, kinds, lens)
    plan = orc_amd.Plan(data.tobytes(), max_segment_bytes=512, max_segment_values=700)
    assert plan.values == v.size == oracle.rlev2_count(data.tobytes(), True)
    assert plan.error() is None
    segs = plan.segments()
    run_starts = {int(o): int(s) for o, s in zip(offs, np.concatenate([[0], np.cumsum(lens)[:-1]]))}
    assert segs[0, 0] == 0
    for b, vi in segs:
        assert run_starts[int(b)] == int(vi)  # every cut is a run start with its value index


def test_plan_reports_first_corrupt_run():
    good, _ = orc_amd.encode_direct(np.arange(600, dtype=np.int64), False)
    bad = good.tobytes() + bytes([0x8E, 0x09, 0x2B, 0x20])  # PATCHED_BASE with pl == 0
    plan = orc_amd.Plan(bad)
    assert plan.values == 600
    rc, at, msg = plan.error()
    assert rc == _lib.ORCG_PARSE_ERROR and at == 600 and "pl==0" in msg
    trunc = good.tobytes()[:-3]
    rc, at, msg = orc_amd.Plan(trunc).error()
    assert at == 512 and msg == "bad read in RleDecoderV2::readByte"
