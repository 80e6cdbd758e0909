import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# pyarrow (the file-level checker) resolves ORC writer zones under $TZDIR;
# the image has no system tzdata: use the IANA files of the `tzdata` Python
# package when it is installed, else the UTC zones of tests/tzdata.py
if "TZDIR" not in os.environ:
    _tzd = None
    try:
        import importlib.util

        _spec = importlib.util.find_spec("tzdata")
        if _spec and _spec.origin:
            _cand = os.path.join(os.path.dirname(_spec.origin), "zoneinfo")
            if os.path.exists(os.path.join(_cand, "GMT")):
                _tzd = _cand
    except Exception:
        _tzd = None
    if _tzd is None:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from utc_zones import utc_tzdir

        _tzd = utc_tzdir()
    os.environ["TZDIR"] = _tzd


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def decode_batches(dec_next, expected, batch, not_null=None):
    """Read len(expected) values through a stateful next(n, notNull) in
    batches, as the reference checkResults/decodeRLEv2 helpers do
    (c++/test/TestRleDecoder.cc:30-56)."""
    total = len(expected)
    b = total if batch is None else batch
    out = []
    i = 0
    while i < total:
        k = min(b, total - i)
        nn = None if not_null is None else not_null[i:i + k]
        out.extend(int(v) for v in dec_next(k, nn))
        i += k
    return out


def assert_matches(expected, got, not_null=None, ctx=""):
    assert len(expected) == len(got), ctx
    for i, e in enumerate(expected):
        if e is None or (not_null is not None and not not_null[i]):
            continue
        assert e == got[i], "%s: mismatch at %d: expected %d got %d" % (ctx, i, e, got[i])
