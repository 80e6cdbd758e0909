"""Parity at BASELINE.json's full C2 size (configs[1]: 10^8 full-range int64
values, RLEv2 DIRECT W=64 runs of 512, row-index stride 10,000) through
size-independent properties, on the default kernel and on each pinned
instance the default can launch:

  * round trip: decode(encode(v)) == v for every value (the same generator
    and seed as bench.py's stream);
  * seek / row ranges: decoding value windows [b, b + n) that start inside
    a run (RleDecoderV2::seek + skip, c++/src/RleDecoderV2.cc:109-130) gives
    exactly v[b : b + n];
  * idempotence: a second decode into a buffer pre-filled with garbage
    gives the same bytes.

The oracle is checked against the reference's known answers on small cases
(tests/test_oracle_golden.py); here the writer's input is the expected
output.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROWS, STRIDE = 100_000_000, 10_000


@pytest.fixture(scope="module")
def c2():
    import torch

    import orc_amd

    rng = np.random.default_rng(42)  # bench.py make_stream
    v = rng.integers(-(1 << 63), (1 << 63) - 1, size=ROWS, dtype=np.int64, endpoint=True)
    data, pos = orc_amd.encode_direct(v, True, aligned=True, rows_per_group=STRIDE)
    d = {"v": torch.from_numpy(v).cuda(), "src": torch.from_numpy(data).cuda(),
         "pos": torch.from_numpy(pos.view(np.int64)).cuda(), "S": int(data.size)}
    yield d
    del d
    torch.cuda.empty_cache()


@pytest.mark.parametrize("variant", [0, 2, 3, 4, 6, 7])
def test_c2_full_roundtrip(c2, variant):
    import torch

    import orc_amd

    ctx = orc_amd.default_context(0)
    ctx.set_rlev2_variant(variant)
    try:
        out = torch.full((ROWS,), -7, dtype=torch.int64, device="cuda")
        orc_amd.decode_positions_device(ctx, c2["src"], c2["pos"], STRIDE, ROWS, True, out)
        ctx.synchronize()
        assert torch.equal(out, c2["v"])
        # idempotent: decode again over the decoded buffer
        out[::977] = 123
        orc_amd.decode_positions_device(ctx, c2["src"], c2["pos"], STRIDE, ROWS, True, out)
        ctx.synchronize()
        assert torch.equal(out, c2["v"])
    finally:
        ctx.set_rlev2_variant(0)


@pytest.mark.parametrize("begin,count", [(0, 1), (511, 2), (9_999, 10_002), (12_345_677, 1_000_001),
                                         (ROWS - 513, 513), (ROWS - 1, 1), (50_000_000, 50_000_000)])
def test_c2_full_value_windows(c2, begin, count):
    import torch

    import orc_amd

    ctx = orc_amd.default_context(0)
    out = torch.full((count,), -7, dtype=torch.int64, device="cuda")
    orc_amd.decode_positions_device(ctx, c2["src"], c2["pos"], STRIDE, count, True, out, value_begin=begin)
    ctx.synchronize()
    assert torch.equal(out, c2["v"][begin:begin + count])
