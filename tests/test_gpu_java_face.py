"""The Java face of the decoder through the C ABI: IntegerReader.nextVector
(long[] and int[] overloads) as the JNI shim in INTEGRATION.md would call it,
driven with the reference's RLEv2 known-answer streams and null masks.

Expected vectors come from the Java rules restated below (test code, from
java/core/src/java/org/apache/orc/impl/RunLengthIntegerReaderV2.java):
  nextVector(ColumnVector, long[], int)  :371-396
    - previous.isRepeating && !noNulls && isNull[0]: return, data untouched,
      nothing consumed;
    - else isRepeating = true; data[i] = next() for non-null rows, 1 for null
      rows; isRepeating false once data[0] != data[i] or isNull[0] != isNull[i].
  nextVector(ColumnVector, int[], int)   :399-411
    - noNulls: data[r] = (int) next();
    - else unless (isRepeating && isNull[0]): data[r] = isNull[r] ? 1 : (int) next();
    - isRepeating unchanged.
"""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

RLEV2 = load_golden("kat_rlev2.json")


def java_long(values, pos, data, is_null, is_repeating):
    """RunLengthIntegerReaderV2.nextVector(ColumnVector, long[], int); is_null
    None = noNulls (isNull all false, the ColumnVector contract)."""
    n = len(data)
    no_nulls = is_null is None
    isn = np.zeros(n, bool) if no_nulls else np.asarray(is_null, bool)
    if is_repeating and not no_nulls and isn[0]:
        return data, is_repeating, pos
    rep = True
    for i in range(n):
        if no_nulls or not isn[i]:
            data[i] = values[pos]
            pos += 1
        else:
            data[i] = 1
        if rep and i > 0 and (data[0] != data[i] or isn[0] != isn[i]):
            rep = False
    return data, rep, pos


def java_int(values, pos, data, is_null, is_repeating):
    """RunLengthIntegerReaderV2.nextVector(ColumnVector, int[], int)."""
    n = len(data)
    if is_null is None:
        for r in range(n):
            data[r] = np.int64(values[pos]).astype(np.int32)
            pos += 1
    elif not (is_repeating and is_null[0]):
        for r in range(n):
            if is_null[r]:
                data[r] = 1
            else:
                data[r] = np.int64(values[pos]).astype(np.int32)
                pos += 1
    return data, pos


def _masks(rng, n):
    yield None
    yield np.zeros(n, np.uint8)  # nulls allowed, none present
    yield (rng.random(n) < 0.3).astype(np.uint8)
    m = np.ones(n, np.uint8)
    yield m  # all null
    m2 = (rng.random(n) < 0.5).astype(np.uint8)
    m2[0] = 1
    yield m2  # null first row


@pytest.mark.parametrize("fx", RLEV2, ids=[f["name"] for f in RLEV2])
@pytest.mark.parametrize("batch", [1, 3, 7, 1024])
def test_next_vector_long_matches_java_rules(fx, batch):
    import orc_amd

    from oracle import oracle

    data_bytes = bytes.fromhex(fx["data"])
    # the stream's values in order (the oracle, pinned by these KATs; the
    # fixture's None entries are rows the reference test does not check)
    nn = fx.get("not_null")
    exp = [e for e, m in zip(fx["expected"], nn) if m] if nn is not None else fx["expected"]
    vals = [int(x) for x in oracle.rlev2_decode(data_bytes, len(exp), fx["signed"])]
    for v, e in zip(vals, exp):
        assert e is None or v == e
    rng = np.random.default_rng(len(vals) * 31 + batch)
    for mask_seed, mask_all in enumerate(_masks(rng, 4 * len(vals) + 16)):
        dec = orc_amd.create_rle_decoder(data_bytes, fx["signed"])
        pos, at = 0, 0
        rep = bool(mask_seed % 2)  # start from both isRepeating states
        stale = np.full(batch, -777, dtype=np.int64)
        while pos < len(vals):
            isn = None if mask_all is None else mask_all[at:at + batch]
            if isn is not None and len(isn) < batch:
                isn = np.concatenate([isn, np.zeros(batch - len(isn), np.uint8)])
            # never ask for more non-null values than the stream holds
            need = batch if isn is None else int((isn == 0).sum())
            n = batch
            if pos + need > len(vals):
                if isn is None:
                    n = len(vals) - pos
                else:
                    cnt = np.cumsum(isn == 0)
                    n = int(np.searchsorted(cnt, len(vals) - pos, side="right"))
                    n = max(n, 1)
                    if cnt[n - 1] > len(vals) - pos:
                        break
                if isn is not None:
                    isn = isn[:n]
            want = stale[:n].copy()
            want, want_rep, pos2 = java_long(vals, pos, want, isn, rep)
            got, got_rep = dec.next_vector_java(n, isn, rep, out=stale[:n].copy())
            np.testing.assert_array_equal(got, want, err_msg="%s batch %d at %d" % (fx["name"], batch, at))
            assert got_rep == want_rep, (fx["name"], batch, at)
            rep = got_rep
            pos = pos2
            at += n


@pytest.mark.parametrize("fx", [f for f in RLEV2 if f["name"] in (
    "largeNegativesDirect", "overflowDirect", "bitSize64Direct", "basicDelta0", "shortRepeats")],
    ids=lambda f: f["name"])
def test_next_vector_int_matches_java_rules(fx):
    import orc_amd

    vals = [int(v) for v in fx["expected"] if v is not None]
    rng = np.random.default_rng(5)
    for mask in (None, (rng.random(len(vals) * 2) < 0.4).astype(np.uint8)):
        dec = orc_amd.create_rle_decoder(bytes.fromhex(fx["data"]), fx["signed"])
        pos, at = 0, 0
        while pos < len(vals):
            isn = None if mask is None else mask[at:at + 5]
            n = 5 if isn is None else len(isn)
            if isn is None:
                n = min(n, len(vals) - pos)
            elif int((isn == 0).sum()) > len(vals) - pos:
                break
            want, pos2 = java_int(vals, pos, np.zeros(n, np.int32), isn, False)
            got = dec.next_vector_java_int(n, isn, False)
            np.testing.assert_array_equal(got, want)
            pos, at = pos2, at + n
        # the all-null repeating vector is left untouched and consumes nothing
        dec = orc_amd.create_rle_decoder(bytes.fromhex(fx["data"]), fx["signed"])
        keep = np.full(4, 42, np.int32)
        got = dec.next_vector_java_int(4, np.array([1, 0, 0, 1], np.uint8), True, out=keep.copy())
        np.testing.assert_array_equal(got, keep)
        np.testing.assert_array_equal(dec.next_vector_java_int(1, None), np.int64(vals[:1]).astype(np.int32))


def test_is_repeating_on_repeated_runs():
    """A SHORT_REPEAT run read in one vector is repeating; a null row breaks
    it (isNull[0] != isNull[i]); an all-null vector of 1s is repeating."""
    import orc_amd

    data, _ = orc_amd.encode_runs(np.full(10, 7, np.int64), True, [0], [10])
    dec = orc_amd.create_rle_decoder(data.tobytes(), True)
    v, rep = dec.next_vector_java(4)
    assert rep and list(v) == [7] * 4
    v, rep = dec.next_vector_java(3, np.array([0, 1, 0], np.uint8))
    assert not rep and list(v) == [7, 1, 7]
    v, rep = dec.next_vector_java(3, np.array([1, 1, 1], np.uint8), False)
    assert rep and list(v) == [1, 1, 1]
    v, rep = dec.next_vector_java(2)
    assert rep and list(v) == [7, 7]
