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


# ---- Java's corrupt-data rules (orcg_rle_decoder_create_java) --------------
# The runs below are hand-built; the expected values are restated from
# RunLengthIntegerReaderV2.java (readDeltaValues :86-147,
# readPatchedBaseValues :149-260) by java_run() with Java's long semantics
# (64-bit two's complement, shifts by the count mod 64).

def _java_widths(code):
    return code + 1 if code < 24 else [26, 28, 30, 32, 40, 48, 56, 64][code - 24]


def _java_closest(n):
    if n == 0:
        return 1
    for w in (24, 26, 28, 30, 32, 40, 48, 56):
        if n <= w:
            return n if w == 24 else w
    return 64


def _s64(x):
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


def _read_ints(buf, p, n, bits):
    """SerializationUtils.readInts: n big-endian `bits`-bit fields from byte p."""
    out, acc, have = [], 0, 0
    for _ in range(max(n, 0)):
        while have < bits:
            acc = (acc << 8) | buf[p]
            p += 1
            have += 8
        out.append((acc >> (have - bits)) & ((1 << bits) - 1))
        have -= bits
        acc &= (1 << have) - 1
    return out, p


def _varint(buf, p):
    v, sh = 0, 0
    while True:
        b = buf[p]
        p += 1
        v |= (b & 0x7F) << sh
        sh += 7
        if b < 0x80:
            return v, p


def java_run(buf, p, signed, skip_corrupt):
    """One run of RunLengthIntegerReaderV2.readValues: (values, next byte) or
    raises ValueError with the Java exception's message."""
    fb = buf[p]
    kind = fb >> 6
    if kind == 0:  # readShortRepeatValues
        size, n = ((fb >> 3) & 7) + 1, (fb & 7) + 3
        v = int.from_bytes(bytes(buf[p + 1:p + 1 + size]), "big")
        if signed:
            v = (v >> 1) ^ -(v & 1)
        return [v] * n, p + 1 + size
    if kind == 3:  # readDeltaValues
        fbw = (fb >> 1) & 0x1F
        fbw = _java_widths(fbw) if fbw else 0
        ln = ((fb & 1) << 8) | buf[p + 1]  # no + 1 in Java
        first, q = _varint(buf, p + 2)
        if signed:
            first = (first >> 1) ^ -(first & 1)
        out = [first]
        db, q = _varint(buf, q)
        db = (db >> 1) ^ -(db & 1)
        if fbw == 0:
            out += [first + db * (k + 1) for k in range(ln)]
            return [_s64(x) for x in out], q
        out.append(first + db)
        ln -= 1
        ds, q = _read_ints(buf, q, ln, fbw)
        for d in ds:
            out.append(out[-1] - d if db < 0 else out[-1] + d)
        return [_s64(x) for x in out], q
    assert kind == 2, "test runs are SHORT_REPEAT / DELTA / PATCHED_BASE"
    fbw = _java_widths((fb >> 1) & 0x1F)
    ln = (((fb & 1) << 8) | buf[p + 1]) + 1
    third, fourth = buf[p + 2], buf[p + 3]
    bw, pw = ((third >> 5) & 7) + 1, _java_widths(third & 0x1F)
    pgw, pl = ((fourth >> 5) & 7) + 1, fourth & 0x1F
    base = int.from_bytes(bytes(buf[p + 4:p + 4 + bw]), "big")
    mask = 1 << (bw * 8 - 1)
    if base & mask:
        base = -(base & ~mask)
    unpacked, q = _read_ints(buf, p + 4 + bw, ln, fbw)
    if pw + pgw > 64 and not skip_corrupt:
        raise ValueError("Corruption in ORC data encountered. To skip reading corrupted data, "
                         "set hive.exec.orc.skip.corrupt.data to true")
    patches, q = _read_ints(buf, q, pl, _java_closest(pw + pgw))
    if pl == 0:
        raise ValueError("Index 0 out of bounds for length 0")
    pmask = ((1 << (pw & 63)) - 1) & ((1 << 64) - 1)  # (1L << pw) - 1

    def gp(k):
        return patches[k] >> (pw & 63), patches[k] & pmask

    idx = 0
    gap, patch = gp(0)
    actual = 0
    while gap == 255 and patch == 0:
        actual += 255
        idx += 1
        gap, patch = gp(idx)
    actual += gap
    out = []
    for i in range(ln):
        if i == actual:
            out.append(base + (unpacked[i] | ((patch << (fbw & 63)) & ((1 << 64) - 1))))
            idx += 1
            if idx < pl:
                gap, patch = gp(idx)
                actual = 0
                while gap == 255 and patch == 0:
                    actual += 255
                    idx += 1
                    gap, patch = gp(idx)
                actual += gap + i
        else:
            out.append(base + unpacked[i])
    return [_s64(x) for x in out], q


def java_stream(buf, signed, skip_corrupt):
    out, p = [], 0
    while p < len(buf):
        v, p = java_run(buf, p, signed, skip_corrupt)
        out += v
    return out


SR5 = bytes([0x00, 0x0A])  # SHORT_REPEAT: 3 x 5 (signed)
# PATCHED_BASE, W = 8, 4 values, base 5, pw = 64 (code 31), pgw = 2, pl = 2:
# pw + pgw > 64; entries 3 and 1000 (64 bits each: getClosestFixedBits(66))
PATCHED_PW64 = (bytes([0x80 | (7 << 1), 3, (0 << 5) | 31, (1 << 5) | 2, 0x05, 1, 2, 3, 4]) +
                (3).to_bytes(8, "big") + (1000).to_bytes(8, "big"))
# PATCHED_BASE with pl == 0 (pw = 4, pgw = 1): no patch bytes
PATCHED_PL0 = bytes([0x80 | (7 << 1), 3, (0 << 5) | 3, (0 << 5) | 0, 0x05, 1, 2, 3, 4])
# DELTA, W = 4, length byte 0 (C++: one value, an error), first 100, step -7
DELTA_LEN0 = bytes([0xC0 | (3 << 1), 0x00, 0xC8, 0x01, 0x0D])

JAVA_CASES = [
    ("patched_pw64", PATCHED_PW64 + SR5, "Corrupt PATCHED_BASE encoded data \\(patchBitSize \\+ pgw > 64\\)!"),
    ("patched_pl0", PATCHED_PL0 + SR5, "Corrupt PATCHED_BASE encoded data \\(pl==0\\)!"),
    ("delta_len0", DELTA_LEN0 + SR5, "Illegal run length for delta encoding"),
]


@pytest.mark.parametrize("name,data,cxx_msg", JAVA_CASES, ids=[c[0] for c in JAVA_CASES])
@pytest.mark.parametrize("skip_corrupt", [False, True])
def test_java_corrupt_data_rules(name, data, cxx_msg, skip_corrupt):
    """Java's RunLengthIntegerReaderV2 checks less than RleDecoderV2: with
    skipCorrupt a PATCHED_BASE run with pw + pgw > 64 decodes (otherwise
    Java's IOException text), pl == 0 fails as Java's array index, and a
    one-value DELTA run with a bit width yields two values. The C++-rules
    decoder keeps the reference's ParseErrors on the same bytes."""
    import orc_amd

    try:
        want, err = java_stream(data, True, skip_corrupt), None
    except ValueError as e:
        want, err = None, str(e)
    dec = orc_amd.create_java_rle_decoder(data, True, skip_corrupt=skip_corrupt)
    if err is None:
        got, rep = dec.next_vector_java(len(want))
        assert [int(x) for x in got] == want
        with pytest.raises(orc_amd.ParseError):
            dec.next_vector_java(1)  # past the stream
    else:
        with pytest.raises(orc_amd.ParseError, match=err.replace("(", "\\(").replace(")", "\\)")):
            dec.next_vector_java(4)
    cxx = orc_amd.create_rle_decoder(data, True)
    with pytest.raises(orc_amd.ParseError, match=cxx_msg):
        cxx.next(4)


def test_java_rules_match_cxx_on_good_streams():
    """On the reference's KAT streams (all well-formed) the Java-rules decoder
    gives the C++ decoder's values."""
    import orc_amd

    for fx in RLEV2:
        data = bytes.fromhex(fx["data"])
        n = sum(1 for e in fx["expected"] if e is not None) if fx.get("not_null") is None else \
            sum(1 for m in fx["not_null"] if m)
        a = orc_amd.create_rle_decoder(data, fx["signed"]).next(n)
        b = orc_amd.create_java_rle_decoder(data, fx["signed"], skip_corrupt=True).next(n)
        np.testing.assert_array_equal(a, b, err_msg=fx["name"])
