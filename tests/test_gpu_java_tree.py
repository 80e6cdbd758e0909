"""The Java tree-reader face through the C ABI (include/orcg.h "Java
TreeReader face"): TreeReader.nextVector's PRESENT handling and
StringDictionaryTreeReader's BytesColumnVector.setRef references, as the JNI
shim in INTEGRATION.md would call them, driven with the reference's boolean
RLE known-answer streams (c++/test/TestByteRle.cc) and with dictionary
columns built here.

Expected vectors come from the Java rules restated below (test code, from
java/core/src/java/org/apache/orc/impl/TreeReaderFactory.java):
  TreeReader.nextVector                       :405-441
    - PRESENT stream or parent isNull: noNulls = true, allNull = true; per row
      a null parent -> null; else BitFieldReader.next() != 1 -> null
      (BitFieldReader.java:51-57, MSB-first bits); isRepeating = !noNulls &&
      allNull;
    - neither: noNulls = true, isNull all false, isRepeating unchanged.
  StringDictionaryTreeReader.readDictionaryByteArray  :2396-2466
    - scratch nextVector (RunLengthIntegerReaderV2.java:371-396, the rules of
      tests/test_gpu_java_face.py) with isNull / noNulls / isRepeating of the
      result;
    - not repeating: non-null row -> setRef(dict, offsets[idx],
      getDictionaryEntryLength(idx)), null row -> setRef(dict, 0, 0);
    - repeating: row 0 only, isRepeating = true;
    - getDictionaryEntryLength (:2468-2478): idx < offsets.length - 1 ?
      offsets[idx + 1] - offsets[idx] : buffer.length - offsets[idx];
    - dictionaryBuffer == null: offsets null -> one repeating null row; else
      non-null rows -> the empty string.
"""
import numpy as np
import pytest

from conftest import load_golden
from test_gpu_byterle_columns import byte_rle_encode
from test_gpu_java_face import java_long

pytestmark = pytest.mark.gpu

BOOL = load_golden("kat_boolrle.json")


def java_present(bits, pos, parent_is_null, batch, is_repeating, has_present=True):
    """TreeReader.nextVector; bits = the PRESENT stream's bits in order."""
    is_null = np.zeros(batch, np.uint8)
    if not has_present and parent_is_null is None:
        return is_null, True, is_repeating, pos
    no_nulls, all_null = True, True
    for i in range(batch):
        if parent_is_null is None or not parent_is_null[i]:
            if has_present:
                b = bits[pos]
                pos += 1
            else:
                b = 1
            if b != 1:
                no_nulls = False
                is_null[i] = 1
            else:
                all_null = False
        else:
            no_nulls = False
            is_null[i] = 1
    return is_null, no_nulls, (not no_nulls) and all_null, pos


def java_dictionary(values, pos, offsets, buffer_len, is_null, no_nulls, is_repeating, scratch, start, length,
                    has_buffer=True):
    """readDictionaryByteArray (no filter); scratch / start / length are the
    caller's persistent arrays (updated in place)."""
    batch = len(is_null)
    if not has_buffer:
        if offsets is None:
            start[0] = length[0] = 0
            is_null[0] = 1
            return False, True, pos
        for i in range(batch):
            if not is_null[i]:
                start[i] = length[i] = 0
        return no_nulls, is_repeating, pos
    data, rep, pos = java_long(values, pos, scratch, None if no_nulls else is_null, is_repeating)

    def entry(idx):
        off = offsets[idx]
        return off, (offsets[idx + 1] - off) if idx < len(offsets) - 1 else buffer_len - off

    if not rep:
        for i in range(batch):
            start[i], length[i] = entry(int(data[i])) if not is_null[i] else (0, 0)
    else:
        start[0], length[0] = entry(int(data[0]))
    return no_nulls, rep, pos


def _parent_masks(rng, n):
    yield None
    yield (rng.random(n) < 0.4).astype(np.uint8)
    yield np.ones(n, np.uint8)


@pytest.mark.parametrize("fx", BOOL, ids=[f["name"] for f in BOOL])
@pytest.mark.parametrize("batch", [1, 3, 7, 1024])
def test_tree_present_matches_java_rules(fx, batch):
    import orc_amd

    bits = [int(b) for b in fx["expected"]]
    rng = np.random.default_rng(len(bits) + batch)
    for parent_all in _parent_masks(rng, 3 * len(bits) + 8):
        dec = orc_amd.create_boolean_rle_decoder(bytes.fromhex(fx["data"]))
        pos, at, rep = 0, 0, True
        while pos < len(bits) and at < (len(parent_all) if parent_all is not None else 1 << 60):
            par = None if parent_all is None else parent_all[at:at + batch]
            left = len(bits) - pos
            # never read past the stream (the reference raises there)
            if par is None:
                n = min(batch, left)
            else:
                cnt = np.cumsum(par == 0)
                n = int(np.searchsorted(cnt, left, side="right"))
                if n == 0:
                    break
                par = par[:n]
            want = java_present(bits, pos, par, n, rep)
            got = orc_amd.java_tree_present_next(dec, n, par, rep)
            np.testing.assert_array_equal(got[0], want[0], err_msg="%s batch %d at %d" % (fx["name"], batch, at))
            assert got[1:] == want[1:3], (fx["name"], batch, at, got[1:], want[1:3])
            rep, pos, at = got[2], want[3], at + n


def test_tree_present_without_stream_leaves_is_repeating():
    import orc_amd

    for rep in (False, True):
        isn, nn, r = orc_amd.java_tree_present_next(None, 5, None, rep)
        assert nn and r == rep and not isn.any()
    isn, nn, r = orc_amd.java_tree_present_next(None, 4, np.array([1, 1, 1, 1], np.uint8), False)
    assert not nn and r and isn.all()


def _dictionary_column(rng, rows, dict_size, null_frac, repeat_frac):
    """A dictionary string column: per-row indices (runs of one index make
    repeating batches), a PRESENT bitmap, LENGTH values."""
    idx = np.empty(rows, np.int64)
    i = 0
    while i < rows:
        k = int(rng.integers(1, 40))
        if rng.random() < repeat_frac:
            idx[i:i + k] = int(rng.integers(0, dict_size))
        else:
            idx[i:i + k] = rng.integers(0, dict_size, size=min(k, rows - i))[:min(k, rows - i)]
        i += k
    present = (rng.random(rows) >= null_frac).astype(np.uint8)
    lengths = rng.integers(0, 12, size=dict_size)
    return idx, present, lengths


def _pack_bits(present):
    return np.packbits(present, bitorder="big").tobytes()


@pytest.mark.parametrize("null_frac,repeat_frac", [(0.0, 0.0), (0.3, 0.2), (0.9, 0.5), (1.0, 0.0), (0.0, 1.0)])
@pytest.mark.parametrize("batch", [1, 7, 1024])
def test_dictionary_matches_java_rules(null_frac, repeat_frac, batch):
    import orc_amd

    rng = np.random.default_rng(int(null_frac * 10) * 7 + batch)
    rows, dict_size = 3000, 23
    idx, present, lengths = _dictionary_column(rng, rows, dict_size, null_frac, repeat_frac)
    values = idx[present == 1]
    # DATA: unsigned RLEv2 (the dictionary reader's createIntegerReader(..., false))
    data_stream, _ = orc_amd.encode_direct(values if values.size else np.zeros(1, np.int64), False)
    pres_stream = byte_rle_encode(_pack_bits(present), rng)
    offsets = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int32)
    buffer_len = int(offsets[-1])
    pres = orc_amd.create_boolean_rle_decoder(pres_stream)
    dec = orc_amd.create_rle_decoder(data_stream.tobytes(), False)
    scratch_got = np.full(batch, 5, np.int64)
    scratch_want = scratch_got.copy()
    start_w, len_w = np.full(batch, -1, np.int32), np.full(batch, -1, np.int32)
    start_g, len_g = start_w.copy(), len_w.copy()
    bits = [int(b) for b in present]
    pos_bits = pos_vals = 0
    rep = False
    for at in range(0, rows, batch):
        n = min(batch, rows - at)
        isn_w, nn_w, rep_w, pos_bits = java_present(bits, pos_bits, None, n, rep)
        isn_g, nn_g, rep_g = orc_amd.java_tree_present_next(pres, n, None, rep)
        np.testing.assert_array_equal(isn_g, isn_w)
        assert (nn_g, rep_g) == (nn_w, rep_w)
        nn_w, rep_w, pos_vals = java_dictionary(values, pos_vals, offsets, buffer_len, isn_w, nn_w, rep_w,
                                                scratch_want[:n], start_w[:n], len_w[:n])
        s, ln, nn_g, rep_g = orc_amd.java_dictionary_next(dec, offsets, buffer_len, isn_g, nn_g, rep_g,
                                                          scratch_got[:n], start=start_g[:n], length=len_g[:n])
        assert (nn_g, rep_g) == (nn_w, rep_w), at
        np.testing.assert_array_equal(s, start_w[:n], err_msg="start at %d" % at)
        np.testing.assert_array_equal(ln, len_w[:n], err_msg="length at %d" % at)
        rep = rep_g


def test_dictionary_without_buffer():
    import orc_amd

    # no dictionary bytes, no offsets: the batch is one repeating null
    isn = np.zeros(4, np.uint8)
    s, ln, nn, rep = orc_amd.java_dictionary_next(None, None, 0, isn, True, False, np.zeros(4, np.int64),
                                                  has_buffer=False)
    assert not nn and rep and isn[0] == 1 and s[0] == 0 and ln[0] == 0
    # offsets but no bytes: non-null rows are empty strings, nulls untouched
    isn = np.array([0, 1, 0], np.uint8)
    st, le = np.full(3, 9, np.int32), np.full(3, 9, np.int32)
    s, ln, nn, rep = orc_amd.java_dictionary_next(None, np.array([0, 0], np.int32), 0, isn, False, False,
                                                  np.zeros(3, np.int64), has_buffer=False, start=st, length=le)
    assert list(s) == [0, 9, 0] and list(ln) == [0, 9, 0]


def test_dictionary_index_out_of_bounds_is_java_error():
    import orc_amd

    data_stream, _ = orc_amd.encode_direct(np.array([0, 1, 7], np.int64), False)
    dec = orc_amd.create_rle_decoder(data_stream.tobytes(), False)
    offsets = np.array([0, 2, 5], np.int32)  # two entries
    with pytest.raises(orc_amd.ParseError, match="Index 7 out of bounds for length 3"):
        orc_amd.java_dictionary_next(dec, offsets, 5, np.zeros(3, np.uint8), True, False, np.zeros(3, np.int64))
