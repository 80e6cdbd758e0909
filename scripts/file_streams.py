#!/usr/bin/env python3
"""Stream extraction for kernel A/B on real column shapes: a minimal ORC
tail / stripe-footer walker (protobuf wire format read by hand; ORCv1.md
"File Tail", "Stripes") over UNCOMPRESSED files, returning each stream's
bytes. Used by scripts/ab_streams.py to time one kernel on the streams a
workload file really holds (C4's orderkey / linenumber / dictionary
indices, C5's list lengths and child values) at chosen segment sizes.

Tooling only: the product reader is orc_amd/csrc/orc_file.cpp."""
import numpy as np

KINDS = {0: "PRESENT", 1: "DATA", 2: "LENGTH", 3: "DICTIONARY_DATA", 4: "DICTIONARY_COUNT", 5: "SECONDARY",
         6: "ROW_INDEX", 7: "BLOOM_FILTER", 8: "BLOOM_FILTER_UTF8"}


def _varint(b, i):
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x, i


def fields(b):
    """(field number, value) pairs of one message; length-delimited values
    are bytes, varints ints (no fixed32/64 in the messages read here)."""
    out, i = [], 0
    while i < len(b):
        key, i = _varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 2:
            n, i = _varint(b, i)
            v = bytes(b[i:i + n])
            i += n
        elif wt == 1:
            v = int.from_bytes(b[i:i + 8], "little")
            i += 8
        elif wt == 5:
            v = int.from_bytes(b[i:i + 4], "little")
            i += 4
        else:
            raise ValueError("wire type %d" % wt)
        out.append((f, v))
    return out


def first(fs, f, default=0):
    for k, v in fs:
        if k == f:
            return v
    return default


def stripe_streams(path, stripe=0):
    """[(column, kind name, bytes)] of one stripe plus its encodings
    [(kind, dictionarySize)] and row count (uncompressed files only)."""
    data = np.fromfile(path, dtype=np.uint8)
    b = data.tobytes()
    ps_len = b[-1]
    ps = fields(b[-1 - ps_len:-1])
    if first(ps, 2) != 0:
        raise SystemExit("file_streams: only uncompressed files (compression NONE)")
    flen = first(ps, 1)
    foot = fields(b[-1 - ps_len - flen:-1 - ps_len])
    stripes = [fields(v) for k, v in foot if k == 3]
    si = stripes[stripe]
    off, ilen, dlen, flen2, nrows = (first(si, 1), first(si, 2), first(si, 3), first(si, 4), first(si, 5))
    sf = fields(b[off + ilen + dlen:off + ilen + dlen + flen2])
    streams, at = [], off
    for k, v in sf:
        if k != 1:
            continue
        st = fields(v)
        kind, col, ln = first(st, 1), first(st, 2), first(st, 3)
        streams.append((col, KINDS.get(kind, str(kind)), data[at:at + ln].copy()))
        at += ln
    enc = [(first(fields(v), 1), first(fields(v), 2)) for k, v in sf if k == 2]
    return streams, enc, nrows
