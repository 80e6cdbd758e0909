#!/usr/bin/env python3
"""Generate the known-answer fixtures that pin the oracle and the HIP decoder.

Run in the build container (where /root/reference exists):

    python tests/golden/make_kat_fixtures.py

It writes ``tests/golden/kat_rlev2.json``, ``kat_byterle.json`` and
``kat_boolrle.json``. Each fixture is DATA ONLY: the encoded byte string that a
reference test or spec example feeds the decoder, and the values that test
asserts. Byte strings are extracted verbatim from the reference test sources
(c++/test/TestRleDecoder.cc, c++/test/TestByteRle.cc) and the spec
(site/specification/ORCv1.md); expected values are the formulas / literal
arrays those tests assert, restated here per test. ``null`` in an expected
list means "not asserted by the reference test" (e.g. null slots).

Fixture schema (one JSON object per fixture):
    name        reference TEST name (or spec section)
    source      file:line of the reference test
    kind        "rlev2" | "byterle" | "boolrle"
    signed      bool (rlev2 only)
    data        hex string of the encoded stream
    expected    list of ints / null
    not_null    optional list of 0/1 (positions with 0 are null)
    batches     batch sizes the reference test reads with (checkResults)
    seek        optional {"position": [...], "expected": [...]} seek check
"""
import json
import os
import re
import sys

REF = os.environ.get("ORC_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


def read(rel):
    with open(os.path.join(REF, rel)) as f:
        return f.read()


def test_blocks(src):
    """Map TEST(Suite, name) -> (start line, body text)."""
    out = {}
    starts = [(m.start(), m.group(1), m.group(2)) for m in re.finditer(r"TEST\((\w+),\s*(\w+)\)", src)]
    for i, (pos, suite, name) in enumerate(starts):
        end = starts[i + 1][0] if i + 1 < len(starts) else len(src)
        line = src.count("\n", 0, pos) + 1
        out[(suite, name)] = (line, src[pos:end])
    return out


def arrays(body, ident):
    """All brace-initialised arrays named `ident` in a test body, as ints."""
    res = []
    for m in re.finditer(r"\b" + ident + r"\[\]\s*=\s*\{([^}]*)\}", body):
        text = re.sub(r"//[^\n]*", "", m.group(1))
        toks = [t.strip() for t in text.replace("\n", " ").split(",") if t.strip()]
        vals = []
        for t in toks:
            t = t.rstrip("lL")
            vals.append(int(t, 16) if t.lower().startswith(("0x", "-0x")) else int(t))
        res.append(vals)
    return res


def s64(v):
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >> 63 else v


def main():
    src = read("c++/test/TestRleDecoder.cc")
    blocks = test_blocks(src)
    fx = []
    B = [1, 3, 7, None]  # None == whole count (checkResults(n=count))

    def add(name, data, expected, signed=True, not_null=None, batches=B, seek=None, sub=""):
        line, _ = blocks[("RLEv2", name)]
        d = {
            "name": name + sub,
            "source": "c++/test/TestRleDecoder.cc:%d" % line,
            "kind": "rlev2",
            "signed": signed,
            "data": bytes(data).hex(),
            "expected": expected,
            "batches": batches,
        }
        if not_null is not None:
            d["not_null"] = not_null
        if seek is not None:
            d["seek"] = seek
        fx.append(d)

    def body(name):
        return blocks[("RLEv2", name)][1]

    # basicDelta0: 0..19
    add("basicDelta0", arrays(body("basicDelta0"), "bytes")[0], list(range(20)))
    add("basicDelta1", arrays(body("basicDelta1"), "bytes")[0], [-500, -400, -350, -325, -310])
    add("basicDelta2", arrays(body("basicDelta2"), "bytes")[0], [-500, -600, -650, -675, -710])
    add("basicDelta3", arrays(body("basicDelta3"), "bytes")[0], [500, 400, 350, 325, 310])
    add("basicDelta4", arrays(body("basicDelta4"), "bytes")[0], [500, 600, 650, 675, 710])
    add("basicDelta5", arrays(body("basicDelta5"), "bytes")[0], [i - 32 for i in range(65)])
    add("delta0Width", arrays(body("delta0Width"), "buffer")[0], [0, 1, 2, 0x42, 0x42, 0x42],
        signed=False, batches=[None])
    # basicDelta0WithNulls: value i then a null after every i % 3 == 0
    vals, nn = [], []
    for i in range(20):
        vals.append(i)
        nn.append(1)
        if i % 3 == 0:
            vals.append(None)
            nn.append(0)
    add("basicDelta0WithNulls", arrays(body("basicDelta0WithNulls"), "bytes")[0], vals, not_null=nn)
    add("shortRepeats", arrays(body("shortRepeats"), "bytes")[0],
        [i for i in range(10) for _ in range(7)])
    add("multiByteShortRepeats", arrays(body("multiByteShortRepeats"), "bytes")[0],
        [i + (1 << 62) for i in range(3) for _ in range(7)])
    add("0to2Repeat1Direct", arrays(body("0to2Repeat1Direct"), "buffer")[0], [0, 1, 2], batches=[None])
    b = arrays(body("bitSize1Direct"), "bytes")[0]
    add("bitSize1Direct", b, [i % 2 for i in range(40)], signed=False)
    b2 = arrays(body("bitSize1Direct"), "bytes2")[0]
    add("bitSize1Direct", b2, [0, 1, 1] * 10, signed=False, sub="_bytes2")
    add("bitSize2Direct", arrays(body("bitSize2Direct"), "bytes")[0], [i % 2 for i in range(20)])
    add("bitSize4Direct", arrays(body("bitSize4Direct"), "bytes")[0], [(i % 2) * 2 for i in range(20)])
    add("bitSize4Direct", arrays(body("bitSize4Direct"), "bytes2")[0],
        [(i % 4) * 2 - 2 for i in range(20)], sub="_bytes2")
    for w in (8, 16, 24, 32, 40, 48, 56, 64):
        nb = w // 8
        exp = [s64(sum(i << (8 * k) for k in range(nb))) for i in range(20)]
        add("bitSize%dDirect" % w, arrays(body("bitSize%dDirect" % w), "bytes")[0], exp)
    add("multipleRunsDirect", arrays(body("multipleRunsDirect"), "bytes")[0],
        [i % 2 for i in range(20)] + [(i % 2) * 2 for i in range(20)])
    add("largeNegativesDirect", arrays(body("largeNegativesDirect"), "buffer")[0],
        [-7486502418706614742, 0, 1, 1, -5535739865598783616], batches=[None])
    add("overflowDirect", arrays(body("overflowDirect"), "bytes")[0],
        [4513343538618202719, 4513343538618202711, 2911390882471569739, -9181829309989854913])
    add("basicPatched0", arrays(body("basicPatched0"), "bytes")[0], arrays(body("basicPatched0"), "v")[0])
    add("basicPatched1", arrays(body("basicPatched1"), "bytes")[0], arrays(body("basicPatched1"), "v")[0])
    add("mixedPatchedAndShortRepeats", arrays(body("mixedPatchedAndShortRepeats"), "bytes")[0],
        arrays(body("mixedPatchedAndShortRepeats"), "v")[0])
    # basicDirectSeek: seek to (byte 7, skip 13) then 7 values 2,0,2,0,2,0,2
    add("basicDirectSeek", arrays(body("basicDirectSeek"), "bytes")[0],
        [i % 2 for i in range(20)] + [(i % 2) * 2 for i in range(20)],
        seek={"position": [7, 13], "expected": [2, 0, 2, 0, 2, 0, 2]})
    # bitsLeftByPreviousStream: 118 DIRECT values (not asserted) + patched v[]
    pv = arrays(body("bitsLeftByPreviousStream"), "v")[0]
    add("bitsLeftByPreviousStream", arrays(body("bitsLeftByPreviousStream"), "bytes")[0],
        [None] * 118 + pv, batches=[None])

    # Spec worked examples, site/specification/ORCv1.md
    spec = read("site/specification/ORCv1.md")

    def spec_find(text):
        m = re.search(r"\s+".join(re.escape(w) for w in text.split()), spec)
        if not m:
            raise SystemExit("spec anchor not found: %r" % text)
        return m.start()

    def spec_line(text):
        return "site/specification/ORCv1.md:%d" % (spec[: spec_find(text)].count("\n") + 1)

    def spec_bytes(text_after):
        i = spec_find(text_after)
        m = re.search(r"\[(0x[0-9a-fA-F]{2}(?:,\s*0x[0-9a-fA-F]{2})*)\]", spec[i:])
        return [int(t, 16) for t in re.split(r",\s*", m.group(1))]

    for title, anchor, exp in [
        ("spec_short_repeat", "would be\nserialized with short repeat", [10000] * 5),
        ("spec_direct", "would be\nserialized with direct encoding", [23713, 43806, 57005, 48879]),
        ("spec_patched_base", "The base value is 2000 and the combined result is",
         [2030, 2000, 2020, 1000000] + list(range(2040, 2200, 10))),
        ("spec_delta", "The resulting\nsequence is", [2, 3, 5, 7, 11, 13, 17, 19, 23, 29]),
    ]:
        fx.append({
            "name": title, "source": spec_line(anchor), "kind": "rlev2", "signed": False,
            "data": bytes(spec_bytes(anchor)).hex(), "expected": exp, "batches": B,
        })

    with open(os.path.join(HERE, "kat_rlev2.json"), "w") as f:
        json.dump(fx, f, indent=1)

    # ---------------------------------------------------------------- byte RLE
    bsrc = read("c++/test/TestByteRle.cc")
    bb = test_blocks(bsrc)
    byte_fx = []

    def addb(suite, name, data, expected, kind, not_null=None, batches=None, sub=""):
        line, _ = bb[(suite, name)]
        d = {"name": name + sub, "source": "c++/test/TestByteRle.cc:%d" % line, "kind": kind,
             "data": bytes(data).hex(), "expected": expected, "batches": batches or [None]}
        if not_null is not None:
            d["not_null"] = not_null
        byte_fx.append(d)

    addb("ByteRle", "simpleTest", arrays(bb[("ByteRle", "simpleTest")][1], "buffer")[0],
         [0] * 100 + [0x44, 0x45, 0x46], "byterle")
    # nullTest: two 128-literal groups 0..255, 10 leading nulls
    buf = [0x80] + list(range(128)) + [0x80] + list(range(128, 256))
    addb("ByteRle", "nullTest", buf, [None] * 10 + [(i - 10) & 0xFF for i in range(10, 266)], "byterle",
         not_null=[int(i >= 10) for i in range(266)])
    addb("ByteRle", "literalCrossBuffer", arrays(bb[("ByteRle", "literalCrossBuffer")][1], "buffer")[0],
         list(range(10)) + [16] * 10, "byterle")
    addb("ByteRle", "simpleRuns", arrays(bb[("ByteRle", "simpleRuns")][1], "buffer")[0],
         [0xFF] * 16 + [0xFE] * 16 + [0xFD] * 16, "byterle", batches=[16])
    addb("ByteRle", "splitHeader", arrays(bb[("ByteRle", "splitHeader")][1], "buffer")[0],
         [1, 1, 1] + [i - 2 for i in range(3, 35)], "byterle")
    addb("ByteRle", "splitRuns", arrays(bb[("ByteRle", "splitRuns")][1], "buffer")[0],
         [2] * 16 + list(range(1, 17)), "byterle", batches=[5])
    # testNulls: literal 0..15 then run of 64 x 0xdc, every odd position null
    tn = arrays(bb[("ByteRle", "testNulls")][1], "buffer")[0]
    exp, nn = [], []
    k = 0
    for i in range(160):
        if i % 2 == 0:
            exp.append(k if k < 16 else 0xDC)
            k += 1
            nn.append(1)
        else:
            exp.append(None)
            nn.append(0)
    addb("ByteRle", "testNulls", tn, exp, "byterle", not_null=nn, batches=[16])
    # spec byte RLE examples
    byte_fx.append({"name": "spec_byte_run", "source": spec_line("a\nhundred 0's is encoded as"),
                    "kind": "byterle", "data": "6100", "expected": [0] * 100, "batches": [None]})
    byte_fx.append({"name": "spec_byte_literal", "source": spec_line("a\nhundred 0's is encoded as"),
                    "kind": "byterle", "data": "fe4445", "expected": [0x44, 0x45], "batches": [None]})
    with open(os.path.join(HERE, "kat_byterle.json"), "w") as f:
        json.dump(byte_fx, f, indent=1)

    # ------------------------------------------------------------- boolean RLE
    bool_fx = []

    def addz(name, data, expected, not_null=None, batches=None):
        line, _ = bb[("BooleanRle", name)]
        d = {"name": name, "source": "c++/test/TestByteRle.cc:%d" % line, "kind": "boolrle",
             "data": bytes(data).hex(), "expected": expected, "batches": batches or [None]}
        if not_null is not None:
            d["not_null"] = not_null
        bool_fx.append(d)

    st = arrays(bb[("BooleanRle", "simpleTest")][1], "buffer")[0]
    exp = [1 if (p & 4) == 0 else 0 for p in range(800)]
    exp += [0 if (i % 2) == (j % 2) else 1 for i in range(3) for j in range(8)]
    addz("simpleTest", st, exp, batches=[50])
    rt = arrays(bb[("BooleanRle", "runsTest")][1], "buffer")[0]
    addz("runsTest", rt, [1 if i % 18 < 9 else 0 for i in range(72)], batches=[None, 1])
    addz("runsTestWithNull", rt, [1 if i % 18 < 9 else 0 for i in range(72)], not_null=[1] * 72,
         batches=[None, 1])
    bool_fx.append({"name": "spec_boolean", "source": spec_line("the byte sequence [0xff, 0x80]"),
                    "kind": "boolrle", "data": "ff80", "expected": [1, 0, 0, 0, 0, 0, 0, 0],
                    "batches": [None]})
    with open(os.path.join(HERE, "kat_boolrle.json"), "w") as f:
        json.dump(bool_fx, f, indent=1)
    # ------------------------------------------------------------------ RLEv1
    v1_fx = []

    def addv1(name, data, expected, signed, not_null=None, batches=None, seeks=None):
        line, _ = blocks[("RLEv1", name)]
        d = {"name": name, "source": "c++/test/TestRleDecoder.cc:%d" % line, "kind": "rlev1",
             "signed": signed, "data": bytes(data).hex(), "expected": expected, "batches": batches or [None]}
        if not_null is not None:
            d["not_null"] = not_null
        if seeks is not None:
            d["seeks"] = seeks
        v1_fx.append(d)

    def v1body(name):
        return blocks[("RLEv1", name)][1]

    addv1("simpleTest", arrays(v1body("simpleTest"), "buffer")[0], [100 - i for i in range(100)] + [2, 3, 5, 7, 11],
          False)
    addv1("signedNullLiteralTest", arrays(v1body("signedNullLiteralTest"), "buffer")[0],
          [i // 2 if i % 2 == 0 else -((i + 1) // 2) for i in range(8)], True, not_null=[1] * 8)
    addv1("splitHeader", arrays(v1body("splitHeader"), "buffer")[0], [247864668] * 3, False)
    addv1("splitRuns", arrays(v1body("splitRuns"), "buffer")[0], [255 + i for i in range(128)] + [1, 2, 3, 4, 5],
          False, batches=[3])
    addv1("testSigned", arrays(v1body("testSigned"), "buffer")[0], [16 - i for i in range(130)], True,
          batches=[100, None])
    # testNull: odd positions null, values count up through 10 batches of 24
    exp, nn = [], []
    for i in range(10):
        for j in range(24):
            on = (j + 1) % 2
            nn.append(on)
            exp.append(i * 24 + j if on else None)
    addv1("testNull", arrays(v1body("testNull"), "buffer")[0], exp, True, not_null=nn, batches=[24])
    addv1("testLeadingNulls", arrays(v1body("testLeadingNulls"), "buffer")[0], [None] * 5 + [1, 2, 3, 4, 5], False,
          not_null=[0] * 5 + [1] * 5)
    addv1("skipTest", arrays(v1body("skipTest"), "buffer")[0], [i if i < 1024 else 256 * i for i in range(2048)],
          True, batches=[None, 7])
    sb = v1body("seekTest")
    junk = arrays(sb, "junk")[0]
    file_loc = arrays(sb, "fileLoc")[0]
    rle_loc = arrays(sb, "rleLoc")[0]
    want = [i // 4 if i < 1024 else 2 * i for i in range(2048)] + junk

    def at(i):
        return want[i]

    picks = list(range(0, 4096, 61)) + [1023, 1024, 2047, 2048, 4095]
    addv1("seekTest", arrays(sb, "buffer")[0], want, True, batches=[2048],
          seeks=[{"position": [file_loc[i], rle_loc[i]], "expected": [at(i)]} for i in picks])
    with open(os.path.join(HERE, "kat_rlev1.json"), "w") as f:
        json.dump(v1_fx, f, indent=1)
    print("wrote %d rlev2, %d byte-rle, %d bool-rle, %d rlev1 fixtures" % (len(fx), len(byte_fx), len(bool_fx),
                                                                         len(v1_fx)))


if __name__ == "__main__":
    sys.exit(main())
