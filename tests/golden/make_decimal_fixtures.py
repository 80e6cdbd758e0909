#!/usr/bin/env python3
"""Generate ``tests/golden/kat_decimal.json``: the decimal and timestamp
column known answers of the reference's c++/test/TestColumnReader.cc, as
data (stream byte strings + the values the tests assert).

Run in the build container (where /root/reference exists):

    python tests/golden/make_decimal_fixtures.py

Byte strings are extracted verbatim from the test sources (the two
loop-generated DATA buffers of testDecimal64 / testDecimal128 are rebuilt
with the tests' own loop); expected values are the literals / formulas those
tests assert, restated per test. Streams of DIRECT-encoded columns are RLEv1
(the tests' getEncoding returns DIRECT).

Fixture schema:
    name, source      reference TEST and file:line
    kind              "decimal" | "timestamp"
    present           hex of the PRESENT stream (boolean RLE) or null
    data              hex of DATA (varints / RLEv1 seconds)
    secondary         hex of SECONDARY (RLEv1 scales, signed / nanos, unsigned)
    precision, scale  decimal type
    expected          non-null values in row order (ints; Decimal128 as ints)
    expected_nanos    timestamp nanoseconds
"""
import calendar
import json
import os
import re
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_kat_fixtures import arrays, read, test_blocks  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def loop_num_buffer():
    # testDecimal64 / testDecimal128 (TestColumnReader.cc:2669-2676)
    return [(0x3f - 2 * i) if i < 32 else 2 * (i - 32) for i in range(65)]


def main():
    src = read("c++/test/TestColumnReader.cc")
    blocks = test_blocks(src)
    out = []

    def blk(name, suite="DecimalColumnReader"):
        line, body = blocks[(suite, name)]
        return line, body

    for name, prec in (("testDecimal64", 12), ("testDecimal128", 32)):
        line, body = blk(name)
        out.append({
            "name": name, "source": "c++/test/TestColumnReader.cc:%d" % line, "kind": "decimal",
            "present": bytes(arrays(body, "buffer1")[0]).hex(), "data": bytes(loop_num_buffer()).hex(),
            "secondary": bytes(arrays(body, "buffer2")[0]).hex(), "precision": prec, "scale": 2,
            "expected": list(range(-32, 33)),
        })
    skip_vals = [493827160549382716, 4938271605493827, 49382716054938, 493827160549, 4938271605, 49382716,
                 493827, 4938, 49]
    line, body = blk("testDecimal64Skip")
    out.append({
        "name": "testDecimal64Skip", "source": "c++/test/TestColumnReader.cc:%d" % line, "kind": "decimal",
        "present": bytes(arrays(body, "presentBuffer")[0]).hex(), "data": bytes(arrays(body, "numBuffer")[0]).hex(),
        "secondary": bytes(arrays(body, "buffer1")[0]).hex(), "precision": 12, "scale": 10,
        "expected": skip_vals,
    })
    big = 17320508075688772935274463415058723669
    nines = 99999999999999999999999999999999999999
    line, body = blk("testDecimal128Skip")
    out.append({
        "name": "testDecimal128Skip", "source": "c++/test/TestColumnReader.cc:%d" % line, "kind": "decimal",
        "present": bytes(arrays(body, "presentBuffer")[0]).hex(), "data": bytes(arrays(body, "numBuffer")[0]).hex(),
        "secondary": bytes(arrays(body, "buffer2")[0]).hex(), "precision": 38, "scale": 37,
        "expected": skip_vals + [big, -big, nines, -nines],
    })
    # Hive 0.11 decimals (precision 0, DecimalHive11ColumnReader): `scale` is
    # the forced scale the test's mock returns; "error" = the ParseError the
    # test expects (throwOnHive11DecimalOverflow true)
    hive = [
        ("testDecimalHive11", 6, "buffer1", None, list(range(-32, 33)), None),
        ("testDecimalHive11Skip", 3, "presentBuffer", "numBuffer", skip_vals + [big, -big, nines, -nines], None),
        ("testDecimalHive11ScaleUp", 20, "presentBuffer", "numBuffer", [10 ** i for i in range(21)], None),
        ("testDecimalHive11ScaleDown", 0, "presentBuffer", "numBuffer", [10 ** (20 - i) for i in range(21)], None),
        ("testDecimalHive11OverflowException", 6, "presentBuffer", "numBuffer", [0],
         "Hive 0.11 decimal was more than 38 digits."),
        ("testDecimalHive11OverflowExceptionNull", 6, "presentBuffer", "numBuffer", [0],
         "Hive 0.11 decimal was more than 38 digits."),
        # throwOnHive11DecimalOverflow(false): the two overflowing values of
        # the four non-null rows are replaced by NULL (None), the others read 1
        ("testDecimalHive11OverflowNull", 6, "presentBuffer", "numBuffer", [None, 1, None, 1], None),
    ]
    for name, forced, pres, num, expected, err in hive:
        line, body = blk(name)
        fx = {
            "name": name, "source": "c++/test/TestColumnReader.cc:%d" % line, "kind": "decimal",
            "present": bytes(arrays(body, pres)[0]).hex(),
            "data": bytes(arrays(body, num)[0] if num else loop_num_buffer()).hex(),
            "secondary": bytes(arrays(body, "scaleBuffer")[0]).hex(), "precision": 0, "scale": forced,
            "expected": expected,
        }
        if err:
            fx["error"] = err
        if name == "testDecimalHive11OverflowNull":
            fx["throw_on_overflow"] = False
        out.append(fx)
    line, body = blk("testTimestamp", "TestColumnReader")
    dates = re.findall(r'"(\w{3} \w{3} [ \d]\d \d\d:\d\d:\d\d \d{4})\\n"', body)
    secs = [calendar.timegm(time.strptime(d, "%a %b %d %H:%M:%S %Y")) for d in dates]
    nanos = [int(x) for x in re.search(r"expectedNano\[\]\s*=\s*\{([^}]*)\}", body).group(1).replace(
        "\n", " ").split(",") if x.strip()]
    out.append({
        "name": "testTimestamp", "source": "c++/test/TestColumnReader.cc:%d" % line, "kind": "timestamp",
        "present": None, "data": bytes(arrays(body, "buffer1")[0]).hex(),
        "secondary": bytes(arrays(body, "buffer2")[0]).hex(), "expected": secs, "expected_nanos": nanos,
    })
    path = os.path.join(HERE, "kat_decimal.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote %d fixtures to %s" % (len(out), path))


if __name__ == "__main__":
    main()
