"""A small RLEv1 stream writer for tests (format: site/specification/ORCv1.md
"Integer Run Length Encoding, version 1"; RleEncoderV1, c++/src/RLEv1.cc:
40-139): runs of 3..130 values with a signed-byte delta and a varint base,
and literal groups of 1..128 varints. The run/literal split is chosen by the
caller so tests can force every shape."""
import numpy as np


def _varint(u, out):
    u &= (1 << 64) - 1
    while True:
        b = u & 0x7F
        u >>= 7
        if u:
            out.append(b | 0x80)
        else:
            out.append(b)
            return


def _zz(v):
    v &= (1 << 64) - 1
    s = v >> 63
    return ((v << 1) & ((1 << 64) - 1)) ^ ((1 << 64) - 1 if s else 0)


def encode(groups, signed):
    """groups: list of ("run", base, delta, length) or ("lit", [values])."""
    out = bytearray()
    values = []
    for g in groups:
        if g[0] == "run":
            _, base, delta, length = g
            assert 3 <= length <= 130 and -128 <= delta <= 127
            out.append(length - 3)
            out.append(delta & 0xFF)
            _varint(_zz(base) if signed else base, out)
            for i in range(length):
                v = (base + i * delta) & ((1 << 64) - 1)
                values.append(v - (1 << 64) if v >> 63 else v)
        else:
            vals = g[1]
            assert 1 <= len(vals) <= 128
            out.append((256 - len(vals)) & 0xFF)
            for v in vals:
                _varint(_zz(v) if signed else v, out)
                u = v & ((1 << 64) - 1)
                values.append(u - (1 << 64) if u >> 63 else u)
    return bytes(out), np.array(values, dtype=np.int64)


def random_groups(rng, n, signed, max_bits=64):
    groups, count = [], 0
    while count < n:
        if rng.random() < 0.4:
            length = int(rng.integers(3, 131))
            bits = int(rng.integers(1, max_bits + 1))
            base = int(rng.integers(0, 1 << min(bits, 62)))
            if signed and rng.random() < 0.5:
                base = -base
            groups.append(("run", base, int(rng.integers(-128, 128)), length))
            count += length
        else:
            k = int(rng.integers(1, 129))
            bits = int(rng.integers(1, max_bits + 1))
            if bits >= 63:
                vals = [int(x) for x in rng.integers(-(1 << 63), (1 << 63) - 1, size=k, dtype=np.int64)]
                if not signed:
                    vals = [v & ((1 << 64) - 1) if v >= 0 else v for v in vals]
            else:
                vals = [int(x) for x in rng.integers(0, 1 << bits, size=k)]
                if signed:
                    vals = [v if rng.random() < 0.5 else -v for v in vals]
            groups.append(("lit", vals))
            count += k
    return groups
