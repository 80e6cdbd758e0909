"""Hand-built ORC tails for corrupt-file tests: a minimal protobuf wire
writer for the PostScript / Footer / StripeInformation / Type messages
(field numbers from the ORC spec, site/specification/ORCv1.md "File Tail"),
so tests can produce offsets and lengths no writer would emit."""


def varint(x):
    out = bytearray()
    x &= (1 << 64) - 1
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def field_varint(f, v):
    return varint(f << 3) + varint(v)


def field_bytes(f, b):
    return varint((f << 3) | 2) + varint(len(b)) + b


def stripe_info(offset, index_length, data_length, footer_length, num_rows):
    return (field_varint(1, offset) + field_varint(2, index_length) + field_varint(3, data_length) +
            field_varint(4, footer_length) + field_varint(5, num_rows))


def type_msg(kind, subtypes=(), names=()):
    m = field_varint(1, kind)
    if subtypes:
        m += field_bytes(2, b"".join(varint(s) for s in subtypes))
    for n in names:
        m += field_bytes(3, n.encode())
    return m


def orc_file(body, stripes, types, num_rows, footer_length_override=None):
    """'ORC' + body + Footer + PostScript + 1-byte PostScript length
    (uncompressed)."""
    footer = b"".join(field_bytes(3, s) for s in stripes)
    footer += b"".join(field_bytes(4, t) for t in types)
    footer += field_varint(6, num_rows)
    flen = len(footer) if footer_length_override is None else footer_length_override
    ps = field_varint(1, flen) + field_varint(2, 0) + field_bytes(4, varint(0) + varint(12)) + field_bytes(8000, b"ORC")
    return b"ORC" + body + footer + ps + bytes([len(ps)])
