"""A minimal IANA zone directory for the UTC zones (test data): pyarrow's ORC
writer and reader look up the writer zone ("GMT") under $TZDIR, and this
image ships no tzdata. A TZif v2 file with one type (offset 0, "UTC") and no
transitions, footer "UTC0" (RFC 8536 layout)."""
import os
import struct
import tempfile


def _tzif():
    def block(timesize):
        # counts: isutcnt, isstdcnt, leapcnt, timecnt, typecnt, charcnt
        hdr = b"TZif2" + bytes(15) + struct.pack(">6l", 0, 0, 0, 0, 1, 4)
        return hdr + struct.pack(">lBB", 0, 0, 0) + b"UTC\x00"
    return block(4) + block(8) + b"\nUTC0\n"


def utc_tzdir():
    d = os.path.join(tempfile.gettempdir(), "orcg_tzdata")
    os.makedirs(os.path.join(d, "Etc"), exist_ok=True)
    data = _tzif()
    for name in ("GMT", "UTC", "Etc/UTC", "Etc/GMT"):
        p = os.path.join(d, name)
        if not os.path.exists(p):
            with open(p, "wb") as f:
                f.write(data)
    return d
