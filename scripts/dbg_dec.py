import sys; sys.path.insert(0, "."); sys.path.insert(0, "tests")
import orc_amd
from file_parity import path
for v in (0, 4, 2, 3):
    ctx = orc_amd.default_context(0)
    ctx.set_rlev2_variant(v)
    r = orc_amd.Reader(path("decimal.orc"), ctx)
    try:
        b = r.read_stripe(0)
        print("variant", v, "ok", list(b.columns))
    except Exception as e:
        print("variant", v, "FAIL", type(e).__name__, e)
    ctx.set_rlev2_variant(0)
