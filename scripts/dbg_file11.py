import os, sys
os.environ["ORCG_DEBUG"] = "alloc"
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import orc_amd
from file_parity import path
ctx = orc_amd.Context(0)
r = orc_amd.Reader(path("orc-file-11-format.orc"), ctx)
print("stripes", r.num_stripes, "rows", r.num_rows, flush=True)
for s in range(r.num_stripes):
    try:
        b = r.read_stripe(s)
        print("stripe", s, "ok", sorted(b.columns), flush=True)
    except Exception as e:
        print("stripe", s, "error", e, flush=True)
        for t in r.types:
            print(t, flush=True)
        break
