"""Print one stripe's kernel timeline from a rocprofv3 kernel trace:
python scripts/timeline.py <run_kernel_trace.csv> [anchor kernel substring] [which occurrence from the end]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "dict_multi"
k = int(sys.argv[3]) if len(sys.argv) > 3 else 3
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i = idx[-k]
lo = i
while lo > 0 and int(rows[i]["Start_Timestamp"]) - int(rows[lo - 1]["End_Timestamp"]) < 400_000 and i - lo < 30:
    lo -= 1
t0 = int(rows[lo]["Start_Timestamp"])
for r in rows[lo:i + 8]:
    n = re.sub(r"orcg::\(anonymous namespace\)::", "", r["Kernel_Name"])
    n = re.sub(r"\(.*", "", n)[:80]
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} q{r['Queue_Id']} wg={wg} {n}")
