"""Print the last N kernels of a rocprofv3 kernel_trace.csv: start offset, duration, gap."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 120
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = 0 if prev is None else s - prev
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:7.2f} gap {gap / 1e3:6.2f} q{r.get('Queue_Id', '?'):>3} "
          f"{r['Kernel_Name'][:70]}")
    prev = e
