"""Print a rocprofv3 kernel_stats.csv as a table (per-call averages)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for x in rows:
    print(f"{x['Name'][:50]:50s} {x['Calls']:>6s} {float(x['TotalDurationNs'])/1e6:9.3f}ms "
          f"avg {float(x['AverageNs'])/1e3:8.2f}us min {float(x['MinNs'])/1e3:8.2f} max {float(x['MaxNs'])/1e3:8.2f} "
          f"{float(x['Percentage']):6.2f}%")
