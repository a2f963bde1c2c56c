"""Print a rocprofv3 kernel_stats.csv compactly: calls, avg, ms/step, share.
  python scripts/kstats.py <run_kernel_stats.csv> <steps> [top]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
for r in rows[:top]:
    n = r['Name'].replace('(anonymous namespace)::', '').replace('void ', '')[:100]
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f}us {float(r['TotalDurationNs'])/1e6/steps:8.3f}ms/step {float(r['Percentage']):5.1f}% {n}")
