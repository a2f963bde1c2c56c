"""Per-step GPU idle between consecutive kernels from a rocprofv3
kernel_trace.csv: mean gap after each (kernel -> next kernel) pair over the
steps [first, last) counted by `anchor` (a kernel launched once per step).
  python scripts/kgaps.py <run_kernel_trace.csv> <anchor> <first> <last>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
anchor, first, last = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])


def short(n):
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:44]


idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
gaps = collections.defaultdict(list)
busy = []
for s in range(first, min(last, len(idx) - 1)):
    a, b = idx[s], idx[s + 1]
    busy.append(sum(int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])
                    for i in range(a, b)) / 1e3)
    for i in range(a, b):
        g = (int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3
        gaps[(short(rows[i]["Kernel_Name"]), short(rows[i + 1]["Kernel_Name"]))].append(g)
tot = 0.0
for k, v in gaps.items():
    m = sum(v) / len(v)
    tot += m
    print(f"{m:7.2f} us  {k[0]:44s} -> {k[1]}")
steps = [(int(rows[idx[s + 1]]["Start_Timestamp"]) - int(rows[idx[s]]["Start_Timestamp"])) / 1e3
         for s in range(first, min(last, len(idx) - 1))]
print(f"gap per step {tot:.1f} us; step {sum(steps) / len(steps):.1f} us; "
      f"kernel time {sum(busy) / len(busy):.1f} us")
