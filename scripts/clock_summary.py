"""Effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) and MFMA busy per
kernel from a rocprofv3 --pmc + --kernel-trace pass (scripts/gpu_clock.sh)."""
import csv, glob, collections, re, sys
O=sys.argv[1]
cc = collections.defaultdict(dict)
for f in glob.glob(f"{O}/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d = cc[r["Dispatch_Id"]]
        d["name"] = r["Kernel_Name"]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
dur = {}
for f in glob.glob(f"{O}/p/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
def short(n):
    n=n.replace("(anonymous namespace)::","").replace("void ","")
    m=re.match(r"([A-Za-z_][A-Za-z0-9_:]*(<[^()]*>)?)", n)
    return (m.group(1) if m else n)[:60]
agg = collections.defaultdict(list)
for i, d in cc.items():
    if i in dur and dur[i] > 2e-5:
        clk = d.get("GRBM_GUI_ACTIVE", 0) / 8 / dur[i] / 1e9
        busy = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (d.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024)
        agg[short(d["name"])].append((dur[i] * 1e6, clk, busy))
for k, v in sorted(agg.items(), key=lambda x: -sum(a for a, _, _ in x[1])):
    n = len(v)
    print(f"{k:60s} n={n:3d} us={sum(a for a,_,_ in v)/n:8.1f} GHz={sum(b for _,b,_ in v)/n:5.2f} mfma_busy={100*sum(c for _,_,c in v)/n:5.1f}%")
