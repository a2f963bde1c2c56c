"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean over dispatches).

  python scripts/pmc_summary.py gpurun_out/pmc2 [--match conv_]

Reads every */run_counter_collection.csv under the directory, groups by
(kernel, counter), prints the mean value per dispatch and the derived
metrics used in DESIGN.md (MFMA busy %, HBM bytes per dispatch).
"""
import argparse
import collections
import csv
import glob
import os


def short(name, n=48):
    for pre in ("void ", "(anonymous namespace)::"):
        name = name.replace(pre, "")
    return name.split("(")[0][:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                if a.match and a.match not in k:
                    continue
                # one row per (dispatch, counter): sum over agents/dims first
                vals[(k, row["Counter_Name"], row["Dispatch_Id"])].append(
                    float(row["Counter_Value"]))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, c, d), v in vals.items():
        per[k][c].append(sum(v))
    for k in sorted(per):
        cs = per[k]
        means = {c: sum(v) / len(v) for c, v in cs.items()}
        print(short(k, 90))
        for c in sorted(means):
            print(f"    {c:28s} {means[c]:16.1f}  (n={len(cs[c])})")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in means and "GRBM_GUI_ACTIVE" in means:
            # 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE comes summed over the 8 XCDs
            util = means["SQ_VALU_MFMA_BUSY_CYCLES"] / (means["GRBM_GUI_ACTIVE"] / 8 * 1024)
            print(f"    -> MFMA busy {100 * util:.1f}% of SIMD-cycles")
        if "FETCH_SIZE" in means:
            print(f"    -> FETCH_SIZE {means['FETCH_SIZE'] / 1e6:.1f} (x1 KB units?)")


if __name__ == "__main__":
    main()
