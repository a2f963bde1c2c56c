"""Summarise a rocprofv3 bench profile into profiles/ (committed evidence).

  python scripts/prof_summary.py gpurun_out/r1 profiles r01 --steps 25

Reads <run>/prof/run_kernel_stats.csv (--kernel-trace --stats) and the
<run>/pmc_FETCH_SIZE, <run>/pmc_WRITE_SIZE counter passes; writes
  profiles/<tag>_kernel_stats.md   per-kernel calls / average / share
  profiles/<tag>_kernel_stats.csv  the raw rocprofv3 stats table
  profiles/pmc_traffic.json        HBM bytes per launch of the hot-path kernels
                                   (FETCH_SIZE x2 on gfx950 + WRITE_SIZE, per
                                   MI355X_MICROARCH.md's HBM section)
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (kernel_source_digest)

# hot-path kernel (regex on the demangled name) -> bench.py kernel-table key;
# first match wins
HOT = [
    (r"conv_bwd_x6[pq]_kernel", "conv_bwd_pooled"),
    (r"conv_bwd_x6_kernel<\d+, \w+, \w+, [48](, \d)?>", "conv_bwd_pooled"),
    (r"conv_bwd_x6_kernel", "conv_bwd_fused"),
    (r"conv_bwd_dma_kernel<\d+, \w+, \w+, [48]>", "conv_bwd_pooled"),
    (r"conv_bwd_dma_kernel", "conv_bwd_fused"),
    (r"conv_bwd_frame_kernel", "conv_bwd_fused"),
    (r"conv_fwd_regs_kernel<\d+, \d+, [248](, \w+)*>", "conv_fwd_maxpool"),
    (r"conv_fwd_regs_kernel", "conv_fwd"),
    (r"conv_fwd_slab_kernel", "conv_fwd"),
    (r"conv_fwd_frame_kernel", "conv_fwd"),
    (r"maxpool_mask_backprop_kernel", "maxpool_bwd_mask"),
    (r"maxpool_(group|direct)_prop_kernel", "maxpool_fwd"),
    (r"maxpool_(group|direct)_backprop_kernel", "maxpool_bwd"),
    (r"MaxpoolProp", "maxpool_fwd"),
    (r"MaxpoolBackprop", "maxpool_bwd"),
]


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    m = re.match(r"([A-Za-z_][A-Za-z0-9_:]*(<[^()]*>)?)", name)
    return (m.group(1) if m else name)[:80]


def kernel_key(name):
    for pat, v in HOT:
        if re.search(pat, name):
            return v
    return None


def pmc_means(d, counter):
    """Mean per dispatch of `counter` for each kernel name (summed over dims)."""
    per = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            k = row["Kernel_Name"]
            per[k] += float(row["Counter_Value"])
            n[k].add(row["Dispatch_Id"])
    return {k: per[k] / len(n[k]) for k in per}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run")
    ap.add_argument("out")
    ap.add_argument("tag")
    ap.add_argument("--steps", type=int, default=25, help="bench steps profiled (warmup+timed)")
    ap.add_argument("--cmd", default="python bench.py --steps 20 --warmup 5 --no-cpu-baseline",
                    help="the profiled command, for the report header")
    ap.add_argument("--label", default="c2, N=4096, 1x MI355X", help="workload, for the header")
    ap.add_argument("--frames", type=int, default=4096, help="frames per launch of the run")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    stats = os.path.join(a.run, "prof", "run_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    shutil.copy(stats, os.path.join(a.out, f"{a.tag}_kernel_stats.csv"))
    lines = [f"# {a.tag}: rocprofv3 --kernel-trace --stats, `{a.cmd}` ({a.label})", "",
             "| kernel | calls | avg us | total ms | % |", "|---|---:|---:|---:|---:|"]
    for r in rows:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} "
                     f"| {float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f} |")
    total_ms = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6
    lines += ["", f"GPU kernel time per step: {total_ms / a.steps:.3f} ms over {a.steps} steps."]
    fetch = pmc_means(os.path.join(a.run, "pmc_FETCH_SIZE"), "FETCH_SIZE")
    write = pmc_means(os.path.join(a.run, "pmc_WRITE_SIZE"), "WRITE_SIZE")
    traffic = {}
    if not fetch and not write:
        with open(os.path.join(a.out, f"{a.tag}_kernel_stats.md"), "w") as fh:
            fh.write("\n".join(lines) + "\n")
        print("\n".join(lines))
        return
    lines += ["", "## HBM traffic per launch (PMC, separate passes)", "",
              "FETCH_SIZE and WRITE_SIZE are in KB; on gfx950 FETCH_SIZE counts half the bytes "
              "of 16-B/lane streaming reads, so read bytes = 2 x FETCH_SIZE x 1024.", "",
              "| kernel | FETCH_SIZE (KB) | WRITE_SIZE (KB) | HBM bytes / launch |",
              "|---|---:|---:|---:|"]
    for k in sorted(set(fetch) | set(write)):
        # every kernel in the table (the FC GEMMs' bytes included); the
        # hot-path roles also go to pmc_traffic.json for bench.py's roofline
        key = kernel_key(k)
        f_kb, w_kb = fetch.get(k, 0.0), write.get(k, 0.0)
        byts = 2 * f_kb * 1024 + w_kb * 1024
        if key is not None:
            traffic.setdefault(key, {"kernel": short(k), "hbm_bytes_per_launch": 0.0})
            traffic[key]["hbm_bytes_per_launch"] += byts
        lines.append(f"| `{short(k)}` | {f_kb:.0f} | {w_kb:.0f} | {byts:.3e} |")
    with open(os.path.join(a.out, f"{a.tag}_kernel_stats.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    if traffic:
        for v in traffic.values():
            v["hbm_bytes_per_launch"] = round(v["hbm_bytes_per_launch"])
            v["run"] = a.tag
            v["frames"] = a.frames
            # the digest of the kernel's source: bench.py uses these bytes only
            # while the source is unchanged
            v["source_sha1"] = bench.kernel_source_digest(v["kernel"])
        path = os.path.join(a.out, "pmc_traffic.json")
        merged = json.load(open(path)) if os.path.exists(path) else {}
        merged.update(traffic)  # kernels of several runs (fused / unfused)
        json.dump(merged, open(path, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
