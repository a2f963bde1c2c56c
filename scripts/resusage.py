"""Per-kernel VGPR/AGPR/spill/LDS/occupancy of one HIP source (gfx950).
  python scripts/resusage.py kaldi-cnn_amd/src/cnslmat/cnsl-conv-mfma.hip [name-filter]"""
import re, subprocess, sys
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-Iinclude", "-Ikaldi-cnn_amd/src",
       "-I/opt/rocm/include", "--offload-arch=gfx950", "-c", src, "-o", "/tmp/_res.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for name, r in rows.items():
    if flt and flt not in name:
        continue
    dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    dm = dm.replace("(anonymous namespace)::", "")[:70]
    print(f"{dm:70s} V{r.get('VGPRs','?'):>4} A{r.get('AGPRs','?'):>4} spill{r.get('VGPRs Spill','?'):>4} "
          f"occ{r.get('Occupancy [waves/SIMD]','?'):>2} LDS{r.get('LDS Size [bytes/block]','?'):>7}")
