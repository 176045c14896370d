"""Print VGPRs / scratch / occupancy per kernel of a HIP source (compiler's view).

  python tools/resource_usage.py roboken-fmskf-robot-controller_amd/csrc/kernels_kf.hip [filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                      "-ffp-contract=off", "-fno-slp-vectorize", *[a for a in sys.argv[3:]], "-x", "hip", "-c", src, "-o", "/dev/null",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt"], input=m.group(1), capture_output=True,
                                      text=True).stdout.strip()}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "TotalSGPRs"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0].replace("\\", "")] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        name = re.sub(r"fmskf::KfArgs<[^>]*<[^>]*> >", "", r["name"])
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('ScratchSize', '?'):>4} scr "
              f"{r.get('Occupancy', '?'):>2} w/simd  {r.get('TotalSGPRs', '?'):>3} sgpr  {name[:110]}")
