"""Static instruction mix per kernel of a HIP source (gfx950 device assembly).

  python tools/isa_stats.py roboken-fmskf-robot-controller_amd/csrc/kernels_kf6.hip [filter] [--dump]

Counts every instruction between a kernel's label and its s_endpgm, grouped by class
(VALU / SALU / VMEM / LDS / branch), and lists the most frequent opcodes.  --dump writes
the kernel's assembly to /tmp/<short>.s for reading.
"""
import collections
import re
import subprocess
import sys

src = sys.argv[1]
args = [a for a in sys.argv[2:] if not a.startswith("--")]
flt = args[0] if args else ""
dump = "--dump" in sys.argv
asm = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                      "-ffp-contract=off", "-fno-slp-vectorize", "-x", "hip", "--cuda-device-only", "-S", src, "-o", "-"],
                     capture_output=True, text=True, check=True).stdout

funcs = {}
cur = None
for line in asm.splitlines():
    m = re.match(r"^(_Z\S+):", line)
    if m:
        cur = m.group(1)
        funcs[cur] = []
        continue
    if cur is None:
        continue
    s = line.strip()
    if not s or s.startswith((".", ";", "//")) or s.endswith(":"):
        continue
    op = s.split()[0]
    funcs[cur].append(s)
    if op == "s_endpgm":
        cur = None


def klass(op):
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("v_"):
        return "VALU"
    return "other"


for name, ins in funcs.items():
    dem = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
    if flt not in dem:
        continue
    ops = [i.split()[0] for i in ins]
    cls = collections.Counter(klass(o) for o in ops)
    print(f"{dem[:120]}\n  total {len(ops)}  " + "  ".join(f"{k} {v}" for k, v in cls.most_common()))
    print("  top:", ", ".join(f"{o} {c}" for o, c in collections.Counter(ops).most_common(24)))
    if dump:
        short = re.sub(r"\W+", "_", dem)[:60]
        with open(f"/tmp/{short}.s", "w") as f:
            f.write("\n".join(ins))
        print("  ->", f"/tmp/{short}.s")
