"""Write roboken-fmskf-robot-controller_amd/csrc/cmsis_sintab.inc: CMSIS-DSP's sinTable_f32 as its
513 published 8-decimal literals, sin(2 pi i / 512) rounded to 8 digits after the point (Python's
'%.8f' of the double sine, the same correctly rounded decimal C's printf gives)."""
import math
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "roboken-fmskf-robot-controller_amd", "csrc", "cmsis_sintab.inc")


def literals():
    return ["%.8f" % math.sin(2.0 * math.pi * i / 512.0) for i in range(513)]


if __name__ == "__main__":
    vals = literals()
    with open(OUT) as f:
        head = f.read().split("*/", 1)[0] + "*/\n"
    body = ["    " + ", ".join(v + "f" for v in vals[k:k + 8]) + "," for k in range(0, 513, 8)]
    with open(sys.argv[1] if len(sys.argv) > 1 else OUT, "w") as f:
        f.write(head + "\n".join(body) + "\n")
