#!/usr/bin/env python3
"""Static instruction counts per kernel of one HIP source (gfx950 device
asm): tools/isa_count.py stereovisionarray_amd/csrc/wta_hv.hip [filter]
[--dir SRC_DIR].  Counts VALU (v_*), SALU (s_*), VMEM (buffer_/global_),
LDS (ds_*) and s_waitcnt lines per function."""
import os
import re
import subprocess
import sys
import tempfile


def main():
    args = [a for a in sys.argv[1:]]
    src_dir = None
    if "--dir" in args:
        i = args.index("--dir")
        src_dir = args[i + 1]
        del args[i:i + 2]
    src = args[0]
    flt = args[1] if len(args) > 1 else ""
    d = src_dir or os.path.dirname(os.path.abspath(src))
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    out = tempfile.mktemp(suffix=".s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                    "--cuda-device-only", "-S", "-I", os.path.join(os.path.dirname(__file__), "..", "include"),
                    os.path.join(d, os.path.basename(src)), "-o", out], check=True, cwd=d)
    cur, rows = None, {}
    for line in open(out):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            rows[cur] = {"valu": 0, "salu": 0, "vmem": 0, "lds": 0, "waitcnt": 0}
            continue
        if cur is None:
            continue
        if line.startswith("\t.end_amdhsa_kernel") or line.startswith(".Lfunc_end"):
            cur = None
            continue
        s = line.strip()
        if not s or s.startswith((".", ";")):
            continue
        op = s.split()[0]
        r = rows[cur]
        if op.startswith("s_waitcnt"):
            r["waitcnt"] += 1
        elif op.startswith("v_"):
            r["valu"] += 1
        elif op.startswith(("buffer_", "global_", "flat_")):
            r["vmem"] += 1
        elif op.startswith("ds_"):
            r["lds"] += 1
        elif op.startswith("s_"):
            r["salu"] += 1
    os.unlink(out)
    for n, r in rows.items():
        if flt and flt not in n:
            continue
        print(f"{n[:90]:90s} " + " ".join(f"{k}={v}" for k, v in r.items()))


if __name__ == "__main__":
    main()
