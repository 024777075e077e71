#!/usr/bin/env python3
"""Build an experiment (ablation) variant of libsva.so from a scratch copy of
stereovisionarray_amd/csrc with literal text replacements applied:

    tools/build_patch_variant.py NAME FILE 'OLD' 'NEW' [FILE 'OLD' 'NEW' ...]

Each OLD must occur in FILE (all occurrences are replaced); OLD = '@' copies
the file at path NEW over FILE.  Output:
$AB_DIR/libsva_NAME.so (default ab_libs/); the product sources and libsva.so are untouched.
Ablation builds compute other values on purpose (run tools/ab_paths.py with
AB_NOCHECK=1)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name, rest = sys.argv[1], sys.argv[2:]
    if len(rest) % 3:
        raise SystemExit("usage: NAME FILE OLD NEW [FILE OLD NEW ...]")
    src = os.path.join(ROOT, "build", f"var_{name}", "src")
    shutil.rmtree(src, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "stereovisionarray_amd", "csrc"), src)
    for i in range(0, len(rest), 3):
        f, old, new = rest[i:i + 3]
        p = os.path.join(src, f)
        if old == "@":                 # replace the whole file by NEW (a path)
            shutil.copy(new, p)
            continue
        t = open(p).read()
        if old not in t:
            raise SystemExit(f"{f}: pattern not found: {old[:80]}")
        open(p, "w").write(t.replace(old, new))
    out = os.environ.get("AB_DIR", "ab_libs")      # ab_run/ for libraries a GPU run loads
    os.makedirs(os.path.join(ROOT, out), exist_ok=True)
    subprocess.run(["make", "-s", "-j8", "-C", src, f"BUILD={ROOT}/build/var_{name}/obj",
                    f"OUT={ROOT}/{out}/libsva_{name}.so", f"INC={ROOT}/include"], check=True)
    print(f"built {out}/libsva_{name}.so")


if __name__ == "__main__":
    main()
