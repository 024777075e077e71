#!/usr/bin/env python3
"""VALU opcode mix of one kernel in a gfx950 device .s file:

    tools/isa_mix.py FILE.s KERNEL_SUBSTRING [--block PATTERN] [--json]

Without --block the histogram covers the whole function (wta_hv_kernel is
straight-line, so static = dynamic per wave).  With --block
it covers only the basic blocks whose text contains PATTERN (e.g.
ds_bpermute for ref_plane3_kernel's per-plane body).  Opcodes are folded to
the classes tools/microbench_valu.hip times (dpp / sdwa / e32 / e64 suffixes
dropped, DPP forms kept apart because they issue differently)."""
import json
import re
import sys


def classify(line):
    s = line.strip()
    if not s.startswith("v_"):
        return None
    op = s.split()[0]
    dpp = " row_" in s or "quad_perm" in s or "row_bcast" in s or "row_mirror" in s \
        or "row_half_mirror" in s or "wave_" in s
    for suf in ("_e32", "_e64", "_sdwa", "_dpp"):
        if op.endswith(suf):
            op = op[: -len(suf)]
    return op + ("+dpp" if dpp else "")


def blocks_of(lines):
    """[(label, [lines])] basic blocks of one function's body."""
    out, cur, label = [], [], "entry"
    for ln in lines:
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            out.append((label, cur))
            cur, label = [], m.group(1)
            continue
        cur.append(ln)
        if ln.strip().startswith(("s_branch", "s_cbranch")):
            out.append((label, cur))
            cur, label = [], label + "+"
    out.append((label, cur))
    return out


def function_lines(path, name):
    body, on = [], False
    for ln in open(path):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            on = name in m.group(1)
            continue
        if on and (ln.startswith(".Lfunc_end") or ln.startswith("\t.end_amdhsa_kernel")):
            break
        if on:
            body.append(ln)
    return body


def mix(path, name, block=None):
    lines = function_lines(path, name)
    if block:
        sel = []
        for _, b in blocks_of(lines):
            if any(block in x for x in b):
                sel.extend(b)
        lines = sel
    h = {}
    for ln in lines:
        c = classify(ln)
        if c:
            h[c] = h.get(c, 0) + 1
    return dict(sorted(h.items(), key=lambda kv: -kv[1]))


def main():
    args = sys.argv[1:]
    block = None
    if "--block" in args:
        i = args.index("--block")
        block = args[i + 1]
        del args[i:i + 2]
    as_json = "--json" in args
    args = [a for a in args if a != "--json"]
    h = mix(args[0], args[1], block)
    if as_json:
        print(json.dumps(h))
        return
    tot = sum(h.values())
    print(f"{tot} VALU instructions")
    for k, v in h.items():
        print(f"  {k:32s} {v:6d}  {100.0 * v / tot:5.1f} %")


if __name__ == "__main__":
    main()
