#!/usr/bin/env python3
"""How much of Mode R's offset-plane work is used:
per reference-rig pair, the pixel-SADs the plane kernel computes against the
candidate SADs the reference evaluates.

ref_plane3_kernel (refpath.hip) gives every wave 8 rows x 64 columns of a
64 x 32 tile and evaluates, for every offset plane in the union of the tile's
pixels' Bresenham offsets, the box sums of all 512 of its pixels; a pixel
uses only the planes on its own line (functions.cpp:253-321).  This script
samples tiles of a W x H frame (endpoints from the oracle's restatement of
CameraStereoVision.cpp:60-71), forms each pixel's offset set with the same
closed-form Bresenham as the kernel, and reports

  tile_ratio  = sum over sampled tiles of 4 waves x |tile union| x 512
                / candidates used,
  wave_ratio  = the same with per-wave unions (what a per-wave plane skip
                could reach),
  rows_of_offsets = distinct minor offsets of the tile union (the 1-3 offset
                rows that the off-by-one endpoint rows create).

    python tools/mode_r_planes.py [--size 1920x1080] [--pairs 12-11,12-7,12-6,12-18] [--k 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def line_offsets(x, y, a, b):
    """Offsets (cx - x, cy - y) of bresenham(pixel1 = a, pixel2 = b) in the
    closed form of refpath.hip make_line / line_point."""
    ax, ay, bx, by = int(a[0]), int(a[1]), int(b[0]), int(b[1])
    pts = []
    if abs(ay - by) < abs(ax - bx):
        x0, y0, x1, y1 = (ax, ay, bx, by) if bx > ax else (bx, by, ax, ay)
        dx, dy = x1 - x0, y1 - y0
        st = -1 if dy < 0 else 1
        aa, bb = 2 * abs(dy), 2 * dx
        for i in range(dx + 1):
            m = (aa * i + dx - 1) // bb if bb > 0 else 0
            pts.append((x0 + i - x, y0 + st * m - y))
    else:
        x0, y0, x1, y1 = (ax, ay, bx, by) if by > ay else (bx, by, ax, ay)
        dx, dy = x1 - x0, y1 - y0
        st = -1 if dx < 0 else 1
        aa, bb = 2 * abs(dx), 2 * dy
        for i in range(dy + 1):
            m = (aa * i + dy - 1) // bb if bb > 0 else 0
            pts.append((x0 + st * m - x, y0 + i - y))
    return pts


def pair_ratio(W, H, k, i_ref, i_oth, tiles, ends=None, ok=None):
    """ends / ok: the pixels' endpoints [H][W][4] and valid mask [H][W] when
    the caller has them (bench.py passes the GPU's own sva_ref_endpoints_d
    output); otherwise they come from the oracle's restatement."""
    from stereovisionarray_amd import synth
    g = synth.reference_array(0.036 / W)
    if ends is None:
        import pyoracle as o
        cr, co = o.OCamera.make(*g[i_ref]), o.OCamera.make(*g[i_oth])
    tot_tile = tot_wave = used = 0
    minor_rows = []
    for (tx, ty) in tiles:
        tx0, ty0 = k + tx * 64, k + ty * 32
        tile, waves = set(), [set() for _ in range(4)]
        for r in range(32):
            for c in range(64):
                x, y = tx0 + c, ty0 + r
                if x >= W - k or y >= H - k:
                    continue
                if ends is None:
                    okp, a, b = o.ref_endpoints(cr, co, W, H, k, 0.5, 1.0, x, y)
                else:
                    okp, a, b = bool(ok[y, x]), ends[y, x, :2], ends[y, x, 2:]
                if not okp:
                    continue
                offs = set(line_offsets(x, y, a, b))
                used += len(offs)
                tile |= offs
                waves[r // 8] |= offs
        tot_tile += 4 * len(tile) * 512
        tot_wave += sum(len(w) for w in waves) * 512
        horiz = abs(g[i_oth][1][0] - g[i_ref][1][0]) >= abs(g[i_oth][1][1] - g[i_ref][1][1])
        minor_rows.append(len({(p[1] if horiz else p[0]) for p in tile}))
    return {"pair": f"{i_ref}->{i_oth}", "tiles_sampled": len(tiles), "candidates_used": used,
            "tile_ratio": round(tot_tile / used, 3) if used else None,
            "wave_ratio": round(tot_wave / used, 3) if used else None,
            "minor_offsets_per_tile": minor_rows}


def sample_tiles(W, H, k):
    gx, gy = (W - 2 * k + 63) // 64, (H - 2 * k + 31) // 32
    return [(int(gx * fx), int(gy * fy)) for fx, fy in ((0.15, 0.1), (0.5, 0.5), (0.8, 0.6), (0.3, 0.9))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--pairs", default="12-11,12-7,12-6,12-18")
    ap.add_argument("--k", type=int, default=20)
    a = ap.parse_args()
    W, H = (int(v) for v in a.size.split("x"))
    for p in a.pairs.split(","):
        i, j = (int(v) for v in p.split("-"))
        r = pair_ratio(W, H, a.k, i, j, sample_tiles(W, H, a.k))
        r["size"] = a.size
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
