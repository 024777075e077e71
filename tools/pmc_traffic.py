#!/usr/bin/env python3
"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, as
MI355X_MICROARCH.md's HBM section prescribes) into per-launch HBM bytes.

gfx950 correction: FETCH_SIZE reports 1/2 of the bytes of a wide coalesced
stream.  When the run has wta_paths_kernel (the 8-volume route) we calibrate
on it instead of assuming: it reads exactly the 8 path volumes (8*W*H*D bytes,
each byte once, dwordx2-wide like sgm_paths), so fetch_scale = known_bytes /
(FETCH_SIZE*1024); otherwise the guide's factor 2.0 applies (calibrated on
wta_paths_kernel at 2.0 in round 1).  WRITE_SIZE is exact for these store
widths.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR W H D OUT.json
"""
import collections
import csv
import json
import os
import sys

SHORT = {
    "sgm_paths_kernel": "sgm_paths",
    "hamming_cost2_kernel": "cost2", "fuse_depth_kernel": "fuse_depth",
    "hamming_cost_rows_kernel": "cost", "census9x7_rows_kernel": "census",
    "census_cost_mma_kernel": "cost", "wta_hv_kernel": "wta_hv",
}


def per_kernel(dirname):
    path = os.path.join(dirname, "run_counter_collection.csv")
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        for key, short in SHORT.items():
            if key + "<" in name or key + "(" in name:
                agg[short].append(float(r["Counter_Value"]))
                break
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    fdir, wdir, W, H, D, out = sys.argv[1], sys.argv[2], *map(int, sys.argv[3:6]), sys.argv[6]
    fetch, write = per_kernel(fdir), per_kernel(wdir)
    known_wta_read = 8 * W * H * D
    scale = known_wta_read / (fetch["wta"] * 1024) if "wta" in fetch else 2.0
    res = {"workload": f"{W}x{H} D={D}", "fetch_scale_calibrated_on_wta": round(scale, 4),
           "units": "bytes per launch", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, 0.0) * 1024 * scale
        wb = write.get(k, 0.0) * 1024
        res["kernels"][k] = {"fetch_raw_kb": fetch.get(k), "write_raw_kb": write.get(k),
                             "hbm_read_bytes": int(fb), "hbm_write_bytes": int(wb),
                             "hbm_bytes_per_launch": int(fb + wb)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
