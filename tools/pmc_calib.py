#!/usr/bin/env python3
"""Split tools/pmc_calib.sh's per-dispatch counters of conv3x3_v7 into the two convs of a residual
block (the trunk alternates conv1: input halo only / conv2: input halo + residual join), and set
each against its algorithmic bytes at C3 (B = 2048, 15x15, 256 channels):

  conv1 reads the g8 16-bit input (2048 x 225 x 256 x 2 B = 235.9 MB) + 1.2 MB weights, writes 235.9 MB;
  conv2 also reads the residual (16-bit 235.9 MB + int8 remainder 118.0 MB) and writes both planes.

FETCH_SIZE is reported raw and doubled (MI355X_MICROARCH.md: gfx950 tallies a wide streaming read at
half its bytes); the request-size counters give the bytes directly (64 x RDREQ_64B + 128 x RDREQ_128B);
conv2 - conv1 isolates the residual loads (8-B / 4-B per lane).

  python3 tools/pmc_calib.py gpurun_out/calib --out profiles/r06_c3_fp16_pmc_calib.json
"""
import argparse
import collections
import csv
import glob
import json
import os

B, HW, C = 2048, 225, 256
ACT16 = B * HW * C * 2
ACT8 = B * HW * C
WEIGHTS = 9 * C * C * 2
ALG = {"conv1": {"read": ACT16 + WEIGHTS, "write": ACT16},
       "conv2": {"read": ACT16 + WEIGHTS + ACT16 + ACT8, "write": ACT16 + ACT8}}


def dispatches(path, kernel):
    vals = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                key = int(r["Dispatch_Id"])
                vals[key][r["Counter_Name"]] = vals[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                vals[key]["duration_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="conv3x3_v7")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    res = {"kernel": a.kernel, "workload": "tools/net_bench.py --game gomoku15 --batch 2048 --precision fp16",
           "algorithmic_bytes": ALG, "classes": {}}
    for sub in ("fetch", "req", "hit", "write", "wrreq"):
        d = dispatches(os.path.join(a.dir, sub), a.kernel)
        if not d:
            continue
        for cls, par in (("conv1", 0), ("conv2", 1)):
            sel = d[par::2]
            avg = {k: sum(x.get(k, 0.0) for x in sel) / len(sel) for k in sel[0]}
            c = res["classes"].setdefault(cls, {"dispatches": len(sel)})
            dur = avg.pop("duration_us")
            c.update({f"{k}": v for k, v in avg.items()})
            c.setdefault("duration_us_per_pass", {})[sub] = dur
    for cls, c in res["classes"].items():
        alg = ALG[cls]
        if "FETCH_SIZE" in c:
            raw = c["FETCH_SIZE"] * 1024
            c["fetch_bytes_raw"] = raw
            c["fetch_bytes_x2"] = 2 * raw
            c["read_over_alg_x2"] = 2 * raw / alg["read"]
            c["read_over_alg_raw"] = raw / alg["read"]
        if "WRITE_SIZE" in c:
            c["write_over_alg"] = c["WRITE_SIZE"] * 1024 / alg["write"]
        if "TCC_EA0_RDREQ_64B_sum" in c and "TCC_EA0_RDREQ_128B_sum" in c:
            c["rdreq_bytes"] = 64 * c["TCC_EA0_RDREQ_64B_sum"] + 128 * c["TCC_EA0_RDREQ_128B_sum"]
            c["rdreq_bytes_over_alg"] = c["rdreq_bytes"] / alg["read"]
        if "TCC_EA0_WRREQ_sum" in c and "TCC_EA0_WRREQ_64B_sum" in c:   # 32-B and 64-B write requests
            n, n64 = c["TCC_EA0_WRREQ_sum"], c["TCC_EA0_WRREQ_64B_sum"]
            c["wrreq_bytes"] = 64 * n64 + 32 * (n - n64)
            c["wrreq_bytes_over_alg"] = c["wrreq_bytes"] / alg["write"]
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            c["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    k1, k2 = res["classes"].get("conv1", {}), res["classes"].get("conv2", {})
    if "fetch_bytes_raw" in k1 and "fetch_bytes_raw" in k2:
        dr = k2["fetch_bytes_raw"] - k1["fetch_bytes_raw"]
        res["residual_fetch_raw"] = dr
        res["residual_alg"] = ACT16 + ACT8
        res["residual_over_alg_raw"] = dr / (ACT16 + ACT8)
        res["residual_over_alg_x2"] = 2 * dr / (ACT16 + ACT8)
    if "rdreq_bytes" in k1 and "rdreq_bytes" in k2:
        res["residual_rdreq_bytes"] = k2["rdreq_bytes"] - k1["rdreq_bytes"]
        res["residual_rdreq_over_alg"] = res["residual_rdreq_bytes"] / (ACT16 + ACT8)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
