#!/usr/bin/env python3
"""Fold rocprofv3 PMC passes (tools/pmc_conv.sh output) into profiles/<tag>_trunk_pmc.json.

Per-dispatch averages over the dispatches whose kernel name contains --kernel, with the
corrections of MI355X_MICROARCH.md's HBM/rocprofv3 section: FETCH_SIZE / WRITE_SIZE are KiB,
and gfx950's FETCH_SIZE counts 64 B per 128 B request (x2).  GRBM_GUI_ACTIVE is summed over the
8 XCDs, so the effective clock is GRBM/8 / duration and MFMA busy is SQ_VALU_MFMA_BUSY_CYCLES
over (GRBM/8 x 256 CUs x 4 SIMDs).

  python3 tools/pmc_summary.py gpurun_out/pmc_fp16 --kernel conv3x3_v6 --out profiles/r01_fp16_v6_trunk_pmc.json
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_dispatch(path, kernel):
    vals = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                key = (f, r["Dispatch_Id"])
                vals[key][r["Counter_Name"]] = vals[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = collections.defaultdict(list)
    for d in vals.values():
        for k, v in d.items():
            out[k].append(v)
    return {k: sum(v) / len(v) for k, v in out.items()}, len(vals)


def avg_duration_ns(path, kernel):
    for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Name"]:
                return float(r["AverageNs"]), r["Name"]
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="conv3x3_v6")
    ap.add_argument("--out", required=True)
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--boards", type=int, default=2048)
    ap.add_argument("--board", type=int, default=15)
    ap.add_argument("--channels", type=int, default=256)
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--game", default="gomoku15", help="tools/net_bench.py --game of the profiled run")
    a = ap.parse_args()
    c = {}
    n = 0
    for sub in ("sq", "fetch", "write"):
        v, k = per_dispatch(os.path.join(a.dir, sub), a.kernel)
        c.update(v)
        n = max(n, k)
    dur, name = avg_duration_ns(os.path.join(a.dir, "trace"), a.kernel)
    rd = c["FETCH_SIZE"] * 1024 * 2
    wr = c["WRITE_SIZE"] * 1024
    B, C, HW = a.boards, a.channels, a.board * a.board
    x3 = a.precision in ("bf16x3", "f16x3")
    act = B * HW * C * (4 if x3 else 2)          # bf16x3 / f16x3: hi + lo 16-bit planes; fp16: one 16-bit plane
    out = {"kernel": name or a.kernel,
           "workload": f"tools/net_bench.py --game {a.game} --precision {a.precision} --batch {B}: "
                       f"{'C3' if a.game == 'gomoku15' else a.game} net forward, B={B} boards per launch "
                       f"({2 * a.blocks} trunk launches per forward)",
           "command": "tools/pmc_conv.sh (rocprofv3 --kernel-trace --stats pass, then separate --pmc passes: "
                      "SQ/GRBM, FETCH_SIZE, WRITE_SIZE)",
           "dispatches": n, "avg_duration_ns": dur}
    out.update(c)
    out.update({"hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                "hbm_bytes_per_launch": rd + wr, "boards_per_launch": B,
                "algorithmic_bytes_per_launch":
                    {"activations_in": act, "residual_in_avg": act / 2 if x3 else act * 1.5 / 2,
                     "out_avg": act if x3 else act * 1.25, "weights": 9 * C * C * (4 if x3 else 2)},
                "algorithmic_note":
                    (f"g8 hi + lo activations {B}x{HW}x{C}x4 B = {act / 1e6:.0f} MB in and out per launch; "
                     "the 2nd conv of a block also reads the residual (hi + lo); weights hi + lo 2.4 MB") if x3 else
                    (f"g8 activations {B}x{HW}x{C}x2 B = {act / 1e6:.0f} MB in and out per launch; "
                     "the 2nd conv of a block also reads the residual (16-bit + int8) and writes the "
                     "int8 remainder; weights 1.2 MB")})
    if dur and "GRBM_GUI_ACTIVE" in c:
        clk = c["GRBM_GUI_ACTIVE"] / 8 / dur
        out["clock_ghz_effective"] = clk
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            out["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
        out["hbm_GB_per_s"] = (rd + wr) / dur
    out.update({"precision": a.precision, "board": a.board, "channels": a.channels, "blocks": a.blocks})
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
