"""Summarise rocprofv3 runs of bench.py (kernel trace + --pmc passes) per kernel.

Usage:
    python tools/pmc_summary.py <prof_dir> [--packets N --len L --out profiles/rNN]

<prof_dir> holds trace/run_kernel_trace.csv and <pass>/run_counter_collection.csv
for the passes tools/prof.sh writes (fetch, write, sq, sq2).  Prints, per
kernel of the SRTP pipeline, the average duration and every counter averaged
over dispatches, then derived figures for k_protect / k_unprotect:

* HBM traffic per launch.  FETCH_SIZE (KB) is TCC_EA0_RDREQ x 64 B and counts
  half the bytes of a 16-B-per-lane coalesced read stream on gfx950
  (MI355X_MICROARCH.md, HBM section): the guide's correction is FETCH_SIZE x 2
  + WRITE_SIZE x 1.  The kernels' own pattern (one lane per packet, 16-B
  accesses walking each packet in 64-B chunks) is calibrated separately by
  tools/pmc_calib.hip (its k_lane_rw4 moves every byte of 2^18 such packets
  exactly once): with --calib <factor.json> (tools/pmc_calib_factor.py)
  traffic = FETCH_SIZE x read_factor + WRITE_SIZE x write_factor of k_lane_rw4,
  and the guide's figure is kept beside it.
* VALU / LDS issue: instructions per wave, LDS-array cycles, bank conflicts,
  effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration).

With --out, writes <out>/pmc_summary.txt and profiles/pmc_traffic.json (read
by bench.py to fill roofline.traffic).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import sys

KERNELS = ("k_parse", "k_sort_scatter", "k_unprotect", "k_walk<true>", "k_walk<false>", "k_protect",
           "k_unprotect_fix", "k_ext")


def short(name: str) -> str:
    if "rocprim" in name:
        return "rocprim::" + ("onesweep" if "onesweep_iteration" in name else
                              "histogram" if "histogram" in name else "other")
    n = name.split("(")[0].replace("srtp::", "").replace("void ", "")
    # the full-bundle instances of the crypto kernels keep their plain names
    return n.replace("k_protect<false>", "k_protect").replace("k_unprotect<false>", "k_unprotect")


def load_trace(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return agg


def load_pmc(path):
    """{kernel: {counter: [values per dispatch]}} and durations per dispatch."""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return vals, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--packets", type=int, default=1 << 18)
    ap.add_argument("--len", type=int, default=1200)
    ap.add_argument("--tag", type=int, default=10)
    ap.add_argument("--out")
    ap.add_argument("--calib", help="factor.json of tools/pmc_calib_factor.py")
    ap.add_argument("--kernels", default="k_protect,k_unprotect",
                    help="kernels to derive figures for (the split path: k_ctr_wide<false>,k_mac_wide<true>, ...)")
    a = ap.parse_args()
    calib = None
    if a.calib:
        calib = json.load(open(a.calib)).get("k_lane_rw4")
    lines = []
    P = lines.append
    trace = load_trace(os.path.join(a.prof_dir, "trace", "run_kernel_trace.csv"))
    P(f"{'kernel':34s} {'n':>4s} {'avg us':>9s} {'total ms':>9s}")
    for k, v in sorted(trace.items(), key=lambda kv: -sum(kv[1])):
        if k.startswith("at::") or "elementwise" in k or "reduce_kernel" in k:
            continue
        P(f"{k[:34]:34s} {len(v):4d} {sum(v) / len(v) / 1e3:9.1f} {sum(v) / 1e6:9.3f}")
    counters = collections.defaultdict(dict)
    pass_dur = collections.defaultdict(list)
    for pas in sorted(os.listdir(a.prof_dir)):
        f = os.path.join(a.prof_dir, pas, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        vals, dur = load_pmc(f)
        for k, cs in vals.items():
            for c, v in cs.items():
                counters[k][c] = sum(v) / len(v)
            pass_dur[k] += list(dur[k].values())
    derived = {}
    for k in a.kernels.split(","):
        c = counters.get(k)
        if not c:
            continue
        P("")
        P(f"{k}: counters averaged per dispatch")
        for name in sorted(c):
            P(f"  {name:24s} {c[name]:16.1f}")
        waves = c.get("SQ_WAVES", 0) or (a.packets / 64)
        avg_us = sum(trace[k]) / len(trace[k]) / 1e3
        d = {"avg_us_trace": round(avg_us, 2)}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            alg = a.packets * (a.len + a.len + a.tag)
            rd_g, wr_g = c["FETCH_SIZE"] * 1024 * 2, c["WRITE_SIZE"] * 1024
            d.update(guide_read_bytes=rd_g, guide_write_bytes=wr_g,
                     guide_traffic_over_algorithmic=round((rd_g + wr_g) / alg, 3))
            if calib:
                rd = c["FETCH_SIZE"] * 1024 * calib["read_factor"]
                wr = c["WRITE_SIZE"] * 1024 * calib["write_factor"]
            else:
                rd, wr = rd_g, wr_g
            d.update(hbm_read_bytes=rd, hbm_write_bytes=wr, hbm_bytes=rd + wr,
                     algorithmic_bytes=alg, traffic_over_algorithmic=round((rd + wr) / alg, 3))
        for name in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                     "SQ_INSTS_VMEM_WR"):
            if name in c:
                d[name.lower() + "_per_wave"] = round(c[name] / waves, 1)
        if "SQ_LDS_IDX_ACTIVE" in c:
            d["lds_busy_frac"] = round(c["SQ_LDS_IDX_ACTIVE"] / (256 * avg_us * 1e-6 *
                                                                 (c.get("GRBM_GUI_ACTIVE", 0) / 8 /
                                                                  (avg_us * 1e-6) if "GRBM_GUI_ACTIVE" in c else 2.4e9)), 3)
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
            d["lds_bank_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / max(1, c["SQ_LDS_IDX_ACTIVE"]), 4)
        if "GRBM_GUI_ACTIVE" in c:
            d["eff_clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (avg_us * 1e3), 3)
            if "SQ_INSTS_VALU" in c:
                # a wave64 VALU instruction occupies a SIMD-32 for 2 cycles; 1024 SIMDs
                cyc = c["GRBM_GUI_ACTIVE"] / 8
                d["valu_busy_frac"] = round(c["SQ_INSTS_VALU"] * 2 / (1024 * cyc), 3)
                # at the issue rate tools/valu_bench.hip measures for the loop's
                # instructions (1.28 cycles per wave64 instruction per SIMD, 4 waves/SIMD)
                d["valu_busy_frac_measured_rate"] = round(c["SQ_INSTS_VALU"] * 1.28 / (1024 * cyc), 3)
        if "SQ_BUSY_CYCLES" in c:
            d["sq_busy_cycles"] = c["SQ_BUSY_CYCLES"]
        for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                     "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if name in c and "SQ_WAVE_CYCLES" in c:
                d[name.lower() + "_frac_of_wave_cycles"] = round(c[name] / c["SQ_WAVE_CYCLES"], 3)
        derived[k] = d
        P(f"{k}: derived")
        for name, v in d.items():
            P(f"  {name:40s} {v}")
    text = "\n".join(lines)
    print(text)
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, "pmc_summary.txt"), "w") as f:
            f.write(text + "\n")
        kp = derived.get("k_protect", {})
        if "hbm_bytes" in kp:
            js = {"packets": a.packets, "len": a.len, "source": os.path.join(a.out, "pmc_summary.txt"),
                  "method": (("FETCH_SIZE x %.3f + WRITE_SIZE x %.3f (x 1024) per dispatch: the factors "
                              "tools/pmc_calib.hip measures for the kernels' access pattern (k_lane_rw4); "
                              "separate --pmc passes" % (calib["read_factor"], calib["write_factor"]))
                             if calib else
                             "FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024 per dispatch (separate --pmc passes; "
                             "gfx950 half-count correction on reads)"),
                  "guide_correction_bytes_per_launch": {
                      "k_protect": round(kp["guide_read_bytes"] + kp["guide_write_bytes"])},
                  "k_protect_bytes_per_launch": round(kp["hbm_bytes"]),
                  "k_protect_read_bytes": round(kp["hbm_read_bytes"]),
                  "k_protect_write_bytes": round(kp["hbm_write_bytes"])}
            js["k_protect_utilisation"] = {
                k: kp.get(k) for k in ("valu_busy_frac", "lds_busy_frac", "lds_bank_conflict_frac",
                                       "eff_clock_ghz")}
            ku = derived.get("k_unprotect", {})
            js["k_unprotect_utilisation"] = {
                k: ku.get(k) for k in ("valu_busy_frac", "lds_busy_frac", "lds_bank_conflict_frac",
                                       "eff_clock_ghz")}
            if "hbm_bytes" in ku:
                js["guide_correction_bytes_per_launch"]["k_unprotect"] = round(
                    ku["guide_read_bytes"] + ku["guide_write_bytes"])
                js.update({"k_unprotect_bytes_per_launch": round(ku["hbm_bytes"]),
                           "k_unprotect_read_bytes": round(ku["hbm_read_bytes"]),
                           "k_unprotect_write_bytes": round(ku["hbm_write_bytes"])})
            root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            sys.path.insert(0, root)
            from libjitsi_amd._native import kernel_source_sha16
            # the build these counters measured (bench.py marks them stale otherwise)
            js["kernel_source_sha16"] = kernel_source_sha16()
            with open(os.path.join(root, "profiles", "pmc_traffic.json"), "w") as f:
                json.dump(js, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
