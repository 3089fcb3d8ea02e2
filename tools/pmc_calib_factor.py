"""FETCH_SIZE / WRITE_SIZE calibration factors from a tools/pmc_calib run
(rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, each into <dir>/fetch and
<dir>/write).  For each calibration kernel, the bytes it must move (every byte
read / written exactly once) over the counter's bytes per launch: the factor
that turns the counter into bytes for that access pattern.

    python tools/pmc_calib_factor.py <dir>   ->  <dir>/factor.json and a table
"""
import csv
import glob
import json
import os
import sys

N, LEN, STRIDE = 262144, 1200, 1216
SEG, PAY = N * STRIDE, N * LEN
# kernel -> (bytes read, bytes written) per launch
MOVED = {
    "k_stream_rd": (SEG, 0), "k_stream_rw": (SEG, SEG), "k_lane_rd": (PAY, 0),
    "k_lane_rw": (PAY, PAY), "k_lane_rw4": (N * 1152, N * 1152), "k_lane_rw4t": (N * 1152, N * 1152),
    "k_lane_rw8": (N * 1152, N * 1152), "k_lane_w4": (0, N * 1152), "k_lane_rw4nt": (N * 1152, N * 1152),
    "k_lane_rw4_half": (N * 1152, N * 1152),
}


def per_kernel(path):
    f = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter CSV under {path}")
    acc = {}
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].split("(")[0].split()[-1]
        acc.setdefault(name, []).append(float(r["Counter_Value"]) * 1024.0)  # KB -> B
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d = sys.argv[1]
    fetch, write = per_kernel(os.path.join(d, "fetch")), per_kernel(os.path.join(d, "write"))
    out = {}
    for k, (rd, wr) in MOVED.items():
        if k not in fetch:
            continue
        out[k] = {"bytes_read": rd, "bytes_written": wr, "fetch_size_bytes": round(fetch[k]),
                  "write_size_bytes": round(write.get(k, 0.0)),
                  "read_factor": round(rd / fetch[k], 3) if fetch[k] and rd else None,
                  "write_factor": round(wr / write[k], 3) if write.get(k) and wr else None}
    json.dump(out, open(os.path.join(d, "factor.json"), "w"), indent=1)
    print("%-16s %12s %12s %8s %8s" % ("kernel", "FETCH B", "WRITE B", "rd fac", "wr fac"))
    for k, v in out.items():
        print("%-16s %12d %12d %8s %8s" % (k, v["fetch_size_bytes"], v["write_size_bytes"],
                                          v["read_factor"], v["write_factor"]))


if __name__ == "__main__":
    main()
