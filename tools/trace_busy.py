"""GPU occupancy of a rocprofv3 kernel + memory-copy trace (csv):
kernels and copies per name / direction, the fraction of the window in which a
kernel runs, a copy runs, either, and both at once.

Usage: python tools/trace_busy.py <dir holding *_kernel_trace.csv [*_memory_copy_trace.csv]>"""
import collections
import csv
import glob
import os
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def total(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    t = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            t += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return t


def main(d):
    kt = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    rows = list(csv.DictReader(open(kt)))
    k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    mc = glob.glob(os.path.join(d, "*memory_copy_trace.csv"))
    m = []
    if mc:
        m = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"]) for r in csv.DictReader(open(mc[0]))]
    t0 = min(s for s, _, _ in k + m)
    t1 = max(e for _, e, _ in k + m)
    win = t1 - t0
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n in k + m:
        key = n.split("(")[0].replace("void ", "")[:48]
        per[key][0] += 1
        per[key][1] += e - s
    print(f"window {win / 1e6:.1f} ms")
    for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"  {n:50s} {c:7d} x {t / c / 1e3:8.1f} us = {t / 1e6:8.1f} ms")
    ku, mu = union([(s, e) for s, e, _ in k]), union([(s, e) for s, e, _ in m])
    print(f"kernel busy {total(ku) / win:.3f}  copy busy {total(mu) / win:.3f}  "
          f"either {total(union(ku + mu)) / win:.3f}  both {intersect(ku, mu) / win:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
