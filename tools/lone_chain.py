"""The per-call chain of a lone synchronous caller from a rocprofv3 kernel +
memory-copy trace of `sync_bench 1 one 0 1 rt`: for the last calls, each
operation's start relative to the call's first operation and its duration,
then the average duration per kernel / copy and the average span of a call.

Usage: python tools/lone_chain.py <dir holding run_kernel_trace.csv, run_memory_copy_trace.csv>"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
ev = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r["Kernel_Name"].split("(")[0].replace("srtp::", "").replace("void ", "")))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")))
ev.sort()
# a call = the events from one H2D copy burst to the next after a gap of > 20 us with nothing running
calls, cur, last_end = [], [], None
for s, e, n in ev:
    if cur and s - last_end > 20_000:
        calls.append(cur)
        cur = []
    cur.append((s, e, n))
    last_end = max(last_end or e, e)
if cur:
    calls.append(cur)
calls = calls[len(calls) // 4:]  # skip the warm-up
per = collections.defaultdict(list)
spans = []
for c in calls:
    spans.append(max(e for _, e, _ in c) - c[0][0])
    for s, e, n in c:
        per[n].append(e - s)
print(f"calls {len(calls)}, span per call (first op start -> last op end): "
      f"avg {sum(spans) / max(len(spans), 1) / 1e3:.1f} us, median {sorted(spans)[len(spans) // 2] / 1e3:.1f} us")
for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {n[:44]:44s} {len(v) / max(len(calls), 1):5.1f} per call  avg {sum(v) / len(v) / 1e3:7.1f} us")
print("one call:")
c = calls[len(calls) // 2]
for s, e, n in c:
    print(f"  {(s - c[0][0]) / 1e3:8.1f} .. {(e - c[0][0]) / 1e3:8.1f} us  {n}")
