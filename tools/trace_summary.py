"""Per-kernel average durations from a rocprofv3 kernel trace (csv), grouped
by kernel name and by launch position within a step.  Usage:
    python tools/trace_summary.py gpurun_out/prof/trace/run_kernel_trace.csv"""
import collections, csv, sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    short = name.split("(")[0].replace("srtp::", "")
    if "rocprim" in name:
        short = "rocprim::" + ("onesweep_iteration" if "onesweep_iteration" in name else
                               "histogram" if "histogram" in name else "other")
    agg[short].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[:60]:60s} n={len(v):4d} avg={sum(v)/len(v)/1e3:9.1f} us  total={sum(v)/1e6:8.3f} ms  {100*sum(v)/tot:5.1f}%")
