"""Step timeline of a two-stream bench run from a rocprofv3 kernel trace (csv):
for the last N steps, the busy time of each stream's kernels, the time when
both streams run a kernel at once, and the idle gaps with no kernel at all.
Usage: python tools/timeline.py gpurun_out/.../run_kernel_trace.csv [steps]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ev = []
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("srtp::", "")
    # the full-bundle instances of the crypto kernels by their plain names
    name = name.replace("void k_protect<false>", "k_protect").replace("void k_unprotect<false>", "k_unprotect")
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Stream_Id", r.get("Queue_Id", "?"))))
ev.sort()
# one step = one launch of the sender's first crypto kernel (k_protect, or
# k_ctr_wide<false> on the split path); take the span of the last `last` steps
marker = "k_protect" if any(e[2] == "k_protect" for e in ev) else "void k_ctr_wide<false>"
prot = [e for e in ev if e[2] == marker]
if len(prot) < last + 1:
    sys.exit("not enough steps in the trace")
t0, t1 = prot[-last - 1][0], prot[-1][0]
win = [e for e in ev if e[1] > t0 and e[0] < t1]
print(f"window: {last} steps, {(t1 - t0) / 1e3 / last:.1f} us per step")
# sweep: busy / overlap / idle
pts = []
for s, e, n, q in win:
    pts.append((max(s, t0), 1, q))
    pts.append((min(e, t1), -1, q))
pts.sort()
active = collections.Counter()
busy = over = idle = 0
prev = t0
for t, d, q in pts:
    dt = t - prev
    k = sum(1 for v in active.values() if v > 0)
    if k == 0:
        idle += dt
    elif k >= 2:
        over += dt
    busy += dt if k else 0
    active[q] += d
    prev = t
span = t1 - t0
print(f"busy {busy / span:.3f}  two queues at once {over / span:.3f}  idle {idle / span:.3f}")
per = collections.defaultdict(int)
cnt = collections.Counter()
for s, e, n, q in win:
    per[n] += min(e, t1) - max(s, t0)
    cnt[n] += 1
for n, v in sorted(per.items(), key=lambda kv: -kv[1]):
    print(f"  {n[:40]:40s} {v / 1e3 / last:8.1f} us per step  ({cnt[n] / last:.1f} launches)")
# one step's sequence, relative times
print("last step:")
for s, e, n, q in win:
    if s >= prot[-2][0] - 200_000 and s < prot[-1][0]:
        print(f"  q={q:>3} {(s - prot[-2][0]) / 1e3:9.1f} .. {(e - prot[-2][0]) / 1e3:9.1f} us  {n}")
