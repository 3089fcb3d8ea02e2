"""Per-loop scratch (spill) instruction counts of a kernel in a hipcc --save-temps .s

Usage: python tools/isa_spills.py <file.s> <mangled kernel name> ...
"""
import collections
import re
import sys


def analyze(s, name):
    st = [i for i, l in enumerate(s) if l.startswith(name + ':')][0]
    en = st
    while not s[en].startswith('.Lfunc_end'):
        en += 1
    labels = {}
    for i in range(st, en):
        m = re.match(r'^(\.LBB\w+):', s[i])
        if m:
            labels[m.group(1)] = i
    loops = []
    for i in range(st, en):
        m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\w+)', s[i])
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    print(name, 'lines', en - st)
    groups = collections.defaultdict(list)
    for i in range(st, en):
        if 'scratch_' in s[i]:
            inner = [(a, b) for a, b in loops if a <= i <= b]
            key = min(inner, key=lambda x: x[1] - x[0]) if inner else None
            groups[key].append(i)
    for key, v in sorted(groups.items(), key=lambda kv: (kv[0] or (0, 0))):
        if key:
            body = s[key[0]:key[1]]
            c = collections.Counter(l.strip().split()[0] for l in body if l.strip() and not l.strip().startswith(('.', ';')))
            desc = f"ds_read {c['ds_read_b32']} alignbit {c['v_alignbit_b32']} gload {sum(n for k, n in c.items() if k.startswith('global_load'))}"
            print(f"  loop {key[0]-st}-{key[1]-st}: {len(v)} scratch ops; body {desc}")
        else:
            print(f"  outside loops: {len(v)} scratch ops")


if __name__ == '__main__':
    lines = open(sys.argv[1]).read().split('\n')
    for n in sys.argv[2:]:
        analyze(lines, n)
