"""Per-basic-block instruction census of one kernel in a gfx950 .s file:
LDS reads, scratch spills/reloads, VALU, VMEM.  Usage:
    python tools/isa_blocks.py build/srtp_kernels-hip-amdgcn-amd-amdhsa-gfx950.s k_protect [min_ds]"""
import re, sys

path, kern = sys.argv[1], sys.argv[2]
min_ds = int(sys.argv[3]) if len(sys.argv) > 3 else 1
lines = open(path).read().split('\n')
start = next(i for i, l in enumerate(lines) if re.match(r'^_ZN4srtp\d+%sE' % kern, l) or re.match(r'^_ZN4srtp\d+%sENS' % kern, l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
blocks, cur = [], ['entry', 0, 0, 0, 0, 0, 0]
for l in lines[start:end]:
    m = re.match(r'^(\.LBB\d+_\d+):', l) or re.match(r'^; (%bb\.\d+):', l)
    if m:
        blocks.append(cur); cur = [m.group(1), 0, 0, 0, 0, 0, 0]; continue
    t = l.strip().split(' ')[0]
    if not t or t.startswith(('.', ';')):
        continue
    cur[6] += 1
    if t.startswith('ds_read') or t.startswith('ds_load'): cur[1] += 1
    elif t.startswith('scratch_store'): cur[2] += 1
    elif t.startswith('scratch_load'): cur[3] += 1
    elif t.startswith('v_'): cur[4] += 1
    elif t.startswith(('global_', 'buffer_', 'flat_')): cur[5] += 1
blocks.append(cur)
tot = [0] * 7
for b in blocks:
    for i in range(1, 7): tot[i] += b[i]
    if b[1] >= min_ds or b[2] + b[3] >= 8:
        print('%-14s ds=%4d spill_st=%3d spill_ld=%3d valu=%5d vmem=%3d instrs=%5d' % tuple(b))
print('TOTAL %d blocks: ds=%d spill_st=%d spill_ld=%d valu=%d vmem=%d instrs=%d' % (len(blocks), *tot[1:]))

if len(sys.argv) > 4:  # instruction mix of one block
    want, mix, on = sys.argv[4], {}, False
    for l in lines[start:end]:
        m = re.match(r'^(\.LBB\d+_\d+):', l) or re.match(r'^; (%bb\.\d+):', l)
        if m:
            on = m.group(1) == want; continue
        t = l.strip().split(' ')[0]
        if on and t and not t.startswith(('.', ';')):
            mix[t] = mix.get(t, 0) + 1
    for k, v in sorted(mix.items(), key=lambda kv: -kv[1])[:25]:
        print('%6d %s' % (v, k))
