"""gfx950 AES-128 T-table round generator shared by tools/gen_aes_asm.py (the
product's aes_rounds_asm.inc) and tools/aes_bench (the variant micro-benchmark).

A round over B interleaved blocks (state words %[<z>0..3] for z in blocks):
  * every lookup address is one v_perm_b32 of a state word and a per-lane
    table base (see TL() in srtp_kernels.hip);
  * the ds_read_b32 of all blocks are streamed, keeping up to 15 in flight (the
    4-bit lgkmcnt limit), and each output column is folded as soon as its four
    lookups are known to have landed (LDS returns in order).
tables=4: T0..T3 in LDS; column j = T0 ^ T1 ^ T2 ^ T3 ^ rk[j] (2 v_bitop3).
tables=2: T0, T1 in LDS; T2 = rotl16(T0), T3 = rotl16(T1), so column j =
  T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d] ^ rotr16(rk[j])) (2 v_bitop3 + 1 v_alignbit),
  half the LDS image.
"""

MAX_LGKM = 15


def lookups(z, tb, tables):
    out = []
    for j in range(4):
        for t in range(4):
            base = t if tables == 4 else (t & 1)  # table; t is also the state byte
            out.append((f"%[t{tb + 4 * j + t}]", f"%[{z}{(j + t) & 3}]", base, t))
    return out


def consume(z, tb, j, last, tables):
    a, b, c, d = (f"%[t{tb + 4 * j + t}]" for t in range(4))
    if last:
        # S(x): byte 1 of T0 / byte 2 of T1 (tables 2: rotl16 of T0/T1 puts it
        # at byte 3 / byte 0 -- same selectors after the table swap below)
        if tables == 4:
            return [f"v_perm_b32 {a}, {b}, {a}, %[s4]",
                    f"v_perm_b32 {c}, {d}, {c}, %[s5]",
                    f"v_bitop3_b32 %[{z}{j}], {a}, {c}, %[k{j}] bitop3:0x96"]
        return [f"v_perm_b32 {a}, {b}, {a}, %[s4]",
                f"v_perm_b32 {c}, {d}, {c}, %[s6]",
                f"v_bitop3_b32 %[{z}{j}], {a}, {c}, %[k{j}] bitop3:0x96"]
    if tables == 4:
        return [f"v_bitop3_b32 {a}, {a}, {b}, {c} bitop3:0x96",
                f"v_bitop3_b32 %[{z}{j}], {a}, {d}, %[k{j}] bitop3:0x96"]
    return [f"v_bitop3_b32 {c}, {c}, {d}, %[r{j}] bitop3:0x96",
            f"v_alignbit_b32 {c}, {c}, {c}, 16",
            f"v_bitop3_b32 %[{z}{j}], {a}, {b}, {c} bitop3:0x96"]


def round_body(blocks, last, tables=4):
    L = []
    per = [lookups(z, 16 * i, tables) for i, z in enumerate(blocks)]
    reads = [dst for lk in per for dst, _, _, _ in lk]
    cols = [(z, 16 * i, j) for i, z in enumerate(blocks) for j in range(4)]
    # perms of block 0, its first reads, then the perms of each later block
    # interleaved with the remaining reads (one per lgkmcnt(14) wait)
    pending_perms = []
    for i, lk in enumerate(per):
        pending_perms.append([f"v_perm_b32 {dst}, {src}, %[b{t}], %[s{k}]" for dst, src, t, k in lk])
    L += pending_perms[0]
    nread = 0
    for i in range(min(MAX_LGKM, 16)):
        L.append(f"ds_read_b32 {reads[nread]}, {reads[nread]}")
        nread += 1
    for blk in range(1, len(blocks)):
        L += pending_perms[blk]
        # reads of this block become issuable now
    done, nxt = -1, 0
    while nread < len(reads):
        if nread >= MAX_LGKM:
            L.append(f"s_waitcnt lgkmcnt({MAX_LGKM - 1})")
            done = nread - MAX_LGKM
        L.append(f"ds_read_b32 {reads[nread]}, {reads[nread]}")
        nread += 1
        while nxt < len(cols) and 4 * nxt + 3 <= done:
            L.extend(consume(*cols[nxt], last, tables))
            nxt += 1
    L.append("s_waitcnt lgkmcnt(0)")
    while nxt < len(cols):
        L.extend(consume(*cols[nxt], last, tables))
        nxt += 1
    return L


def round_body_lean(blocks, last, tables=4, R=16):
    """round_body with R lookup registers instead of 16 per block: lookup i
    (block-major, column-major) lives in register i mod R, so the perms of a
    later lookup wait until the column that used its register has been
    folded.  A column is folded only once every perm of its block has read
    the block's state.  Keeps up to 15 reads in flight where registers allow."""
    assert R >= 16, "a block's 16 perms must all read its state before any of its folds"
    per = [lookups(z, 16 * i, tables) for i, z in enumerate(blocks)]
    lk = [x for p in per for x in p]
    n = len(lk)
    ncols = n // 4
    reg = lambda i: f"%[t{i % R}]"  # noqa: E731
    L = []
    st = {"issued": 0, "landed": -1, "folded": 0, "permed": 0}

    def fold_ready():
        while (st["folded"] < ncols and 4 * st["folded"] + 3 <= st["landed"]
               and st["permed"] >= 16 * (st["folded"] // 4 + 1)):
            c = st["folded"]
            blk, j = divmod(c, 4)
            z = blocks[blk]
            a, b, cc, d = (reg(4 * c + t) for t in range(4))
            if last:
                if tables == 4:
                    L.extend([f"v_perm_b32 {a}, {b}, {a}, %[s4]", f"v_perm_b32 {cc}, {d}, {cc}, %[s5]",
                              f"v_bitop3_b32 %[{z}{j}], {a}, {cc}, %[k{j}] bitop3:0x96"])
                else:
                    L.extend([f"v_perm_b32 {a}, {b}, {a}, %[s4]", f"v_perm_b32 {cc}, {d}, {cc}, %[s6]",
                              f"v_bitop3_b32 %[{z}{j}], {a}, {cc}, %[k{j}] bitop3:0x96"])
            elif tables == 4:
                L.extend([f"v_bitop3_b32 {a}, {a}, {b}, {cc} bitop3:0x96",
                          f"v_bitop3_b32 %[{z}{j}], {a}, {d}, %[k{j}] bitop3:0x96"])
            else:
                L.extend([f"v_bitop3_b32 {cc}, {cc}, {d}, %[r{j}] bitop3:0x96",
                          f"v_alignbit_b32 {cc}, {cc}, {cc}, 16",
                          f"v_bitop3_b32 %[{z}{j}], {a}, {b}, {cc} bitop3:0x96"])
            st["folded"] += 1

    def wait_until(idx):
        cnt = st["issued"] - 1 - idx
        L.append(f"s_waitcnt lgkmcnt({min(cnt, MAX_LGKM)})")
        st["landed"] = max(st["landed"], idx)
        fold_ready()

    while st["issued"] < n:
        while st["permed"] < n and (st["permed"] < R or (st["permed"] - R) // 4 < st["folded"]):
            i = st["permed"]
            _, src, t, k = lk[i]
            L.append(f"v_perm_b32 {reg(i)}, {src}, %[b{t}], %[s{k}]")
            st["permed"] += 1
        fold_ready()
        while st["issued"] < st["permed"] and st["issued"] - (st["landed"] + 1) < MAX_LGKM:
            L.append(f"ds_read_b32 {reg(st['issued'])}, {reg(st['issued'])}")
            st["issued"] += 1
        if st["issued"] < n:
            if st["issued"] - (st["landed"] + 1) >= MAX_LGKM:
                wait_until(st["issued"] - MAX_LGKM)
            else:  # a register must free: the column that held it
                wait_until(4 * ((st["permed"] - R) // 4) + 3)
    L.append("s_waitcnt lgkmcnt(0)")
    st["landed"] = n - 1
    fold_ready()
    assert st["folded"] == ncols
    return L


LEAN_R = 0  # > 0: emit rounds with LEAN_R lookup registers (round_body_lean)


def body_for(blocks, last, tables):
    return round_body_lean(blocks, last, tables, LEAN_R) if LEAN_R else round_body(blocks, last, tables)


def nregs(nb):
    return LEAN_R if LEAN_R else 16 * nb


SEL4 = ["0x0c020400u", "0x0c020500u", "0x0c020600u", "0x0c020700u"]
SEL2 = ["0x0c0c0400u", "0x0c0c0500u", "0x0c0c0600u", "0x0c0c0700u"]


def emit(name, blocks, last, tables=4, kv=False):
    """A __device__ function running one (middle or last) round on the blocks.
    kv: the round key words are per-lane values (VGPRs: a wave mixing key
    sets) instead of wave-uniform SGPRs."""
    body = body_for(blocks, last, tables)
    nb = len(blocks)
    args = ", ".join(f"uint32_t {z}[4]" for z in blocks)
    s = [f"__device__ __forceinline__ void {name}({args}, const uint32_t bs[4],",
         "                                       const uint32_t *__restrict__ rkr) {",
         f"    uint32_t t[{nregs(nb)}];"]
    if tables == 2 and not last:
        s.append("    uint32_t r16[4];")
        s.append("#pragma unroll")
        s.append("    for (int j = 0; j < 4; j++) r16[j] = __builtin_amdgcn_alignbit(rkr[j], rkr[j], 16);")
    s.append("    asm volatile(")
    for ln in body:
        s.append(f'        "{ln}\\n"')
    outs = [f'[{z}{i}] "+v"({z}[{i}])' for z in blocks for i in range(4)]
    outs += [f'[t{i}] "=&v"(t[{i}])' for i in range(nregs(nb))]
    ins = [f'[b{i}] "v"(bs[{i}])' for i in range(4)]
    sels = SEL4 if tables == 4 else SEL2
    ins += [f'[s{i}] "s"({sels[i]})' for i in range(4)]
    if last:
        ins += ['[s4] "s"(0x0c0c0601u)', '[s5] "s"(0x04000c0cu)']
        if tables == 2:
            ins += ['[s6] "s"(0x06010c0cu)']
    if tables == 2 and not last:
        ins += [f'[r{i}] "s"(r16[{i}])' for i in range(4)]
    ins += [f'[k{i}] "{"v" if kv else "s"}"(rkr[{i}])' for i in range(4)]
    s.append("        : " + ",\n          ".join(outs))
    s.append("        : " + ",\n          ".join(ins))
    s.append('        : "memory");')
    s.append("}")
    return "\n".join(s)


# ---------------------------------------------------------------- SHA-1 inside
SHA_K = [0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xCA62C1D6]


def sha_rounds(t0, n=4, multi_k=False):
    """gfx950 instructions of SHA-1 rounds t0 .. t0+n-1 on the role registers
    %[ha]..%[he] (a..e on entry) and the 16-word schedule %[w0..15]; the
    working variable that becomes the new `a` is written in place of `e`,
    rotl(b, 30) in place of `b`, so after n rounds role r sits in operand
    (r + n) mod 5 (the caller rotates its array)."""
    regs = ["%[ha]", "%[hb]", "%[hc]", "%[hd]", "%[he]"]
    L = []
    for t in range(t0, t0 + n):
        a, b, c, d, e = regs
        w0 = f"%[w{t & 15}]"
        if t >= 16:
            w3, w8, w14 = (f"%[w{(t - k) & 15}]" for k in (3, 8, 14))
            L.append(f"v_bitop3_b32 %[sx], {w3}, {w8}, {w14} bitop3:0x96")
            L.append(f"v_xor_b32 %[sx], %[sx], {w0}")
            L.append(f"v_alignbit_b32 {w0}, %[sx], %[sx], 31")
        op = 0xCA if t < 20 else 0x96 if t < 40 else 0xE8 if t < 60 else 0x96
        L.append(f"v_bitop3_b32 %[sf], {b}, {c}, {d} bitop3:{op:#x}")
        L.append(f"v_alignbit_b32 %[sr], {a}, {a}, 27")
        L.append(f"v_add3_u32 {e}, {e}, %[sf], %[sr]")
        sk = f"%[sk{t // 20}]" if multi_k else "%[sk]"
        L.append(f"v_add3_u32 {e}, {e}, {sk}, {w0}")
        L.append(f"v_alignbit_b32 {b}, {b}, {b}, 2")
        regs = [e, a, b, c, d]
    return L


def merge_sha(aes, sha):
    """Spread the SHA-1 instructions over the LDS wait points of an AES round
    (before each s_waitcnt), so the wave computes the hash while its table
    lookups are in flight."""
    waits = [i for i, ln in enumerate(aes) if ln.startswith("s_waitcnt")]
    slots = len(waits)
    out, k = [], 0
    for i, ln in enumerate(aes):
        if i in waits:
            w = waits.index(i)
            take = (len(sha) * (w + 1)) // slots - k
            out += sha[k:k + take]
            k += take
        out.append(ln)
    out += sha[k:]
    return out


def emit_sha(name, blocks, last, t0, tables=4, kv=False):
    """One AES round on the block pair with SHA-1 rounds t0..t0+3 interleaved;
    v[5]/w[16] are the hash's working variables and schedule.  kv: per-lane
    round key words (see emit)."""
    body = merge_sha(body_for(blocks, last, tables), sha_rounds(t0))
    nb = len(blocks)
    args = ", ".join(f"uint32_t {z}[4]" for z in blocks)
    s = [f"template <> __device__ __forceinline__ void {name}<{t0}>({args}, const uint32_t bs[4],",
         "        const uint32_t *__restrict__ rkr, uint32_t v[5], uint32_t w[16]) {",
         f"    uint32_t t[{nregs(nb)}], sf, sr, sx;"]
    s.append("    asm volatile(")
    for ln in body:
        s.append(f'        "{ln}\\n"')
    outs = [f'[{z}{i}] "+v"({z}[{i}])' for z in blocks for i in range(4)]
    outs += [f'[t{i}] "=&v"(t[{i}])' for i in range(nregs(nb))]
    outs += [f'[h{r}] "+v"(v[{i}])' for i, r in enumerate("abcde")]
    outs += [f'[w{i}] "+v"(w[{i}])' for i in range(16)]
    outs += ['[sf] "=&v"(sf)', '[sr] "=&v"(sr)', '[sx] "=&v"(sx)']
    ins = [f'[b{i}] "v"(bs[{i}])' for i in range(4)]
    sels = SEL4 if tables == 4 else SEL2
    ins += [f'[s{i}] "s"({sels[i]})' for i in range(4)]
    if last:
        ins += ['[s4] "s"(0x0c0c0601u)', '[s5] "s"(0x04000c0cu)']
    ins += [f'[k{i}] "{"v" if kv else "s"}"(rkr[{i}])' for i in range(4)]
    ins += [f'[sk] "s"({SHA_K[t0 // 20]:#010x}u)']
    s.append("        : " + ",\n          ".join(outs))
    s.append("        : " + ",\n          ".join(ins))
    s.append('        : "memory");')
    # roles after 4 rounds: a in v[1], b in v[2], c in v[3], d in v[4], e in v[0]
    s.append("    const uint32_t e_ = v[0];")
    s.append("    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4]; v[4] = e_;")
    s.append("}")
    return "\n".join(s)


# ------------------------------------------- skewed multi-round pipeline + SHA
def pipe_body(blocks, n_mid, sha, last=True):
    """n_mid middle rounds (+ the last round if `last`) on the blocks, with no
    drain between rounds: lookup groups are issued in the order
    (round r, block 0), (round r, block 1), (round r+1, block 0), ... and a
    group's 16 addresses are computed as soon as the same block's previous
    group has landed and been folded -- while the other block's group is still
    in flight -- so each wave keeps up to 15 LDS reads outstanding through all
    rounds.  `sha` (a list of SHA-1 instructions) is spread over the wait
    points.  Round keys: %[k<r>_<j>] for round index r = 0 .. n_rounds-1."""
    nb = len(blocks)
    n_rounds = n_mid + (1 if last else 0)
    groups = [(r, i) for r in range(n_rounds) for i in range(nb)]
    L = []
    issued, landed = 0, -1        # reads issued; highest read index known landed
    consumed = [0] * len(groups)  # columns folded per group
    n_waits = 0
    # reads per group index g: 16g .. 16g+15
    def fold_available():
        out = []
        for g in range(len(groups)):
            r, i = groups[g]
            while consumed[g] < 4 and 16 * g + 4 * consumed[g] + 3 <= landed:
                j = consumed[g]
                z = blocks[i]
                a, b, c, d = (f"%[t{16 * i + 4 * j + t}]" for t in range(4))
                k = f"%[k{r}_{j}]"
                if last and r == n_rounds - 1:
                    out += [f"v_perm_b32 {a}, {b}, {a}, %[s4]",
                            f"v_perm_b32 {c}, {d}, {c}, %[s5]",
                            f"v_bitop3_b32 %[{z}{j}], {a}, {c}, {k} bitop3:0x96"]
                else:
                    out += [f"v_bitop3_b32 {a}, {a}, {b}, {c} bitop3:0x96",
                            f"v_bitop3_b32 %[{z}{j}], {a}, {d}, {k} bitop3:0x96"]
                consumed[g] += 1
        return out
    # wait points: count them first to spread the SHA stream evenly
    total_reads = 16 * len(groups)
    est_waits = total_reads - 15 + len(groups)
    sha_pos = 0
    def sha_take(w):
        nonlocal sha_pos
        want = min(len(sha), (len(sha) * (w + 1)) // est_waits)
        out = sha[sha_pos:want]
        sha_pos = max(sha_pos, want)
        return out
    def wait_for(idx):
        """wait until read index idx has landed"""
        nonlocal landed, n_waits
        if idx <= landed:
            return
        cnt = issued - 1 - idx  # reads after idx that may stay in flight
        L.extend(sha_take(n_waits))
        n_waits += 1
        L.append(f"s_waitcnt lgkmcnt({min(cnt, MAX_LGKM)})")
        landed = idx
        L.extend(fold_available())
    for g, (r, i) in enumerate(groups):
        if g >= nb:  # the same block's previous group must be folded
            wait_for(16 * (g - nb) + 15)
            assert consumed[g - nb] == 4
        z = blocks[i]
        for j in range(4):
            for t in range(4):
                L.append(f"v_perm_b32 %[t{16 * i + 4 * j + t}], %[{z}{(j + t) & 3}], %[b{t}], %[s{t}]")
        for q in range(16):
            if issued - (landed + 1) >= MAX_LGKM:
                wait_for(issued - MAX_LGKM)
            L.append(f"ds_read_b32 %[t{16 * i + q}], %[t{16 * i + q}]")
            issued += 1
    wait_for(issued - 1)
    L.extend(sha[sha_pos:])
    assert all(c == 4 for c in consumed)
    return L


def emit_pipe_sha(name, blocks, n_mid, t0, n_sha, last=True):
    """Rounds (n_mid middle + last) of the block pair as one skewed pipeline
    with SHA-1 rounds t0 .. t0+n_sha-1 spread over its waits.  Round keys come
    from rkr[4 * r + j]."""
    sha = sha_rounds(t0, n_sha, multi_k=True)
    body = pipe_body(blocks, n_mid, sha, last)
    nb = len(blocks)
    n_rounds = n_mid + (1 if last else 0)
    args = ", ".join(f"uint32_t {z}[4]" for z in blocks)
    s = [f"template <> __device__ __forceinline__ void {name}<{t0}>({args}, const uint32_t bs[4],",
         "        const uint32_t *__restrict__ rkr, uint32_t v[5], uint32_t w[16]) {",
         f"    uint32_t t[{16 * nb}], sf, sr, sx;"]
    s.append("    asm volatile(")
    for ln in body:
        s.append(f'        "{ln}\\n"')
    outs = [f'[{z}{i}] "+v"({z}[{i}])' for z in blocks for i in range(4)]
    outs += [f'[t{i}] "=&v"(t[{i}])' for i in range(16 * nb)]
    outs += [f'[h{r}] "+v"(v[{i}])' for i, r in enumerate("abcde")]
    outs += [f'[w{i}] "+v"(w[{i}])' for i in range(16)]
    outs += ['[sf] "=&v"(sf)', '[sr] "=&v"(sr)', '[sx] "=&v"(sx)']
    ins = [f'[b{i}] "v"(bs[{i}])' for i in range(4)]
    ins += [f'[s{i}] "s"({SEL4[i]})' for i in range(4)]
    if last:
        ins += ['[s4] "s"(0x0c0c0601u)', '[s5] "s"(0x04000c0cu)']
    ins += [f'[k{r}_{j}] "s"(rkr[{4 * r + j}])' for r in range(n_rounds) for j in range(4)]
    ks = sorted({(t0 + q) // 20 for q in range(n_sha)})
    ins += [f'[sk{k}] "s"({SHA_K[k]:#010x}u)' for k in ks]
    s.append("        : " + ",\n          ".join(outs))
    s.append("        : " + ",\n          ".join(ins))
    s.append('        : "memory");')
    # after n_sha rounds register i holds role (i + n_sha) mod 5
    s.append(f"    const uint32_t o_[5] = {{v[0], v[1], v[2], v[3], v[4]}};")
    s.append(f"#pragma unroll")
    s.append(f"    for (int i = 0; i < 5; i++) v[(i + {n_sha}) % 5] = o_[i];")
    s.append("}")
    return "\n".join(s)
