#!/usr/bin/env python3
"""Diagnostic only: a k_small variant that times its phases for 1-packet bundles.

    python3 tools/small_phases_variant.py build
        -> libjitsi_amd/variants/ts/libsrtp_mi355x.so (the normal build's other
           objects; the kernels from a patched copy of srtp_kernels.hip under
           libjitsi_amd/csrc/build_ts/, never the tracked source)
    LD_LIBRARY_PATH=libjitsi_amd/variants/ts ./tools/sync_bench 1 one 0 1 rt > LOG
    python3 tools/small_phases_variant.py summary LOG

Thread 0 of workgroup 0 reads the 100-MHz wall clock (wall_clock64) after each
phase barrier of k_small and, for every 41st 1-packet bundle, prints the phase
durations with device printf (profiles/r06/small/lone_k_small_phases.txt).
"""
import os
import re
import statistics
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CSRC = os.path.join(ROOT, "libjitsi_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def patched_source():
    src = open(os.path.join(CSRC, "srtp_kernels.hip")).read()
    i0 = src.index("template <bool REV>\n__global__ __launch_bounds__(kSmallBlock) void k_small(BundleArgs a) {")
    i1 = src.index("hipError_t launch_small(")
    body = src[i0:i1]

    def stamp(k):
        return f"if (blockIdx.x == 0 && threadIdx.x == 0) ts[{k}] = wall_clock64();\n"

    # (anchor, stamp index): the stamp goes right after the anchor
    anchors = [
        ("void k_small(BundleArgs a) {\n    __shared__ uint32_t s[kSmallOffR + kSmallRWords];\n", None),
        ("        small_pull(a);\n        __syncthreads();\n", 1),
        ("    if (!REV || !wave_mac) fill_te4(s); // ends with a barrier\n", 2),
        ("            r[t] = key;\n        }\n        __syncthreads();\n", 3),
        ("            if (REV && key <= a.ctx_mask) a.spos[t] = rank;\n        }\n        __syncthreads();\n", 4),
        ("                mac_check<false>(a, t, nullptr);\n            }\n            __syncthreads();\n", 5),
        ("                walk_tile<REV, false, 1>(a, sh, 0u, 1u);\n            }\n        }\n        __syncthreads();\n", 6),
        ("    if (REV && wave_mac) fill_te4(s); // ends with a barrier\n", 7),
        ("        if (t == kSmallPerWg - 1u) pre[kSmallPerWg] = x;\n    }\n    __syncthreads();\n", 8),
        ("    __syncthreads();\n    // 7. protect", 9),
        ("    flush_status_counts(a, s_cnt);\n", 10),
        ("            mac_seal<false>(a, p, nullptr);\n        }\n    }\n", 11),
        ("        small_push(a, g, G, m);\n    }\n", 12),
    ]
    for anchor, k in anchors:
        assert body.count(anchor) == 1, anchor
        if k is None:
            add = "    uint64_t ts[14] = {};\n    " + stamp(0)
        elif k == 9:
            body = body.replace(anchor, "    __syncthreads();\n    " + stamp(9) + "    // 7. protect")
            continue
        else:
            add = "    " + stamp(k)
        body = body.replace(anchor, anchor + add)
    report = r'''    if (blockIdx.x == 0 && threadIdx.x == 0 && a.n == 1 && (atomicAdd(&g_small_ts_cnt, 1u) % 41u) == 40u) {
        int d[13];
        uint64_t prev = ts[0];
        for (int k = 1; k < 13; k++) { d[k] = ts[k] ? (int)((ts[k] - prev) * 10) : -1; if (ts[k]) prev = ts[k]; }
        printf("KSMALL rev %d n %u ns: pull %d fill %d parse %d sort %d tagchk %d walk %d fill2 %d jobs %d ks %d status %d mac %d push %d total %d\n",
               (int)REV, a.n, d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9], d[10], d[11], d[12], (int)((ts[12] - ts[0]) * 10));
    }
'''
    assert body.endswith("}\n\n")
    body = body[:-3] + report + "}\n\n"
    return src[:i0] + "__device__ unsigned g_small_ts_cnt;\n" + body + src[i1:]


def build():
    bdir = os.path.join(CSRC, "build_ts")
    os.makedirs(bdir, exist_ok=True)
    with open(os.path.join(bdir, "srtp_kernels_ts.hip"), "w") as f:
        f.write(patched_source())
    subprocess.check_call(["make", "-s", "-j8"], cwd=CSRC)
    subprocess.check_call([HIPCC, "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result", "--offload-arch=gfx950",
                           "-mllvm", "-disable-promote-alloca-to-lds", "-I..", "-I../../../include", "-c",
                           "srtp_kernels_ts.hip", "-o", "srtp_kernels.o"], cwd=bdir)
    out = os.path.join(ROOT, "libjitsi_amd", "variants", "ts")
    os.makedirs(out, exist_ok=True)
    objs = ["build_ts/srtp_kernels.o"] + [f"build/{o}.o" for o in
                                          ("engine", "host_crypto", "dispatch", "dtls_keys", "aggregator", "rawpacket")]
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                           os.path.join(out, "libsrtp_mi355x.so")] + objs, cwd=CSRC)
    print("built libjitsi_amd/variants/ts/libsrtp_mi355x.so")


def summary(path):
    rows = {0: [], 1: []}
    for line in open(path):
        if not line.startswith("KSMALL"):
            continue
        rev = int(line.split()[2])
        rows[rev].append({k: int(v) for k, v in re.findall(r"(\w+) (-?\d+)", line.split("ns:")[1])})
    for rev, name in ((0, "protect"), (1, "unprotect")):
        r = rows[rev]
        if not r:
            continue
        cols = [k for k in r[0] if k != "total"] + ["total"]
        med = {k: statistics.median(x[k] for x in r) / 1000 for k in cols}
        print(f"{name} ({len(r)} bundles), median us: " +
              " ".join(f"{k} {med[k]:.2f}" for k in cols if med[k] > 0.05 or k == "total"))


if __name__ == "__main__":
    if sys.argv[1:2] == ["build"]:
        build()
    elif sys.argv[1:2] == ["summary"] and len(sys.argv) == 3:
        summary(sys.argv[2])
    else:
        sys.exit(__doc__)
