"""PCIe copy bandwidth on the GPU box: pinned host <-> HBM, one direction or
both at once, one stream or the copy split over several streams.  Sizes the
e2e leg of bench.py against what the link itself moves."""
import json
import time

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    nb = 320 << 20
    h = [torch.empty(nb, dtype=torch.uint8).pin_memory() for _ in range(2)]
    d = [torch.empty(nb, dtype=torch.uint8, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(8)]
    out = {}

    def h2d(k=1):
        c = nb // k
        for i in range(k):
            with torch.cuda.stream(streams[i]):
                d[0][i * c:(i + 1) * c].copy_(h[0][i * c:(i + 1) * c], non_blocking=True)

    def d2h(k=1):
        c = nb // k
        for i in range(k):
            with torch.cuda.stream(streams[4 + i]):
                h[1][i * c:(i + 1) * c].copy_(d[1][i * c:(i + 1) * c], non_blocking=True)

    for k in (1, 2, 4):
        out[f"h2d_gbps_{k}streams"] = round(nb / timed(lambda: h2d(k)) / 1e9, 1)
        out[f"d2h_gbps_{k}streams"] = round(nb / timed(lambda: d2h(k)) / 1e9, 1)
        out[f"both_gbps_total_{k}streams"] = round(2 * nb / timed(lambda: (h2d(k), d2h(k))) / 1e9, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
