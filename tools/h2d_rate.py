"""Host <-> device copy rates of this box (what bounds C2 from host memory).

Page-locked host buffers of the sizes the C2 / C4 staging copies move (1.28 MB of u8 rows, 5.12 MB
of float rows per frame, 12.8 MB of C4's u8 rows), one copy at a time on one stream, timed with HIP
events over 50 copies; plus the host memcpy rate into page-locked memory (the staging copy).

    python tools/h2d_rate.py
"""
import json
import time

import numpy as np
import torch


def main():
    out = {"device": torch.cuda.get_device_name(0)}
    s = torch.cuda.Stream()
    for mb in (1.28, 5.12, 10.24, 12.8):
        n = int(mb * 1e6)
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        d = torch.empty(n, dtype=torch.uint8, device="cuda")
        src = np.random.default_rng(0).integers(0, 255, n, dtype=np.uint8)
        with torch.cuda.stream(s):
            for _ in range(5):
                d.copy_(h, non_blocking=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(50):
                d.copy_(h, non_blocking=True)
            e1.record(s)
            e1.synchronize()
            h2d = e0.elapsed_time(e1) / 50
            e0.record(s)
            for _ in range(50):
                h.copy_(d, non_blocking=True)
            e1.record(s)
            e1.synchronize()
            d2h = e0.elapsed_time(e1) / 50
        hv = h.numpy()
        t = time.perf_counter()
        for _ in range(50):
            np.copyto(hv, src)
        mc = (time.perf_counter() - t) / 50 * 1e3
        out[f"{mb}MB"] = {"h2d_ms": h2d, "h2d_GBps": n / h2d / 1e6, "d2h_ms": d2h, "d2h_GBps": n / d2h / 1e6,
                          "host_memcpy_to_pinned_ms": mc, "host_memcpy_GBps": n / mc / 1e6}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
