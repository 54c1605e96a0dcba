"""Latency of one tiny kernel + sync after the GPU sat idle for a while (is the drop-in's first
engine call after an idle gap paying the GPU's wake-up?).  Prints one JSON line."""
import json
import time

import torch


def main():
    x = torch.ones(16, device="cuda")
    for _ in range(20):
        x.add_(1)
    torch.cuda.synchronize()
    out = {}
    for gap in (0.0, 0.001, 0.01, 0.05, 0.1, 0.3, 1.0, 3.0):
        ts = []
        for _ in range(3):
            time.sleep(gap)
            t0 = time.perf_counter()
            x.add_(1)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        out[f"idle_{gap}s_ms"] = [round(t, 3) for t in ts]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
