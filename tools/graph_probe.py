"""Launch-latency probe (design tool, GPU): back-to-back dependent tiny
kernels, eager vs replayed from a HIP graph (torch.cuda.CUDAGraph on ROCm),
to size what graph capture would buy the small-mesh eager path.

    python tools/graph_probe.py [N]
"""
import json
import sys
import time

import torch


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    dev = torch.device("cuda", 0)
    x = torch.zeros(4096, device=dev)
    s = torch.cuda.Stream(dev)
    out = {"kernels": n}
    with torch.cuda.stream(s):
        for _ in range(50):
            x.add_(1.0)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            x.add_(1.0)
        torch.cuda.synchronize(dev)
        out["eager_us_per_kernel"] = round((time.perf_counter() - t0) * 1e6 / n, 2)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                x.add_(1.0)
        g.replay()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize(dev)
        out["graph_us_per_kernel"] = round((time.perf_counter() - t0) * 1e6 / (5 * n), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
