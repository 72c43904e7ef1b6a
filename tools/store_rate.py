"""HBM write rate of plain streaming stores on the GPU box (torch fill of a large fp64 buffer), as the ceiling the
residual stores of the interpolation kernels are compared with (their 256-byte row segments reach ~5.7 TB/s).

    python tools/store_rate.py [--gb 6.5]
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=6.5)
    args = ap.parse_args()
    n = int(args.gb * 1e9 / 8)
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    for _ in range(3):
        x.fill_(1.0)
    torch.cuda.synchronize()
    reps = 10
    t0 = time.perf_counter()
    for i in range(reps):
        x.fill_(float(i))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    y = torch.empty_like(x)
    y.copy_(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        y.copy_(x)
    torch.cuda.synchronize()
    dc = (time.perf_counter() - t0) / reps
    print(json.dumps({"bytes": 8 * n, "fill_ms": dt * 1e3, "fill_TBps": 8 * n / dt / 1e12,
                      "copy_ms": dc * 1e3, "copy_TBps_read_plus_write": 16 * n / dc / 1e12}))


if __name__ == "__main__":
    main()
