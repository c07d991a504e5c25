"""Practical HBM ceilings on this box, for reading the decode's roofline
fraction: device-to-device copy (1:1 read:write), fill (write only), a
read-only reduction, and the decode's own 1:2 read:write ratio as a copy
of 330 MB into 640 MB (each source byte written twice)."""
import json
import time

import torch


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    dev = torch.device("cuda", 0)
    n = 1 << 30
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    a.fill_(1)
    out = {}
    t = timeit(lambda: b.copy_(a))
    out["copy_1GiB_GBs"] = round(2 * n / t / 1e9, 1)
    t = timeit(lambda: b.fill_(3))
    out["fill_1GiB_GBs"] = round(n / t / 1e9, 1)
    af = a.view(torch.float32)
    t = timeit(lambda: af.sum())
    out["read_sum_1GiB_GBs"] = round(n / t / 1e9, 1)
    src = torch.empty(330_000_000 // 4, dtype=torch.int32, device=dev)
    dst = torch.empty(2, 330_000_000 // 4, dtype=torch.int32, device=dev)
    t = timeit(lambda: dst.copy_(src.unsqueeze(0).expand(2, -1)))
    out["expand_330MB_to_660MB_GBs"] = round(990e6 / t / 1e9, 1)
    out["device"] = torch.cuda.get_device_name(0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
