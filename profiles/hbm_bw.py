"""HBM bandwidth of plain streaming kernels on this box (torch's own fill / copy / sum), as the
achievable write-only, read+write and read-only rates the trendline config's stores compare with.
Usage: python profiles/hbm_bw.py [GiB]"""
import json
import sys

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    n = int(gib * 2**30) // 8
    x = torch.empty(n, dtype=torch.float64, device='cuda')
    y = torch.empty(n, dtype=torch.float64, device='cuda')
    x.fill_(1.0)
    nb = n * 8
    res = {'bytes': nb,
           'write_fill_tbs': nb / timed(lambda: x.fill_(2.0)) / 1e12,
           'copy_rw_tbs': 2 * nb / timed(lambda: y.copy_(x)) / 1e12,
           'read_sum_tbs': nb / timed(lambda: x.sum()) / 1e12,
           'device': torch.cuda.get_device_name(0)}
    print(json.dumps(res))


if __name__ == '__main__':
    main()
