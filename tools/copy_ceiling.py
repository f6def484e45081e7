"""Read + write HBM ceiling of the rolling-mean S = 1 line's shape: a device
copy (torch copy_, i.e. the runtime's D2D copy kernel) and a fill of the same
5,000 x 600,000 float32 array (12 GB in, 12 GB out), to set the S = 1 line's
0.66-0.71 of 8 TB/s (8 B per sample, read + write) against what a plain
stream of that traffic reaches on the box.

    python tools/copy_ceiling.py
"""
import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n_ch, n = 5000, 600_000
    x = torch.empty((n_ch, n), dtype=torch.float32, device="cuda")
    x.uniform_()
    y = torch.empty_like(x)
    nb = x.numel() * 4
    ms = timed(lambda: y.copy_(x))
    print(f"copy  {n_ch} x {n} f32: {ms:.3f} ms  {2 * nb / ms / 1e6:.0f} GB/s  frac {2 * nb / ms / 1e6 / 8000:.3f}"
          " (read + write)", flush=True)
    ms = timed(lambda: y.fill_(1.0))
    print(f"fill  {n_ch} x {n} f32: {ms:.3f} ms  {nb / ms / 1e6:.0f} GB/s  frac {nb / ms / 1e6 / 8000:.3f} (write)",
          flush=True)
    ms = timed(lambda: torch.sum(x, dim=1))
    print(f"sum   {n_ch} x {n} f32: {ms:.3f} ms  {nb / ms / 1e6:.0f} GB/s  frac {nb / ms / 1e6 / 8000:.3f} (read)",
          flush=True)


if __name__ == "__main__":
    main()
