"""CPU baseline thread sweep: the fp64 C/OpenMP oracle on whole 4K RGB
images (r2h -> HexConv2d -> h2r, the bench's cpu_baseline workload) at 8..256 threads,
ignoring the cgroup quota, with the quota and affinity printed beside it.

usage: python tools/cpu_sweep.py [images_per_count] > profiles/r03/cpu_sweep.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import numpy as np  # noqa: E402

import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    n_img = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    avail, quota, cap = bench.cpu_quota()
    rng = np.random.default_rng(2)
    H, W = 2160, 3840
    x = rng.random((1, 3, H, W))
    k = (rng.random((3, 3, 7)) - 0.5) * 0.5
    b = rng.random(3) - 0.5
    out = {"cpu_model": bench.cpu_model(), "nproc": os.cpu_count(), "affinity": avail,
           "cgroup_cpu_quota": quota, "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
           "images_per_count": n_img, "mpix_s": {}}
    for c in (8, 16, 32, 64, 128, 256):
        if c > avail:
            break
        O.set_num_threads(c)
        bench.cpu_image_rate(O, x, k, b, H, W, 0.0, 1)   # warm
        rate, n, dt = bench.cpu_image_rate(O, x, k, b, H, W, 0.0, n_img)
        out["mpix_s"][str(c)] = round(rate, 2)
        print(f"threads {c:4d}: {rate:8.2f} Mpix/s ({n} images, {dt:.2f} s)", file=sys.stderr,
              flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
