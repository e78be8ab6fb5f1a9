#!/usr/bin/env python3
"""Benchmark of the hot path on BASELINE.json's headline workload.

Workload (BASELINE.json configs[2], "config 3"): per GPU a batch of 128 4K RGB
rasters (3 x 2160 x 3840, bf16, synthetic U[0,1), seed 2+rank), one step =
rect->hex bilinear resample (2160x3840) -> HexConv2d(3, 3, even_odd_offset=0,
radius 2, padding=1, bias; weights drawn with torch.manual_seed(3) and the
reference initialiser) -> hex->rect linear resample (2160x3840), all on the
gfx950 kernels of libhygrid_hip.so, with bf16 tensors between stages.

Multi-GPU: one process per GPU; every rank owns its own 128 images (weak scaling, no
data-path collective).  `--gpus N` with N > 1 and no WORLD_SIZE in the environment starts
`torch.distributed.run --nproc-per-node N` as a CHILD process (nothing here has touched the
GPU yet; never an exec) and exits with its return code; under a launcher, WORLD_SIZE must
equal --gpus or the bench exits with status 2.  value = all ranks' input pixels / the
max-over-ranks wall time of K steps.  Every timed step, at every N including N = 1 (a
world-1 process group), ends with per-image, per-channel sums of a row sample of its output
(every 256th row) all-gathered over RCCL (the collective stays inside the timed
loop; a few KB per rank), so the per-step work is the same at every N.  After the timed
region, full per-image checksums are all-gathered, and (N>1) the full-output gather to
rank 0 is timed and reported on its own (`gather`), never folded into `value`.
`--dry-run`: the same launch, process groups (gloo), barriers, per-step collective,
max-over-ranks timing and JSON line on the CPU with a stand-in step and no HIP kernel
(tests/test_bench_launch.py); its value is not a measurement.

Extra JSON fields: `kernels` (per-stage HIP-event times and algorithmic GB/s),
`roofline` (dominant kernel vs 8 TB/s HBM), `cpu_baseline` (the C/OpenMP oracle
restatement on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")
for _p in (ROOT, PKG_DIR):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# What bounds the headline kernel (rounds 5-6): its cache-resident build
# (every load / store hits one row) runs 1.83-2.02 ms, the real one ~0.6-0.7 ms more; loads
# alone or stores alone add ~0.25 ms each, both together ~0.7 ms; bytes are 1.035x (round 6).
FUSED4_LIMITER = ("the streaming rate of the band walk on top of VALU issue (k_fused4: 136 VGPRs, "
                  "3 waves per SIMD, 2 rect rows of prefetch): HBM traffic is 1.035x the "
                  "algorithmic bytes (round 6), the cache-resident floor 1.83-2.02 ms per 4K b128 "
                  "launch, and the interleaved row-load / row-store stream adds ~0.6 ms that does "
                  "not overlap with the stencil; the same walk with no arithmetic reaches 0.57 of "
                  "8 TB/s, 0.65 with a store wave (profiles/r05/fused4_floor_ab.txt, "
                  "fused4_additivity_ab.txt, profiles/r06/walk9_store_wave.txt)")
PEAK_BPS = HBM_PEAK_GBS * 1e9


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--prewarm-ms", type=float, default=1000.0,
                    help="untimed run of the headline step before its W warmup steps, until this "
                         "much wall time has passed: the MI355X raises its clock over the first "
                         "~40 ms of a cold start (kernel traces in profiles/r02/k), and a "
                         "serving process runs in that steady state")
    ap.add_argument("--batch", type=int, default=128, help="images per GPU")
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--cpu-images", type=int, default=64,
                    help="max images in the CPU-baseline sample (~10 s; 0 disables it)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every CPU this process may run on (sched_getaffinity)")
    ap.add_argument("--no-gather", action="store_true", help="skip the timed output gather")
    ap.add_argument("--unfused", action="store_true",
                    help="time the three operators (r2h, HexConv2d, h2r) instead of the fused kernel")
    ap.add_argument("--no-compare", action="store_true",
                    help="skip the secondary (unfused) measurement in the fused run")
    ap.add_argument("--no-pyramid", action="store_true",
                    help="skip the secondary config-5 line (8K fp16 3-level hex pyramid)")
    ap.add_argument("--no-roundtrip", action="store_true",
                    help="skip the secondary config-2 line (1080p fp32 rect->hex->rect)")
    ap.add_argument("--no-wide-conv", action="store_true",
                    help="skip the secondary wide-channel HexConv2d line (64->64, 1080p)")
    ap.add_argument("--no-lattices", action="store_true",
                    help="skip the reference entry points' own (non-identity) lattices")
    ap.add_argument("--lattice-batch", type=int, default=32, help="4K images per lattice line")
    ap.add_argument("--pyramid-batch", type=int, default=8, help="8K images per GPU (config 5)")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="N > 1 with every rank on cuda:0 and the collectives over gloo (host "
                         "staged): exercises the multi-rank bench path on a one-GPU box; the "
                         "ranks share one GPU, so the value is not a scaling measurement")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: the launcher, process groups (gloo), barriers, per-step "
                         "collective, timing and JSON line with a CPU stand-in step (tests)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-kernel HBM bytes from rocprofv3 PMC passes (optional)")
    return ap.parse_args()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """CPUs this process may actually use: the affinity mask, capped by the cgroup CPU quota
    (cgroup v2 cpu.max "quota period", v1 cfs_quota_us / cfs_period_us).  On the GPU box the
    mask shows the whole machine while the quota is the box's share; OpenMP sized to the mask
    oversubscribes the quota (round 2: 13 Mpix/s on 256 threads vs 70 on 16 in round 1)."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    cap = avail if quota is None else max(1, min(avail, int(quota)))
    return avail, quota, cap


def cpu_image_rate(O, x, kernel, bias, H, W, budget_s, max_images):
    """Whole images, one at a time, until budget_s of CPU work: Mpix/s, images, seconds."""
    n, dt = 0, 0.0
    while n < max_images and (n == 0 or dt < budget_s):
        t0 = time.perf_counter()
        hexim = O.rect_to_hex(x, (H, W), 1)
        c = O.hexconv2d(hexim, kernel, bias, 0, 2, padding=1)
        O.hex_to_rect(c, (H, W), 1)
        dt += time.perf_counter() - t0
        n += 1
    return n * H * W / dt / 1e6, n, dt


def cpu_baseline(args, kernel, bias):
    """Oracle (C/OpenMP fp64 restatement) on a bounded sample of the same workload: whole
    4K images, one at a time.  The thread count is picked by a short sweep (one image per
    count) over counts up to the cgroup CPU quota, then the best count is timed for ~10 s.
    Round 3: the sweep replaces 'every CPU in the affinity mask' (see cpu_quota)."""
    import numpy as np

    from oracle import oracle as O
    avail, quota, cap = cpu_quota()
    rng = np.random.default_rng(2)
    x = rng.random((1, args.channels, args.height, args.width))
    H, W = args.height, args.width
    if args.cpu_threads:
        counts = [args.cpu_threads]
    else:
        counts = sorted({c for c in (1, 4, 8, 16, 32, 64, 128, 256) if c <= cap} | {cap})
        counts = [c for c in counts if c >= min(8, cap)]
    sweep = {}
    for c in counts:
        O.set_num_threads(c)
        cpu_image_rate(O, x, kernel, bias, H, W, 0.0, 1)        # warm (first touch, threads)
        sweep[c] = round(cpu_image_rate(O, x, kernel, bias, H, W, 0.0, 1)[0], 3)
    threads = max(sweep, key=sweep.get)
    O.set_num_threads(threads)
    rate, n, dt = cpu_image_rate(O, x, kernel, bias, H, W, 10.0, args.cpu_images)
    return {"value": round(rate, 3), "unit": "Mpix/s",
            "cores": threads, "kind": "port",
            "sample": f"{n} image(s) of {args.channels}x{H}x{W}, one at a "
                      f"time (fp64 oracle/hg_oracle.c, r2h->HexConv2d->h2r), {dt:.2f} s, on "
                      f"the best of a one-image thread sweep",
            "thread_sweep_mpix_s": {str(k): v for k, v in sweep.items()},
            "cpu_model": cpu_model(), "nproc": os.cpu_count(), "cpus_available": avail,
            "cgroup_cpu_quota": quota,
            "reference_measured": {"value": 1.05, "unit": "Mpix/s",
                                   "what": "the reference's own geometry_np + HexFrames "
                                           "(NumPy, one core), one 4K RGB image, survey "
                                           "container (BASELINE.md section 2)"}}


def touched_rows_bytes(ops, op, h, w, h1, w1, dev, nearest, elem):
    """Bytes of the source rows a resample's lattice references (every referenced row is
    read once, whole: its cache lines are streamed), from the kernel's own integer maps.
    hex -> rect upsampling references every source row: the whole source."""
    if op != "rect_to_hex":
        return h * w * elem
    m = ops.lattice_maps(op, h, w, h1, w1, device=dev)
    i_n, valid = m["i_n"].long(), m["valid"].long()
    if nearest:
        rows = i_n + (m["argmin"].long() >> 1)
        rows = rows[((valid >> m["argmin"].long()) & 1) == 1]
    else:   # taps (i_n, .) valid bits 0/1, (i_n + 1, .) bits 2/3
        rows = torch.cat([i_n[(valid & 3) != 0], (i_n + 1)[(valid & 12) != 0]])
    n = int(torch.unique(rows).numel())
    return n * w * elem


def bench_lattices(ops, measure, gen, dev, world, Bl, C, H, W):
    """The reference's own entry-point lattices, which are not the same-size one the fused
    kernel covers: IMAGE.ConvertToHexagon (Image.py:111-116: rect -> hex at (h//2, w//2),
    'nearest', the image's own dtype, u8 here) and the geometry_np demo's bilinear
    downsample (geometry_np.py:772-776: an ADE image to (256, 341), ratio ~2; bf16 here), on
    4K RGB batches.  Algorithmic bytes = the source rows the lattice references (whole rows)
    + the output; each line carries its own fraction of the 8 TB/s peak."""
    hs, ws = H // 2, W // 2
    xu8 = torch.randint(0, 256, (Bl, C, H, W), generator=gen, device=dev, dtype=torch.uint8)
    xbf = torch.rand((Bl, C, H, W), generator=gen, device=dev, dtype=torch.bfloat16)
    # the inverse lattice of ConvertToHexagon: a (h//2, w//2) hex image back to the (h, w)
    # rect raster (hex_to_rect_resample, geometry_np.py:191-356; 'nearest' is
    # geometry_torch.py:335-347)
    hu8 = xu8[:, :, :hs, :ws].contiguous()
    hbf = xbf[:, :, :hs, :ws].contiguous()
    out = {}
    cases = (("convert_to_hexagon", "rect_to_hex", xu8, 0, 1, (hs, ws),
              "Image.py:111-116: rect->hex (h//2, w//2) nearest, u8"),
             ("r2h_bilinear_2x", "rect_to_hex", xbf, 1, 2, (hs, ws),
              "geometry_np.py:772-776 ratio: rect->hex (h//2, w//2) bilinear, bf16"),
             ("hexresize_2x", "hexresize", xbf, 1, 2, (hs, ws),
              "geometry_np.py:520-681: hexresize hex (h, w) -> hex (h//2, w//2) linear, bf16 "
              "(one pyramid level's resample alone)"),
             ("h2r_linear_2x_up", "hex_to_rect", hbf, 1, 2, (H, W),
              "geometry_np.py:191-356: hex (h//2, w//2) -> rect (h, w) linear, bf16 (inverse of "
              "ConvertToHexagon's lattice)"),
             ("h2r_nearest_2x_up", "hex_to_rect", hu8, 0, 1, (H, W),
              "geometry_torch.py:335-347: hex (h//2, w//2) -> rect (h, w) nearest, u8"))
    for name, op, xin, interp, elem, osz, what in cases:
        def run(record, ev, xin=xin, interp=interp, op=op, osz=osz):
            if record:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record()
            y = getattr(ops, op)(xin, osz, interp=interp)
            if record:
                e[1].record()
                ev.append(e)
            return y
        steps = 10
        _, el, sms = measure(run, steps)
        hi, wi = int(xin.shape[-2]), int(xin.shape[-1])
        rb = touched_rows_bytes(ops, op, hi, wi, osz[0], osz[1], dev, interp == 0, elem)
        alg = Bl * C * (rb + osz[0] * osz[1] * elem)
        out[name] = {"what": what, "batch_per_gpu": Bl, "in_shape": [Bl, C, hi, wi],
                     "out_shape": [Bl, C, osz[0], osz[1]], "ms": round(sms[0], 4),
                     "value": round(world * Bl * osz[0] * osz[1] * steps / el / 1e6, 1),
                     "unit": "Mpix/s (output samples)",
                     "alg_GB": round(alg / 1e9, 4),
                     "src_rows_referenced_frac": round(rb / (hi * wi * elem), 4),
                     "GB_per_s": round(alg / (sms[0] * 1e-3) / 1e9, 1),
                     "frac_of_peak": round(alg / (sms[0] * 1e-3) / PEAK_BPS, 4)}
    del xu8, xbf, hu8, hbf
    return out


def free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv):
    """`--gpus N` (N > 1) outside a launcher: run this script under torch.distributed.run as a
    child process, one rank per GPU on 127.0.0.1, and return its exit status.  Called before
    anything here touches the GPU; the parent only waits (no exec)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on these hosts
    log("bench: launching", n, "ranks:", " ".join(cmd))
    return subprocess.run(cmd, env=env).returncode


class CpuEvent:
    """torch.cuda.Event's record / elapsed_time on the host clock (--dry-run)."""
    def __init__(self, **_):
        self.t = None

    def record(self):
        self.t = time.perf_counter()

    def elapsed_time(self, end):
        return (end.t - self.t) * 1e3


def main():
    args = parse()
    if args.gpus < 1:
        log("bench: --gpus must be >= 1")
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    # stdout carries one line, the JSON result: from here on anything else written to fd 1 (RCCL
    # prints a version banner to stdout when a communicator is created, at N = 1 too) goes to
    # stderr, and the line goes to a duplicate of the original stdout
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: the line would report the wrong "
            f"n_gpus; launch with --nproc-per-node {args.gpus} or drop the launcher")
        sys.exit(2)
    dry = args.dry_run
    rehearse = world > 1 and args.rehearse_gloo
    # every N has a process group (N = 1: world 1 on an in-process store), so the per-step
    # collective runs at N = 1 too and the 1 -> N efficiency compares equal per-step work
    pg_kw = {} if world > 1 else {"store": dist.HashStore(), "rank": 0, "world_size": 1}
    if dry or rehearse:
        local_rank = 0
        dist.init_process_group("gloo", **pg_kw)
    else:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), **pg_kw)
    dev = torch.device("cpu") if dry else torch.device("cuda", local_rank)
    if not dry:
        torch.cuda.set_device(dev)
    cdev = torch.device("cpu") if (rehearse or dry) else dev   # where the collectives' tensors live
    Event = CpuEvent if dry else torch.cuda.Event

    def sync():
        if not dry:
            torch.cuda.synchronize()

    B, C, H, W = args.batch, args.channels, args.height, args.width
    bf16 = torch.bfloat16
    if dry:
        # stand-in step on the host: no HIP kernel runs, the value is not a measurement
        B, H, W = min(B, 4), min(H, 64), min(W, 128)
        gen = torch.Generator().manual_seed(2 + rank)
        x = torch.rand((B, C, H, W), generator=gen, dtype=torch.float32)
        conv = None
        # test hook: rank r starts its pre-warm r x BENCH_DRY_SKEW_MS later, so the ranks'
        # wall-clock budgets end at different times (tests/test_bench_launch.py)
        skew = float(os.environ.get("BENCH_DRY_SKEW_MS", "0")) * 1e-3 * rank

        def run_fused(record, ev):
            if record:
                e = [Event(enable_timing=True) for _ in range(2)]
                e[0].record()
            y = (x * 0.75 + 0.125).to(bf16)
            if record:
                e[1].record()
                ev.append(e)
            return y
        run_unfused = run_fused
    else:
        from HyGrid import ops
        from HyGrid.HexFrames import HexConv2d
        from HyGrid.pipeline import hex_pyramid, rect_hex_conv_rect, rect_hex_rect

        gen = torch.Generator(device=dev).manual_seed(2 + rank)
        x = torch.rand((B, C, H, W), generator=gen, device=dev, dtype=bf16)
        torch.manual_seed(3)
        conv = HexConv2d(C, C, 0, 2, padding=1, groups=1, bias=True).to(dev)
        conv.out_dtype = bf16

        def run_unfused(record, ev):
            if record:
                e = [Event(enable_timing=True) for _ in range(4)]
                e[0].record()
            h = ops.rect_to_hex(x, (H, W), out_dtype=bf16)
            if record:
                e[1].record()
            c = conv(h)
            if record:
                e[2].record()
            y = ops.hex_to_rect(c, (H, W), out_dtype=bf16)
            if record:
                e[3].record()
                ev.append(e)
            return y

        def run_fused(record, ev):
            if record:
                e = [Event(enable_timing=True) for _ in range(2)]
                e[0].record()
            y = rect_hex_conv_rect(x, conv, (H, W), (H, W), out_dtype=bf16)
            if record:
                e[1].record()
                ev.append(e)
            return y

    from HyGrid.dist import gather_sums
    sums_buf = {}

    def step_sums(y):
        """Per-image, per-channel sums of every 256th output row, all-gathered over RCCL: the
        collective every timed step ends with (a few KB per rank), at every N (N = 1: the
        world-1 group).  Row sums first (contiguous inner reduction), then over the sampled
        rows: every 64th row cost 0.037 ms per 4K b128 step this way, against 0.159 ms for one
        reduction over both dims of the strided view (profiles/r06/step_sums_probe.txt); every
        256th row (9 of 2160) keeps it near 0.01 ms.  The world-1 all-gather is 0.017 ms."""
        s_ = torch.sum(y[:, :, ::256], -1, dtype=torch.float32).sum(-1).to(cdev)
        key = tuple(s_.shape)
        if key not in sums_buf:
            sums_buf[key] = torch.empty((world * s_.shape[0],) + key[1:], dtype=s_.dtype,
                                        device=cdev)
        gather_sums(s_, out=sums_buf[key])

    def measure(fn, steps, warmup, collective=True):
        """W untimed steps, then K steps between barrier + synchronize; max over ranks."""
        ev = []
        with torch.no_grad():
            for _ in range(warmup):
                y = fn(False, ev)
                if collective:
                    step_sums(y)
            sync()
            dist.barrier()
            sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                y = fn(True, ev)
                if collective:
                    step_sums(y)
            sync()
            dist.barrier()
            t1 = time.perf_counter()
        el = torch.tensor([t1 - t0], dtype=torch.float64, device=cdev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        n = len(ev[0]) - 1
        # per-kernel times from HIP events recorded on the launch stream
        stage_ms = [sum(e[i].elapsed_time(e[i + 1]) for e in ev) / len(ev) for i in range(n)]
        return y, float(el.item()), stage_ms

    def prewarm(fn, ms):
        """Untimed steps (with the per-step collective) for `ms` of wall time: clock /
        power-state settle, and first-use costs (allocations, code-object loads) paid here
        rather than as an idle gap right before the timed steps.  Every rank runs the same
        number of rounds of 8 steps (a MAX all-reduce of "my time is not up" after each round):
        a per-rank wall-clock loop would let ranks run different numbers of collectives and
        hang at N > 1."""
        if ms <= 0:
            return 0
        ev_, n = [], 0
        with torch.no_grad():
            t_end = time.perf_counter() + ms * 1e-3
            while True:
                for _ in range(8):
                    step_sums(fn(False, ev_))
                n += 8
                sync()
                go = torch.tensor([1.0 if time.perf_counter() < t_end else 0.0],
                                  dtype=torch.float64, device=cdev)
                dist.all_reduce(go, op=dist.ReduceOp.MAX)
                if go.item() == 0.0:
                    break
        dist.barrier()
        return n

    def measure_line(fn, steps):
        """A secondary line: 100 ms of untimed pre-warm of its own step and max(3, W) warmup
        steps (the same steady state the headline is timed in: a kernel run right after a
        different one starts at a lower clock, profiles/r03/final/kernel_medians.json), then
        K timed steps; never the per-step collective (not the headline)."""
        with torch.no_grad():
            t_end = time.perf_counter() + 0.1
            while time.perf_counter() < t_end:
                fn(False, [])
                sync()
        return measure(fn, steps, max(3, args.warmup), collective=False)

    img_bytes = B * C * H * W * 2          # one bf16 batch tensor
    if dry and skew > 0:
        time.sleep(skew)
    n_pre = prewarm(run_unfused if args.unfused else run_fused, args.prewarm_ms)
    # every rank's pre-warm step count (equal by construction; reported so a test can check)
    pre_all = torch.zeros(world, dtype=torch.float64, device=cdev)
    dist.all_gather_into_tensor(pre_all, torch.tensor([float(n_pre)], dtype=torch.float64,
                                                      device=cdev))
    prewarm_steps = [int(v) for v in pre_all.tolist()]
    if args.unfused:
        stages = ("rect_to_hex", "hexconv2d", "hex_to_rect")
        y, elapsed, sms = measure(run_unfused, args.steps, args.warmup)
    else:
        stages = ("pipeline_r2h_conv_h2r",)
        y, elapsed, sms = measure(run_fused, args.steps, args.warmup)
    stage_ms = dict(zip(stages, sms))
    ms_per_step = elapsed / args.steps * 1e3
    mpix = world * B * H * W * args.steps / elapsed / 1e6
    alg_bytes = {s: 2 * img_bytes for s in stages}   # each kernel: read once + write once
    kernels = {s: {"ms": round(stage_ms[s], 4), "alg_GB": round(alg_bytes[s] / 1e9, 4),
                   "GB_per_s": round(alg_bytes[s] / (stage_ms[s] * 1e-3) / 1e9, 1)}
               for s in stages}
    dom = max(stages, key=lambda s: stage_ms[s])
    achieved = alg_bytes[dom] / (stage_ms[dom] * 1e-3) / 1e9
    traffic, traffic_note = None, "no PMC profile"
    if not dry and os.path.exists(args.pmc_json):
        try:
            from HyGrid._abi import kernel_source_digest
            with open(args.pmc_json) as f:
                pmc = json.load(f)
            here = kernel_source_digest()
            if pmc.get("kernel_source_digest") != here:
                # a profile of other kernel code is not evidence for this build
                traffic_note = (f"{args.pmc_json} profiled kernel sources "
                                f"{pmc.get('kernel_source_digest')}, this tree is {here}")
            elif dom in pmc.get("kernels", {}):
                # per launch at the profiled batch, scaled to this run's batch
                traffic = pmc["kernels"][dom]["hbm_bytes_per_launch"] * B / pmc.get("batch", B)
                traffic_note = (f"rocprofv3 FETCH_SIZE(x2)+WRITE_SIZE at batch "
                                f"{pmc.get('batch', B)}, kernel sources {here}")
        except Exception as exc:  # keep the bench line even if the file is malformed
            log("pmc json unreadable:", exc)
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": traffic_note,
                "alg_bytes_per_launch": alg_bytes[dom],
                "limiter": FUSED4_LIMITER
                if dom == "pipeline_r2h_conv_h2r" else "hbm"}

    compare = None
    if not args.unfused and not dry and not args.no_compare:
        # the three-operator chain on the same data, reported beside `value` (never as it)
        steps_u = max(2, args.steps // 2)
        _, el_u, sms_u = measure_line(run_unfused, steps_u)
        ks = ("rect_to_hex", "hexconv2d", "hex_to_rect")
        compare = {"path": "rect_to_hex -> HexConv2d -> hex_to_rect (3 kernels, bf16 between)",
                   "value": round(world * B * H * W * steps_u / el_u / 1e6, 1),
                   "ms_per_step": round(el_u / steps_u * 1e3, 4),
                   "kernels": {k: {"ms": round(m, 4),
                                   "GB_per_s": round(2 * img_bytes / (m * 1e-3) / 1e9, 1)}
                               for k, m in zip(ks, sms_u)}}

    pyramid = None
    if not args.unfused and not dry and not args.no_pyramid:
        # BASELINE configs[4], per GPU: 8K fp16 rasters, r2h at full
        # size, then 3 x [depthwise HexConv2d(3,3,0,2,padding=1,groups=3) with Gaussian
        # taps [1,1,1,6,1,1,1]/12 -> hexresize to (h//2, w//2)].  Reported beside
        # `value`, never as it.
        f16 = torch.float16
        Hp, Wp, Bp = 4320, 7680, args.pyramid_batch
        xp = torch.rand((Bp, C, Hp, Wp), generator=gen, device=dev, dtype=f16)
        gconv = HexConv2d(C, C, 0, 2, padding=1, groups=C, bias=False).to(dev)
        with torch.no_grad():
            gconv.kernel.copy_(torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32,
                                            device=dev).div_(12).expand_as(gconv.kernel))
        gconv.out_dtype = f16
        levels = []

        def run_pyramid_unfused(record, ev):
            if record:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
                e[0].record()
            hx = ops.rect_to_hex(xp, (Hp, Wp), out_dtype=f16)
            if record:
                e[1].record()
            h_, w_ = Hp, Wp
            for lv in range(3):
                hx = gconv(hx)
                if record:
                    e[2 + 2 * lv].record()
                h_, w_ = h_ // 2, w_ // 2
                hx = ops.hexresize(hx, (h_, w_), out_dtype=f16)
                if record:
                    e[3 + 2 * lv].record()
            if record:
                ev.append(e)
            return hx

        def run_pyramid(record, ev):
            """HyGrid.pipeline.hex_pyramid, the product entry: the fused levels (level 0 straight
            from the rect image), one launch per level; HIP events around the whole step."""
            if record:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record()
            outs = hex_pyramid(xp, gconv, levels=3, out_dtype=f16)
            if record:
                e[1].record()
                ev.append(e)
            if not levels:
                levels.append(tuple(outs[-1].shape))
            return outs[-1]

        def run_pyramid_levels(record, ev):
            """The same levels as one launch each on one stream (hg_hex_pyramid_level x 3):
            HIP events per kernel, for the per-level breakdown."""
            if record:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                e[0].record()
            cur = xp
            h_, w_ = Hp, Wp
            for lv in range(3):
                h_, w_ = h_ // 2, w_ // 2
                cur = ops.hex_pyramid_level(cur, gconv.kernel, None, (h_, w_), 0,
                                            from_rect=(lv == 0), out_dtype=f16)
                if cur is None:
                    raise RuntimeError("pyramid level not fusable")
                if record:
                    e[1 + lv].record()
            if record:
                ev.append(e)
            if not levels:
                levels.append(tuple(cur.shape))
            return cur

        steps_p = max(2, args.steps // 2)
        _, el_p, _ = measure_line(run_pyramid, steps_p)
        _, el_p1, sms_p = measure_line(run_pyramid_levels, steps_p)
        _, el_pu, sms_pu = measure_line(run_pyramid_unfused, steps_p)
        lvl_bytes = []                                  # each level: read input + write output
        h_, w_ = Hp, Wp
        for lv in range(3):
            lvl_bytes.append(Bp * C * (h_ * w_ + (h_ // 2) * (w_ // 2)) * 2)
            h_, w_ = h_ // 2, w_ // 2
        # the unfused chain's own bytes: r2h read + write, then per level
        # the conv read + write and the hexresize read + write
        unf_bytes, h_, w_ = 2 * Hp * Wp, Hp, Wp
        for lv in range(3):
            unf_bytes += 2 * h_ * w_ + h_ * w_ + (h_ // 2) * (w_ // 2)
            h_, w_ = h_ // 2, w_ // 2
        unf_bytes *= Bp * C * 2
        names_u = ["rect_to_hex"] + [f"{k}_l{lv}" for lv in range(3) for k in ("hexconv_dw", "hexresize")]
        # each operator's own bytes (read its input + write its output), for its own fraction
        own_u, h_, w_ = [2 * Hp * Wp], Hp, Wp
        for lv in range(3):
            own_u += [2 * h_ * w_, h_ * w_ + (h_ // 2) * (w_ // 2)]
            h_, w_ = h_ // 2, w_ // 2
        own_u = [Bp * C * 2 * v for v in own_u]
        pyramid = {"workload": "config5: 8K RGB fp16, r2h -> 3 x [depthwise Gaussian HexConv2d "
                               "-> hexresize /2]",
                   "path": "HyGrid.pipeline.hex_pyramid: hg_hex_pyramid_level x 3 (conv + "
                           "hexresize, fp32 on chip; level 0 reads the rect image: rect -> hex "
                           "made on the fly)",
                   "levels_run": {"ms_per_step": round(el_p1 / steps_p * 1e3, 4),
                                  "what": "the same levels as one hg_hex_pyramid_level launch "
                                          "each, an event between kernels (the per-level times "
                                          "below)"},
                   "batch_per_gpu": Bp, "value": round(world * Bp * Hp * Wp * steps_p / el_p / 1e6, 1),
                   "unit": "Mpix/s", "ms_per_step": round(el_p / steps_p * 1e3, 4),
                   "dtype": "f16", "out_shape": list(levels[0]),
                   "alg_GB_fused": round(sum(lvl_bytes) / 1e9, 4),
                   "frac_of_peak": round(sum(lvl_bytes) / (el_p / steps_p) / PEAK_BPS, 4),
                   "kernels": {k: {"ms": round(m, 4), "alg_GB": round(b / 1e9, 4),
                                   "GB_per_s": round(b / (m * 1e-3) / 1e9, 1)}
                               for k, m, b in zip(["level0_from_rect", "level1", "level2"],
                                                  sms_p, lvl_bytes)},
                   "unfused": {"ms_per_step": round(el_pu / steps_p * 1e3, 4),
                               "alg_GB": round(unf_bytes / 1e9, 4),
                               "frac_of_peak": round(unf_bytes / (el_pu / steps_p) / PEAK_BPS, 4),
                               "kernels_ms": {k: round(m, 4) for k, m in zip(names_u, sms_pu)},
                               "kernels": {k: {"ms": round(m, 4), "alg_GB": round(b / 1e9, 4),
                                               "frac_of_peak": round(b / (m * 1e-3) / PEAK_BPS, 4)}
                                           for k, m, b in zip(names_u, sms_pu, own_u)}}}
        del xp

    roundtrip = None
    if not args.unfused and not dry and not args.no_roundtrip:
        # BASELINE configs[1]: 1080p RGB fp32, batch 32 per GPU,
        # rect->hex bilinear -> hex->rect linear.  Reported beside `value`, never as it.
        Hr, Wr, Br = 1080, 1920, 32
        xr = torch.rand((Br, C, Hr, Wr), generator=gen, device=dev, dtype=torch.float32)

        def run_roundtrip(record, ev):
            if record:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record()
            hx = ops.rect_to_hex(xr, (Hr, Wr))
            if record:
                e[1].record()
            out = ops.hex_to_rect(hx, (Hr, Wr))
            if record:
                e[2].record()
                ev.append(e)
            return out

        def run_roundtrip_fused(record, ev):
            if record:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record()
            out = rect_hex_rect(xr)
            if record:
                e[1].record()
                ev.append(e)
            return out

        steps_r = max(2, args.steps // 2)
        tb = Br * C * Hr * Wr * 4 * 2                 # each kernel: read once + write once
        # the round trip as one pass (hg_pipeline_r2h_h2r: hex image on chip in fp32) ...
        _, el_f, sms_f = measure_line(run_roundtrip_fused, steps_r)
        # ... and as the two resampler calls of the reference's API, beside it
        _, el_r, sms_r = measure_line(run_roundtrip, steps_r)
        roundtrip = {"workload": "config2: 1080p RGB fp32, rect->hex bilinear -> hex->rect linear",
                     "batch_per_gpu": Br, "dtype": "f32", "path": "fused (hg_pipeline_r2h_h2r)",
                     "value": round(world * Br * Hr * Wr * steps_r / el_f / 1e6, 1),
                     "unit": "Mpix/s", "ms_per_step": round(el_f / steps_r * 1e3, 4),
                     "kernels": {"pipeline_r2h_h2r": {
                         "ms": round(sms_f[0], 4), "alg_GB": round(tb / 1e9, 4),
                         "GB_per_s": round(tb / (sms_f[0] * 1e-3) / 1e9, 1),
                         "frac_of_peak": round(tb / (sms_f[0] * 1e-3) / PEAK_BPS, 4)}},
                     "unfused": {
                         "path": "rect_to_hex -> hex_to_rect (2 kernels, fp32 hex image in HBM)",
                         "value": round(world * Br * Hr * Wr * steps_r / el_r / 1e6, 1),
                         "ms_per_step": round(el_r / steps_r * 1e3, 4),
                         "alg_GB": round(2 * tb / 1e9, 4),
                         "frac_of_peak": round(2 * tb / (el_r / steps_r) / PEAK_BPS, 4),
                         "kernels": {k: {"ms": round(m, 4),
                                         "GB_per_s": round(tb / (m * 1e-3) / 1e9, 1)}
                                     for k, m in zip(("rect_to_hex", "hex_to_rect"), sms_r)}}}
        del xr

    wide = None
    if not args.unfused and not dry and not args.no_wide_conv:
        # HexConvModule-sized HexConv2d (HexModules.py:97-288): 64 -> 64 channels on a
        # 1080p bf16 batch of 4, the implicit GEMM on the bf16 matrix cores with every fp32
        # weight split into three bf16 parts (conv_mfma.hip, k_hexconv_mfma_bf16: exact
        # products, fp32 accumulation).  Compute-bound: algorithmic TFLOP/s (2 * O * 7 * C per
        # output sample) and the MFMA work actually issued (x 3 weight parts x 8/7 for the
        # zero eighth tap slot) against the dense bf16 MFMA peak.  Beside `value`, never as it.
        Bw, Cw, Ow, Hw, Ww = 4, 64, 64, 1080, 1920
        xw = (torch.rand((Bw, Cw, Hw, Ww), generator=gen, device=dev) - 0.5).to(bf16)
        torch.manual_seed(5)
        wconv = HexConv2d(Cw, Ow, 0, 2, padding=1, bias=True).to(dev)
        wconv.out_dtype = bf16

        def run_wide(record, ev):
            if record:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record()
            out = wconv(xw)
            if record:
                e[1].record()
                ev.append(e)
            return out

        steps_w = max(2, args.steps // 2)
        _, el_w, sms_w = measure_line(run_wide, steps_w)
        flop = 2.0 * Ow * 7 * Cw * Bw * Hw * Ww
        tf = flop / (sms_w[0] * 1e-3) / 1e12
        issued = tf * 3 * 8 / 7
        wide = {"workload": f"HexConv2d({Cw},{Ow},0,2,padding=1) bf16, {Bw}x{Cw}x{Hw}x{Ww}",
                "ms": round(sms_w[0], 4), "TFLOP_s": round(tf, 2),
                "vs_f32_mfma_peak": round(tf / 157.3, 4),
                "roofline": {"bound": "mfma", "achieved": round(issued, 1), "peak": 2500.0,
                             "unit": "TFLOP/s", "frac": round(issued / 2500.0, 4),
                             "note": "bf16 MFMA work issued (3 bf16 weight parts x 8/7 tap "
                                     "slots x the algorithmic flops) vs the dense bf16 peak; "
                                     "the algorithm's own ceiling is 2500 / 3 / (8/7) = 729 "
                                     "TFLOP/s of fp32-exact conv"}}
        del xw
        # the 3-channel stem of the same model, HexConv2d(3, 64) on the 1080p bf16 batch (round
        # 6: on the bf16 MFMA kernel with its channel chunk zero-padded, was the generic kernel):
        # bytes = input + 64-channel output, TFLOP/s on the algorithmic 2 * O * 7 * C
        Cs = 3
        xs_ = (torch.rand((Bw, Cs, Hw, Ww), generator=gen, device=dev) - 0.5).to(bf16)
        torch.manual_seed(6)
        sconv = HexConv2d(Cs, Ow, 0, 2, padding=1, bias=True).to(dev)
        sconv.out_dtype = bf16

        def run_stem(record, ev):
            if record:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record()
            out = sconv(xs_)
            if record:
                e[1].record()
                ev.append(e)
            return out

        _, _, sms_s = measure_line(run_stem, steps_w)
        sb = 2.0 * Bw * Hw * Ww * (Cs + Ow)
        wide["stem"] = {"workload": f"HexConv2d({Cs},{Ow},0,2,padding=1) bf16, {Bw}x{Cs}x{Hw}x{Ww}",
                        "ms": round(sms_s[0], 4), "alg_GB": round(sb / 1e9, 4),
                        "GB_per_s": round(sb / (sms_s[0] * 1e-3) / 1e9, 1),
                        "frac_of_peak": round(sb / (sms_s[0] * 1e-3) / PEAK_BPS, 4),
                        "TFLOP_s": round(2.0 * Ow * 7 * Cs * Bw * Hw * Ww / (sms_s[0] * 1e-3) / 1e12, 2)}
        del xs_

    lattices = None
    if not args.unfused and not dry and not args.no_lattices:
        lattices = bench_lattices(ops, measure_line, gen, dev, world, args.lattice_batch, C, H, W)

    # checksums over RCCL (not timed), and the full-output gather on its own
    from HyGrid.dist import gather_checksums, gather_to_root, image_checksums
    cs = image_checksums(y)
    gather = None
    if world > 1:
        cs = gather_checksums(cs.to(cdev))
        if not args.no_gather and not rehearse and not dry:
            try:
                gather_to_root(y)            # warm the RCCL channels
                torch.cuda.synchronize()
                dist.barrier()
                g0 = time.perf_counter()
                out = gather_to_root(y)
                torch.cuda.synchronize()
                g1 = time.perf_counter()
                del out
                gb = (world - 1) * y.numel() * y.element_size() / 1e9
                gather = {"GB_into_root": round(gb, 3), "ms": round((g1 - g0) * 1e3, 3),
                          "GB_per_s": round(gb / (g1 - g0), 1),
                          "xgmi_ingress_bound_GB_per_s": round(min(world - 1, 7) * 153.0, 1)}
            except Exception as exc:
                log("gather failed:", exc)
    checksum = float(cs[..., 0].sum().item())

    cpu = None
    if rank == 0 and world == 1 and args.cpu_images > 0 and not dry:
        try:
            cpu = cpu_baseline(args, conv.kernel.detach().cpu().numpy(),
                               conv.bias.detach().cpu().numpy())
        except Exception as exc:
            log("cpu baseline failed:", exc)

    if rank == 0:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            metric = json.load(f)["metric"]
        line = {
            "metric": metric, "value": round(mpix, 1), "unit": "Mpix/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "prewarm_ms": args.prewarm_ms, "prewarm_steps": prewarm_steps, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic U[0,1) bf16 rasters generated on device, seed 2+rank; "
                    "HexConv2d weights torch.manual_seed(3) + reference init",
            "config": {"workload": "config3: 4K RGB batch=128/GPU, rect->hex bilinear -> "
                                   "HexConv2d(3,3,off=0,r=2,pad=1) -> hex->rect linear",
                       "batch_per_gpu": B, "global_batch": B * world, "channels": C,
                       "height": H, "width": W,
                       "parallelism": f"dp{world}" + ("-rehearsal-gloo-1gpu" if rehearse else ""),
                       "fused": not args.unfused},
            "kernels": kernels, "roofline": roofline, "cpu_baseline": cpu,
            "unfused": compare, "roundtrip": roundtrip, "pyramid": pyramid, "wide_conv": wide,
            "lattices": lattices,
            "gather": gather, "checksum": checksum,
            "device": "cpu (dry run)" if dry else torch.cuda.get_device_name(dev),
        }
        if dry:
            line["dry_run"] = True
            line["data"] = ("--dry-run: a host stand-in step (no HIP kernel) on a "
                            f"{B}x{C}x{H}x{W} tensor; launcher / collectives / timing only, the "
                            "value is not a measurement")
        if line["n_gpus"] != args.gpus:
            raise SystemExit(f"bench: n_gpus {line['n_gpus']} != --gpus {args.gpus}")
        print(json.dumps(line), file=result_out, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
