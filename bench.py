#!/usr/bin/env python3
"""Benchmark of the Haar LL ("icon") hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--depth D] [--images B]

Workload (BASELINE.json configs[2], the roofline run, at the metric's depth 5):
a batch of B = 128 synthetic 8K RGB images (7680x4320x3 uint8) per GPU,
generated on device and resident in HBM before timing.  One step = one pass
of HaarCoder.get_small_copy's work over the whole batch through the C ABI
(``wicca_haar_ll_u8_uniform``: ONE kernel launch, no host copies).

Multi-GPU (``torch.distributed.run``, one rank per GPU): images shard
image-parallel with no data-path collective (weak scaling: B images per
rank).  A barrier + device sync brackets the K timed steps and the maximum
over ranks is reported.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (HIP
events on the launch stream) and, at N=1, the CPU baseline: the NumPy port of
the reference (oracle/haar_numpy.py) timed on a bounded sample of the same
workload on this host.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASELINE = json.load(open(os.path.join(REPO, "BASELINE.json")))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=["batch", "tiled", "multi", "ragged", "stage", "jpeg", "png", "bmp", "plan"],
                    default="batch",
                    help="batch: configs[2]/[3] image-parallel (default); "
                         "tiled: configs[4], one 65536^2 RGB image row-sharded at depth 8; "
                         "multi: configs[2]'s depth sweep 1..6 from one read (SURVEY 8f); "
                         "ragged: a batch of random-size images in one launch (A7 caller); "
                         "stage: the caller's whole per-image stage from host arrays "
                         "(resize + icon + icon resize, HaarCoder.icon_stage); "
                         "jpeg: GPU decode of 8K JPEG files (load_image) and the file-based "
                         "caller stage (decode + resize + icon + icon resize); "
                         "png / bmp: the same for 8K PNG (zlib level 6) / 24-bit BMP files")
    ap.add_argument("--quality", type=int, default=90, help="--config jpeg: encoder quality")
    ap.add_argument("--shape", default="224,224", help="--config stage: classifier input (w,h)")
    ap.add_argument("--tiled-as-rank", default="", help=argparse.SUPPRESS)
    ap.add_argument("--plan-no-loop", action="store_true",
                    help="--config plan: skip the per-call loop and its check (profiling runs)")
    ap.add_argument("--plan-batches", type=int, default=12,
                    help="--config plan: batches of distinct files the StagePlan loop walks")
    ap.add_argument("--kernel-only", action="store_true",
                    help="--config jpeg / plan: only the synchronous calls (the kernel-trace child run)")
    ap.add_argument("--no-kernel-trace", action="store_true",
                    help="skip the rocprofv3 --kernel-trace child run that times each kernel (batch: "
                         "the headline launch and the sweep; jpeg / plan: the per-kernel roofline entries)")
    ap.add_argument("--interpolation", type=int, default=3, help="--config stage: cv2.INTER_*")
    ap.add_argument("--depths", default="1,2,3,4,5,6", help="depth list of --config multi")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--images", type=int, default=128, help="images per GPU")
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--border", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--ragged-align", type=int, default=16,
                    help="--config ragged: row pitch alignment of the images (bytes)")
    ap.add_argument("--ragged-min", type=float, default=0.5,
                    help="--config ragged: sizes drawn from [ragged_min * size, size]")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-sweep", action="store_true",
                    help="batch config: skip the depth sweep 1..6 and the configs[1] leg")
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="batch config at N=1: skip the two rocprofv3 --pmc child runs that "
                         "measure roofline.traffic live (the committed --pmc summary is used)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print each rank's (rank, world) and exit before touching the GPU")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_r02.json"),
                    help="PMC summary (rocprofv3 FETCH_SIZE/WRITE_SIZE) for roofline.traffic")
    return ap.parse_args()


def _cpu_share():
    """CPUs this process may run on (affinity), the cgroup CPU quota (cpus, or
    None) and the memory the host reports available (bytes)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    avail = None
    try:
        with open("/proc/meminfo") as f:
            for ln in f:
                if ln.startswith("MemAvailable:"):
                    avail = int(ln.split()[1]) * 1024
    except (OSError, ValueError):
        pass
    return aff, quota, avail


def cpu_baseline(args, budget_s: float):
    """NumPy port of the reference on this host (oracle/haar_numpy.py).

    BASELINE.md §3(b): image-parallel ``ThreadPoolExecutor`` sized to what
    the host lets this process run — min(CPU affinity, cgroup CPU quota,
    memory: the port widens an 8K RGB image to a 398 MB float32 plane, ~0.8 GB
    of working set per thread).  A 16-thread pool and (when small enough) the
    whole-affinity pool are timed beside it; ``value`` is the best of them.
    The single-thread rate (one ClassifierProcessor worker) is reported too.
    """
    from concurrent.futures import ThreadPoolExecutor

    from oracle import haar_numpy
    from wicca_amd.synth import synth_image

    H, W, C, d = args.height, args.width, args.channels, args.depth
    mp = H * W / 1e6
    per_thread_bytes = 8 * H * W * C  # u8 image + f32 plane + level-1 sums, with slack
    pool_imgs = [synth_image(1234, i, H, W, C) for i in range(4)]

    def one(i):
        haar_numpy.get_small_copy(pool_imgs[i % 4], d, args.border)

    # single thread, as ClassifierProcessor runs it in one worker
    t0 = time.perf_counter()
    n1 = 0
    while True:
        one(n1)
        n1 += 1
        if time.perf_counter() - t0 > budget_s / 4 or n1 >= 64:
            break
    single = n1 * mp / (time.perf_counter() - t0)

    def pool_rate(threads: int, n: int) -> float:
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(one, range(min(threads, 8))))  # warm the pool
            t = time.perf_counter()
            list(ex.map(one, range(n)))
            return n * mp / (time.perf_counter() - t)

    aff, quota, avail = _cpu_share()
    mem_cap = max(1, int(0.5 * avail / per_thread_bytes)) if avail else 64
    # the pool the host can actually run: min(affinity, cgroup quota, memory)
    threads = max(1, min(aff, int(quota) if quota else aff, mem_cap))
    n_all = max(threads, int(single * threads * budget_s / 2 / mp) // threads * threads)
    n_all = min(n_all, 4 * threads)
    rates = {threads: pool_rate(threads, n_all)}
    t16 = min(16, aff, mem_cap)
    if t16 not in rates:
        rates[t16] = pool_rate(t16, 2 * t16)
    t_aff = min(aff, mem_cap)
    if t_aff not in rates and t_aff <= 64:  # a pool past the quota (throttled), for comparison
        rates[t_aff] = pool_rate(t_aff, t_aff)
    best = max(rates, key=lambda t: rates[t])
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {
        "value": round(rates[best], 2), "unit": "MP/s", "cores": best, "kind": "port",
        "sample": f"synthetic {W}x{H}x{C} images (seed 1234) at depth {d}: {n_all} images on "
                  f"ThreadPoolExecutor({threads}) (min of CPU affinity {aff}, cgroup quota "
                  f"{quota}, memory cap {mem_cap}); {n1} images single-threaded; value = the "
                  "best pool rate",
        "single_thread_value": round(single, 2),
        "pool_rates": {str(t): round(r, 2) for t, r in sorted(rates.items())},
        "affinity_cpus": aff, "cgroup_cpu_quota": quota, "memory_thread_cap": mem_cap,
        "host_cpus": os.cpu_count(), "cpu_model": model,
    }


def live_pmc(args, kernel: str, timeout_s: float = 150.0, extra=None):
    """roofline.traffic measured in this run: two child runs of this bench's
    workload under rocprofv3, one counter per pass (FETCH_SIZE, WRITE_SIZE;
    gfx950 TCC slots cannot hold both), corrected as tools/pmc_summary.py does
    (KiB; FETCH_SIZE counts half of a wide coalesced read stream).  Children,
    not exec: this process has initialised the GPU.  None when rocprofv3 is
    absent or a pass fails (the caller falls back to the committed summary)."""
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    # already under a profiler (e.g. rocprofv3 --kernel-trace around this
    # bench): a nested rocprofv3 would inherit its preload, so use the fallback
    if any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ) or \
            "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None
    child = [sys.executable, os.path.abspath(__file__), "--steps", "3", "--warmup", "1",
             "--no-verify", "--no-cpu-baseline", "--no-live-pmc", "--no-sweep", "--no-kernel-trace",
             "--images", str(args.images), "--height", str(args.height), "--width", str(args.width),
             "--channels", str(args.channels), "--depth", str(args.depth),
             "--border", str(args.border), "--seed", str(args.seed)] + list(extra or [])
    env = dict(os.environ, TMPDIR="/tmp")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    kib = {}
    with tempfile.TemporaryDirectory(prefix="wicca_pmc_", dir="/tmp") as tmp:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out_dir = os.path.join(tmp, counter)
            try:
                r = subprocess.run([prof, "--pmc", counter, "--output-format", "csv", "-d", out_dir,
                                    "--"] + child, cwd="/tmp", env=env, timeout=timeout_s,
                                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            except (OSError, subprocess.TimeoutExpired):
                return None
            if r.returncode != 0:
                return None
            kib[counter] = pmc_counter_kib(out_dir, counter, kernel)
            if kib[counter] is None:
                return None
    return pmc_hbm_bytes(kib["FETCH_SIZE"], kib["WRITE_SIZE"])


def pmc_counter_kib(out_dir: str, counter: str, kernel: str):
    """Mean per-launch value of `counter` over the launches of `kernel` (a
    substring of rocprofv3's Kernel_Name) in a --pmc run's counter_collection
    CSVs under out_dir; None when there are none."""
    import csv
    import glob

    vals = []
    for path in glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == counter and kernel in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


def pmc_hbm_bytes(fetch_kib: float, write_kib: float):
    """gfx950 corrections (MI355X_MICROARCH.md, HBM section): both counters
    in KiB; FETCH_SIZE reports half of a wide coalesced read stream."""
    read_b = fetch_kib * 1024 * 2
    write_b = write_kib * 1024
    return {"read_bytes": read_b, "write_bytes": write_b, "hbm_bytes_per_launch": read_b + write_b}


def kernel_trace_child(args, extra, timeout_s: float = 300.0):
    """Per-kernel durations of this bench's workload: a child run of it under
    rocprofv3 --kernel-trace (a child, not exec: this process has initialised
    the GPU).  {kernel name: (launches, mean duration in us)}; None when
    rocprofv3 is absent, nested, or the run fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof) or any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ) or \
            "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None
    child = [sys.executable, os.path.abspath(__file__), "--no-verify", "--no-cpu-baseline", "--no-live-pmc",
             "--no-kernel-trace", "--kernel-only"] + list(extra)
    env = dict(os.environ, TMPDIR="/tmp")
    with tempfile.TemporaryDirectory(prefix="wicca_kt_", dir="/tmp") as tmp:
        try:
            r = subprocess.run([prof, "--kernel-trace", "--output-format", "csv", "-d", tmp, "--"] + child,
                               cwd="/tmp", env=env, timeout=timeout_s, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL)
        except (OSError, subprocess.TimeoutExpired):
            return None
        if r.returncode != 0:
            return None
        durs = {}
        for path in glob.glob(os.path.join(tmp, "**", "*kernel_trace.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    durs.setdefault(row["Kernel_Name"], []).append(
                        int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return {k: (len(v), sum(v) / len(v) / 1e3) for k, v in durs.items()} if durs else None


def kernel_trace_grid(args, extra, timeout_s: float = 240.0):
    """The headline's kernel-trace child: this bench's workload (timed steps,
    depth sweep, configs[1] leg) under rocprofv3 --kernel-trace, a child run
    (this process has initialised the GPU).  {(kernel name, grid x): (launches,
    mean duration in us)} -- the grid separates launches of one kernel on
    different batches (configs[2] and configs[1] at depth 3); None when
    rocprofv3 is absent, nested, or the run fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof) or any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ) or \
            "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None
    child = [sys.executable, os.path.abspath(__file__), "--no-verify", "--no-cpu-baseline", "--no-live-pmc",
             "--no-kernel-trace"] + list(extra)
    env = dict(os.environ, TMPDIR="/tmp")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    with tempfile.TemporaryDirectory(prefix="wicca_kt_", dir="/tmp") as tmp:
        try:
            r = subprocess.run([prof, "--kernel-trace", "--output-format", "csv", "-d", tmp, "--"] + child,
                               cwd="/tmp", env=env, timeout=timeout_s, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL)
        except (OSError, subprocess.TimeoutExpired):
            return None
        if r.returncode != 0:
            return None
        durs = {}
        for path in glob.glob(os.path.join(tmp, "**", "*kernel_trace.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    key = (row["Kernel_Name"], int(row.get("Grid_Size_X") or 0))
                    t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                    durs.setdefault(key, []).append((t0, t1 - t0))
    return {k: (len(v), sum(d for _, d in v) / len(v) / 1e3, min(t for t, _ in v))
            for k, v in durs.items()} if durs else None


def trace_lookup(stats, name, which=0):
    """(launches, mean us) of the kernel-trace group (one kernel name
    containing `name`, one grid) that ran `which`-th among that kernel's
    groups (by first launch: 0 the first, -1 the last); None when absent."""
    hits = sorted((t, n, us) for (k, _), (n, us, t) in (stats or {}).items() if name in k)
    if not hits:
        return None
    _, n, us = hits[which]
    return n, us


def run_sweep(args, torch, lib, src, B, H, W, C, pitch, stream, sh, seed):
    """BASELINE configs[2]'s transform_depth sweep 1..6 on the headline's
    device-resident batch, and configs[1] (32 x 4K RGB, depth 3) on a batch of
    its own: per entry one wicca_haar_ll_u8_uniform launch per step timed by
    HIP events on the launch stream, algorithmic bytes (image read once, icon
    written once) over that time, and -- unless --no-verify -- the first and
    last image of the batch checked against the C oracle (oracle/haar_oracle.c,
    pinned by the reference's goldens).  Returns the entries, one per leg, in
    the order the legs run (configs[2] first)."""
    from wicca_amd import _lib

    steps = args.steps
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    legs = [("configs[2]", d, B, H, W) for d in range(1, 7)] + [("configs[1]", 3, 32, 2160, 3840)]
    big = max(n * -(-h >> d) * ((-(-w >> d) * C + 15) // 16 * 16) for _, d, n, h, w in legs)
    dst = torch.empty(big, dtype=torch.uint8, device="cuda")
    src4k = None
    for cfg, d, n, h, w in legs:
        if cfg == "configs[1]":
            p = (w * C + 15) // 16 * 16
            src4k = torch.empty(n * h * p, dtype=torch.uint8, device="cuda")
            _lib.check(lib.wicca_synth_u8(ctypes.c_void_p(src4k.data_ptr()), n, h, w, C, p, h * p,
                                          seed + 7919, -1, sh))
            s, sp, sd = src4k, p, seed + 7919
        else:
            s, sp, sd = src, pitch, seed
        oh, ow = -(-h >> d), -(-w >> d)
        op = (ow * C + 15) // 16 * 16

        def launch():
            _lib.check(lib.wicca_haar_ll_u8_uniform(
                ctypes.c_void_p(s.data_ptr()), n, h, w, C, sp, h * sp, d, args.border, 0,
                ctypes.c_void_p(dst.data_ptr()), op, oh * op, -1, sh))
        for _ in range(max(1, args.warmup)):
            launch()
        torch.cuda.synchronize()
        ev0.record(stream)
        for _ in range(steps):
            launch()
        ev1.record(stream)
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / steps
        alg = n * (h * w * C + oh * ow * C)
        e = {"config": cfg, "images": n, "height": h, "width": w, "depth": d,
             "kernel": lib.wicca_kernel_name(d, C, 0).decode(), "launches": steps,
             "kernel_ms": round(ms, 4), "alg_bytes_per_launch": alg,
             "achieved": round(alg / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
             "MP_per_s": round(n * h * w / 1e6 / (ms / 1e3), 1)}
        if not args.no_verify:
            from oracle import c_oracle
            from wicca_amd.synth import synth_image
            ok = True
            for i in sorted({0, n - 1}):
                ref = c_oracle.ll_int_block(synth_image(sd, i, h, w, C), d, args.border)[0]
                got = dst[i * oh * op:(i + 1) * oh * op].view(oh, op)[:, :ow * C].cpu().numpy()
                ok = ok and bool(np.array_equal(got.reshape(oh, ow, C), ref))
            if not ok:
                raise SystemExit(f"bench sweep verification FAILED: {cfg} depth {d}")
            e["verified_images"] = sorted({0, n - 1})
        out.append(e)
    del src4k, dst
    return out


def kernel_rooflines(stats, table):
    """Per-kernel roofline entries: table = [(label, name substring, algorithmic
    bytes per launch, what the bytes are)]; the duration is the mean over the
    launches whose name contains the substring (rocprofv3 kernel trace)."""
    out = []
    for entry in table:
        label, sub, alg, what = entry[:4]
        per = entry[4] if len(entry) > 4 else 1  # launches per call: alg is then the call's bytes
        hits = [(n, us) for k, (n, us) in (stats or {}).items() if sub in k]
        if not hits:
            continue
        n = sum(h[0] for h in hits)
        us = sum(h[0] * h[1] for h in hits) / n * per
        gbs = alg / (us * 1e-6) / 1e9
        e = {"kernel": label, "launches": n, "avg_us": round(us, 1), "alg_bytes_per_launch": int(alg),
             "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes": what}
        if per > 1:
            e["launches_per_call"] = per
            e["note"] = f"avg_us and alg_bytes_per_launch are per call ({per} launches)"
        out.append(e)
    return out


def distinct_jpegs(args, count, H, W, seed0=40):
    """`count` distinct JPEG files of H x W: four synthetic scenes, each file a
    different cyclic shift (and every other group mirrored) of one of them, so
    no two files share their entropy-coded data; encoded in parallel."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import jpeg_pil
    base = [jpeg_pil.test_image("scene", H, W, seed0 + k) for k in range(min(4, count))]

    def make(j):
        img = np.roll(base[j % len(base)], ((j * 977) % H, (j * 1931) % W), (0, 1))
        if (j // len(base)) % 2:
            img = img[:, ::-1]
        return jpeg_pil.encode(np.ascontiguousarray(img), args.quality, 2)
    if os.environ.get("WICCA_BENCH_REPEAT4"):  # diagnostic: four files repeated (the round-4 legs)
        four = [jpeg_pil.encode(b, args.quality, 2) for b in base]
        return [four[j % len(four)] for j in range(count)]
    with ThreadPoolExecutor(min(16, len(os.sched_getaffinity(0)))) as ex:
        return list(ex.map(make, range(count)))


def jpeg_geometry(H, W):
    """Bytes of one H x W 4:2:0 JPEG's decode buffers: (luma coefficient, chroma
    coefficient, chroma plane, RGB) -- int16 blocks padded to whole MCUs, 8-bit
    chroma planes at whole-MCU size, RGB at a 128-B pitch."""
    mx, my = -(-W // 16), -(-H // 16)
    luma = mx * 2 * my * 2 * 128
    chroma = 2 * mx * my * 128
    planes = 2 * mx * 8 * my * 8
    rgb = W * 3 * H  # the bytes of the image (the pitch's slack is never written)
    return luma, chroma, planes, rgb


def read_pmc(path: str, workload_key: str):
    try:
        with open(path) as f:
            data = json.load(f)
        return data.get(workload_key)
    except (OSError, ValueError):
        return None


def run_tiled(args, torch, dist, world, rank, local_rank):
    """BASELINE configs[4]: one oversize image, 2^D-aligned row bands per rank,
    no halo, one RCCL all_gather of the icon slabs (wicca_amd.parallel.TiledHaar)."""
    from wicca_amd import _lib
    from wicca_amd.parallel import TiledHaar, aligned_bands

    lib = _lib.load()
    H = args.height if args.height != 4320 else 65536
    W = args.width if args.width != 7680 else 65536
    C, D = args.channels, (args.depth if args.depth != 5 else 8)
    band_rank, band_world = rank, world
    if args.tiled_as_rank:  # a single-process child timing one rank's band (live PMC of the N-rank line)
        band_rank, band_world = (int(x) for x in args.tiled_as_rank.split("/"))
    bounds = aligned_bands(H, band_world, D)
    y0, y1 = bounds[band_rank]
    pitch = W * C
    if pitch % 16:
        raise SystemExit("tiled bench needs W*C % 16 == 0")
    band = torch.empty((y1 - y0, W, C), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sh = ctypes.c_void_p(stream.cuda_stream)
    _lib.check(lib.wicca_synth_band_u8(ctypes.c_void_p(band.data_ptr()), y1 - y0, W, C, pitch,
                                       args.seed, 0, y0, -1, sh))
    r = 1 << D
    oh, ow = -(-H // r), -(-W // r)
    th = TiledHaar(D, args.border, 0)
    icon_local = torch.empty(((y1 - y0 + r - 1) // r, ow, C), dtype=torch.uint8, device="cuda")

    def slab_kernel():
        _lib.check(lib.wicca_haar_ll_u8(
            ctypes.c_void_p(band.data_ptr()), y1 - y0, W, C, pitch, D, args.border, 0,
            ctypes.c_void_p(icon_local.data_ptr()), ow * C, 1, 1, -1, sh))

    def step():
        if dist is None:
            slab_kernel()
            return icon_local
        return th(band, y0, H, bounds)

    if args.tiled_as_rank:  # PMC child: the band kernel only
        for _ in range(args.warmup + args.steps):
            slab_kernel()
        torch.cuda.synchronize()
        return None

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # kernel-only timing of this rank's band (roofline)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        slab_kernel()
    e1.record(stream)
    torch.cuda.synchronize()
    kernel_ms = e0.elapsed_time(e1) / args.steps
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        icon = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([wall, kernel_ms], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, kernel_ms = float(t[0]), float(t[1])
    verified = None
    if not args.no_verify and rank == 0:
        # spot-check the first and the last two icon rows against the CPU port
        from oracle import haar_numpy
        from wicca_amd.synth import synth_rows
        full = icon.cpu().numpy()
        verified = tuple(full.shape) == (oh, ow, C)
        last0 = max(0, (oh - 2) * r)
        for a, b in ((0, min(H, 2 * r)), (last0, H)):
            ref = haar_numpy.get_small_copy(synth_rows(args.seed, 0, a, b - a, W, C), D,
                                            args.border)
            verified = verified and bool(np.array_equal(full[a // r:a // r + ref.shape[0]], ref))
        if not verified:
            raise SystemExit("tiled bench verification FAILED")
    if rank != 0:
        return None
    ms = wall / args.steps * 1e3
    band_bytes = (y1 - y0) * W * C + ((y1 - y0 + r - 1) // r) * ow * C
    kname = lib.wicca_kernel_name(D, C, 0).decode()
    pmc = None
    if not args.no_live_pmc:  # HBM bytes of rank 0's band kernel, two PMC child runs
        pmc = live_pmc(args, kname.split("<")[0], extra=["--config", "tiled", "--tiled-as-rank",
                                                         f"0/{world}"])
    return {
        "metric": BASELINE["metric"],
        "value": round(H * W / 1e6 / (ms / 1e3), 1),
        "unit": "MP/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (on-device splitmix64 image bands, HBM-resident before timing)",
        "config": {"workload": f"1 x {W}x{H}x{C} uint8 image, Haar LL depth {D}, row bands "
                               f"aligned to 2^{D} (BASELINE.json configs[4])",
                   "height": H, "width": W, "channels": C, "depth": D,
                   "parallelism": f"row-band tiles x{world}, no halo, all_gather of icon slabs"},
        "roofline": {"bound": "hbm", "achieved": round(band_bytes / (kernel_ms / 1e3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(band_bytes / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": round(pmc["hbm_bytes_per_launch"]) if pmc else None,
                     "kernel": kname + " (rank-0 band)",
                     "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": band_bytes,
                     "pmc_source": "live (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child runs of rank 0's band)"
                     if pmc else None},
        "cpu_baseline": None,
        "verified_vs_numpy_port": verified,
    }


def run_ragged(args, torch, rank):
    """A ragged batch (the caller's real shape: files of different sizes) in
    ONE launch through wicca_haar_ll_u8_batch with device descriptors."""
    from wicca_amd import _lib
    lib = _lib.load()
    B, C, D = args.images, args.channels, args.depth
    rng = np.random.default_rng(args.seed)
    Hs = rng.integers(int(args.height * args.ragged_min), args.height + 1, B)
    Ws = rng.integers(int(args.width * args.ragged_min), args.width + 1, B)
    r = 1 << D
    al = args.ragged_align
    pitches = [(int(w) * C + al - 1) // al * al for w in Ws]
    ohs = [-(-int(h) // r) for h in Hs]
    ows = [-(-int(w) // r) for w in Ws]
    opitches = [(ow * C + 15) // 16 * 16 for ow in ows]
    in_off = np.concatenate([[0], np.cumsum([p * int(h) for p, h in zip(pitches, Hs)])])
    out_off = np.concatenate([[0], np.cumsum([p * oh for p, oh in zip(opitches, ohs)])])
    src = torch.empty(int(in_off[-1]), dtype=torch.uint8, device="cuda")
    dst = torch.empty(int(out_off[-1]), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sh = ctypes.c_void_p(stream.cuda_stream)
    for i in range(B):
        h, w = int(Hs[i]), int(Ws[i])
        _lib.check(lib.wicca_synth_u8(ctypes.c_void_p(src.data_ptr() + int(in_off[i])), 1, h, w, C,
                                      pitches[i], h * pitches[i], args.seed * 1000003 + i, -1, sh))
    # three orderings of the same images, used in turn: the library keeps the
    # last two descriptor sets on device, so every call uploads its descriptors
    # as a new batch would (no reuse in the timed region)
    rot = []
    for k in range(3):
        order = list(range(k, B)) + list(range(k))
        descs = (_lib.ImageDesc * B)()
        for j, i in enumerate(order):
            descs[j] = _lib.ImageDesc(src.data_ptr() + int(in_off[i]), dst.data_ptr() + int(out_off[i]),
                                      int(Hs[i]), int(Ws[i]), pitches[i], opitches[i])
        rot.append(descs)
    calls = [0]

    def step():
        descs = rot[calls[0] % 3]
        calls[0] += 1
        _lib.check(lib.wicca_haar_ll_u8_batch(descs, B, C, D, args.border, 0, 1, 1, -1, sh))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t0) / args.steps * 1e3
    dev_ms = e0.elapsed_time(e1) / args.steps
    verified = None
    if not args.no_verify:
        from oracle import haar_numpy
        from wicca_amd.synth import synth_image
        i = B - 1
        h, w = int(Hs[i]), int(Ws[i])
        ref = haar_numpy.get_small_copy(synth_image(args.seed * 1000003 + i, 0, h, w, C), D,
                                        args.border)
        raw = dst[int(out_off[i]):int(out_off[i]) + opitches[i] * ohs[i]].view(ohs[i], opitches[i])
        got = raw[:, :ows[i] * C].cpu().numpy().reshape(ohs[i], ows[i], C)
        verified = bool(np.array_equal(got, ref))
        if not verified:
            raise SystemExit("ragged bench verification FAILED")
    alg = int(sum(int(h) * int(w) * C for h, w in zip(Hs, Ws)) + sum(oh * ow * C for oh, ow in zip(ohs, ows)))
    mpix = float(sum(int(h) * int(w) for h, w in zip(Hs, Ws))) / 1e6
    return {
        "metric": BASELINE["metric"], "value": round(mpix / (wall_ms / 1e3), 1), "unit": "MP/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall_ms, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (on-device splitmix64 images of random sizes, HBM-resident before timing)",
        "config": {"workload": f"ragged batch of {B} RGB images, H in [{int(args.height * args.ragged_min)}, "
                               f"{args.height}], W in [{int(args.width * args.ragged_min)}, {args.width}], depth {D}, "
                               "one launch (device descriptors)",
                   "images": B, "megapixels": round(mpix, 2), "depth": D},
        "roofline": {"bound": "hbm", "achieved": round(alg / (dev_ms / 1e3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(alg / (dev_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": lib.wicca_kernel_name(D, C, 1).decode() +
                               " (+ descriptor upload; stream time per call)",
                     "kernel_ms": round(dev_ms, 4), "alg_bytes_per_launch": alg},
        "cpu_baseline": None, "verified_vs_numpy_port": verified,
    }


def run_stage(args, torch, rank):
    """ClassifierProcessor._get_img_batch's per-image work (classifying_tools.py:
    312-323: source resize, icon, icon resize, stack) for a batch of decoded
    HOST images — PCIe-inclusive, so never the headline value."""
    from wicca_amd import HaarCoder, _lib
    lib = _lib.load()
    B = 25 if args.images == 128 else args.images  # the caller's batch_size default (:124)
    H, W, C, D = args.height, args.width, args.channels, args.depth
    shape = tuple(int(x) for x in args.shape.split(","))
    pitch = W * C
    dev = torch.empty(B * H * pitch, dtype=torch.uint8, device="cuda")
    _lib.check(lib.wicca_synth_u8(ctypes.c_void_p(dev.data_ptr()), B, H, W, C, pitch, H * pitch,
                                  args.seed, -1, None))
    host = dev.cpu().numpy().reshape(B, H, W, C)
    del dev
    imgs = [host[i] for i in range(B)]
    coder = HaarCoder(device=None)  # the rank's current device
    for _ in range(args.warmup):
        coder.icon_stage(imgs, D, shape, args.interpolation)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, icons = coder.icon_stage(imgs, D, shape, args.interpolation)
    wall = (time.perf_counter() - t0) / args.steps
    verified = None
    if not args.no_verify:
        from oracle import haar_numpy, resize_cv
        i = B - 1
        verified = bool(np.array_equal(res[i], resize_cv.resize(imgs[i], shape, args.interpolation)))
        icon = haar_numpy.get_small_copy(imgs[i], D)
        verified = verified and bool(np.array_equal(icons[i], resize_cv.resize(icon, shape,
                                                                               args.interpolation)))
        if not verified:
            raise SystemExit("stage bench verification FAILED")
    mpix = B * H * W / 1e6
    return {
        "metric": BASELINE["metric"], "value": round(mpix / wall, 1), "unit": "MP/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic host images (numpy, pageable), PCIe inside the timed region",
        "config": {"workload": f"{B} host {W}x{H}x{C} images per call: cv2.resize to {shape} "
                               f"(INTER {args.interpolation}) + icon depth {D} + icon resize "
                               "(classifying_tools.py:312-323)",
                   "images": B, "depth": D, "shape": shape},
        "h2d_GBps_effective": round(B * H * W * C / wall / 1e9, 2),
        "roofline": None, "cpu_baseline": None, "verified_vs_numpy_port": verified,
    }


def run_jpeg(args, torch, rank):
    """load_image (data_loader.py:31-63) on the GPU: B JPEG files of the
    configs[2] size decoded in one call into device RGB buffers, then the whole
    file-based _get_img_batch stage (classifying_tools.py:297-323).  The files
    are already in host memory (no disk I/O); the CPU baseline is libjpeg-turbo
    itself through Pillow (the decoder cv2.imread wraps)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import jpeg_pil
    from wicca_amd import _lib
    lib = _lib.load()
    B = 25 if args.images == 128 else args.images
    H, W, D = args.height, args.width, args.depth
    blobs = distinct_jpegs(args, B, H, W)  # B distinct files: no file's data is read twice
    keep = [np.frombuffer(b, np.uint8) for b in blobs]
    ptrs = (ctypes.c_void_p * B)(*[k.ctypes.data for k in keep])
    sizes = (ctypes.c_int64 * B)(*[k.size for k in keep])
    pitch = (W * 3 + 127) // 128 * 128
    dev = torch.empty(B * H * pitch, dtype=torch.uint8, device="cuda")
    dsts = (ctypes.c_void_p * B)(*[dev.data_ptr() + i * H * pitch for i in range(B)])
    pitches = (ctypes.c_int64 * B)(*([pitch] * B))
    stream = torch.cuda.Stream()
    sh = ctypes.c_void_p(stream.cuda_stream)

    def decode():
        _lib.check(lib.wicca_jpeg_decode_u8(ptrs, sizes, B, dsts, pitches, 1, 1, -1, sh, None))
        stream.synchronize()

    for _ in range(args.warmup):
        decode()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        decode()
    dec_s = (time.perf_counter() - t0) / args.steps
    if args.kernel_only:
        return {"kernel_only": True, "ms_per_step": round(dec_s * 1e3, 3)}
    rounds = int(lib.wicca_jpeg_last_sync_rounds())
    verified = None
    if not args.no_verify:  # the first and the last file of the batch
        verified = True
        for i in (0, B - 1):
            got = dev[i * H * pitch:(i + 1) * H * pitch].view(H, pitch)[:, :W * 3].cpu().numpy().reshape(H, W, 3)
            verified &= bool(np.array_equal(got, jpeg_pil.decode_rgb(blobs[i])))
        if not verified:
            raise SystemExit("jpeg bench verification FAILED")
    # a data loader's loop (wicca_jpeg_decode_u8_async): batch k+1 is issued
    # before batch k is waited for, so its host work and PCIe transfer overlap
    # batch k's device decode; two output sets alternate
    dev2 = torch.empty_like(dev)
    sets = [dsts, (ctypes.c_void_p * B)(*[dev2.data_ptr() + i * H * pitch for i in range(B)])]

    def issue(k):
        t = ctypes.c_int64(0)
        _lib.check(lib.wicca_jpeg_decode_u8_async(ptrs, sizes, B, sets[k % 2], pitches, 1, -1, ctypes.byref(t)))
        return t.value

    # warm-up in the same pattern: both workspaces (one per call in flight)
    # get their device and pinned buffers before the timed region
    prev = issue(0)
    for k in range(1, max(2, args.warmup + 1)):
        cur = issue(k)
        _lib.check(lib.wicca_jpeg_wait(prev))
        prev = cur
    _lib.check(lib.wicca_jpeg_wait(prev))
    t0 = time.perf_counter()
    issue_s = 0.0
    prev = issue(0)
    for k in range(1, args.steps):
        ti = time.perf_counter()
        cur = issue(k)
        issue_s += time.perf_counter() - ti
        _lib.check(lib.wicca_jpeg_wait(prev))
        prev = cur
    _lib.check(lib.wicca_jpeg_wait(prev))
    pipe_s = (time.perf_counter() - t0) / args.steps
    issue_ms = issue_s / max(1, args.steps - 1) * 1e3
    if not args.no_verify:
        last = (dev, dev2)[(args.steps - 1) % 2]
        got = last[(B - 1) * H * pitch:B * H * pitch].view(H, pitch)[:, :W * 3].cpu().numpy().reshape(H, W, 3)
        if not np.array_equal(got, jpeg_pil.decode_rgb(blobs[B - 1])):
            raise SystemExit("jpeg bench verification FAILED (pipelined)")
    shape = tuple(int(x) for x in args.shape.split(","))
    res = np.empty((B, shape[1], shape[0], 3), np.uint8)
    ico = np.empty_like(res)

    def stage():
        _lib.check(lib.wicca_jpeg_icon_stage_u8(ptrs, sizes, B, D, 1, 0, shape[0], shape[1],
                                                args.interpolation, res.ctypes.data, ico.ctypes.data, -1, None))

    stage()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        stage()
    stage_s = (time.perf_counter() - t0) / args.steps
    # the same stage in a data loader's loop (wicca_image_icon_stage_async,
    # one batch in flight ahead), two output sets alternating
    outs = [(res, ico), (np.empty_like(res), np.empty_like(ico))]

    def issue_stage(k):
        t = ctypes.c_int64(0)
        r, c = outs[k % 2]
        _lib.check(lib.wicca_image_icon_stage_async(ptrs, sizes, B, D, 1, 0, shape[0], shape[1], args.interpolation,
                                                    r.ctypes.data, c.ctypes.data, -1, ctypes.byref(t)))
        return t.value

    prev = issue_stage(0)
    for k in range(1, max(2, args.warmup + 1)):
        cur = issue_stage(k)
        _lib.check(lib.wicca_image_stage_wait(prev))
        prev = cur
    _lib.check(lib.wicca_image_stage_wait(prev))
    t0 = time.perf_counter()
    prev = issue_stage(0)
    for k in range(1, args.steps):
        cur = issue_stage(k)
        _lib.check(lib.wicca_image_stage_wait(prev))
        prev = cur
    _lib.check(lib.wicca_image_stage_wait(prev))
    stage_pipe_s = (time.perf_counter() - t0) / args.steps
    if not args.no_verify:
        ref_r, ref_c = np.empty_like(res), np.empty_like(ico)
        _lib.check(lib.wicca_jpeg_icon_stage_u8(ptrs, sizes, B, D, 1, 0, shape[0], shape[1], args.interpolation,
                                                ref_r.ctypes.data, ref_c.ctypes.data, -1, None))
        last_r, last_c = outs[(args.steps - 1) % 2]
        if not (np.array_equal(last_r, ref_r) and np.array_equal(last_c, ref_c)):
            raise SystemExit("jpeg bench verification FAILED (pipelined file stage)")
    mpix = B * H * W / 1e6
    # CPU: libjpeg-turbo (Pillow) decode, one thread and a pool over the affinity set
    n1, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 3.0 and n1 < 8:
        jpeg_pil.decode_rgb(blobs[n1 % B], apply_orientation=False)
        n1 += 1
    single = n1 * H * W / 1e6 / (time.perf_counter() - t0)
    threads = min(16, len(os.sched_getaffinity(0)))
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda b: jpeg_pil.decode_rgb(b, False), blobs[:threads]))
        t0 = time.perf_counter()
        list(ex.map(lambda b: jpeg_pil.decode_rgb(b, False), blobs * 2))
        pool = 2 * B * H * W / 1e6 / (time.perf_counter() - t0)
    # per-kernel rooflines: algorithmic bytes per call / rocprofv3 kernel time
    kstats = None if args.no_kernel_trace else kernel_trace_child(
        args, ["--config", "jpeg", "--steps", "3", "--warmup", "1", "--images", str(B), "--height", str(H),
               "--width", str(W), "--quality", str(args.quality)])
    luma, chroma, planes, rgb = jpeg_geometry(H, W)
    stream_b = sum(len(b) for b in blobs)  # entropy-coded bytes, ~ the files
    kernels = kernel_rooflines(kstats, [
        ("jpeg_interleave_kernel", "jpeg_interleave_kernel", 2 * stream_b, "stream read + interleaved copy written"),
        ("jpeg_sync_kernel (guess pass)", "jpeg_sync_kernel<1,", stream_b, "stream read once"),
        ("jpeg_write_kernel", "jpeg_write_kernel", stream_b + B * (luma + chroma),
         "stream read + every coefficient block written once"),
        ("jpeg_idct_kernel (chroma)", "jpeg_idct_kernel", B * (chroma + planes), "chroma blocks read + planes written"),
        ("jpeg_luma_color_kernel", "jpeg_luma_color_kernel", B * (luma + planes + rgb),
         "luma blocks + chroma planes read, RGB written"),
    ])
    dominant = max(kernels, key=lambda e: e["avg_us"], default=None)  # one launch of each per call
    return {
        "metric": "megapixels/sec JPEG decode (load_image) on the GPU", "value": round(mpix / dec_s, 1),
        "unit": "MP/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dec_s * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic scenes encoded by libjpeg-turbo (q{args.quality}, 4:2:0), files in host "
                "memory; decode into device RGB (compressed bytes cross PCIe inside the timed region)",
        "config": {"workload": f"{B} x {W}x{H} JPEG files per call, EXIF orientation applied",
                   "images": B, "mean_file_MB": round(sum(len(b) for b in blobs) / B / 1e6, 2)},
        "sync_rounds": rounds,
        "pipelined": {"ms_per_batch": round(pipe_s * 1e3, 3), "MP_per_s": round(mpix / pipe_s, 1),
                      "host_issue_ms": round(issue_ms, 3),
                      "what": "the same batches through wicca_jpeg_decode_u8_async with one batch in flight "
                              "ahead (host de-stuffing and PCIe of batch k+1 overlap batch k's device decode)"},
        "file_stage": {"ms_per_batch": round(stage_s * 1e3, 3), "MP_per_s": round(mpix / stage_s, 1),
                       "what": f"decode + cv2.resize to {shape} + icon depth {D} + icon resize, "
                               "outputs to host (classifying_tools.py:312-323)"},
        "file_stage_pipelined": {"ms_per_batch": round(stage_pipe_s * 1e3, 3),
                                 "MP_per_s": round(mpix / stage_pipe_s, 1),
                                 "what": "the same stage through wicca_image_icon_stage_async with one batch in "
                                         "flight ahead (get_img_batches)"},
        "cpu_baseline": {"value": round(pool, 1), "unit": "MP/s", "cores": threads, "kind": "reference",
                         "sample": f"Pillow/libjpeg-turbo {jpeg_pil.libjpeg_version()} decode of the same "
                                   f"files, ThreadPoolExecutor({threads}), {2 * B} files",
                         "single_thread_value": round(single, 1)},
        "roofline": ({"bound": "hbm", **{k: dominant[k] for k in ("achieved", "peak", "unit", "frac")},
                      "traffic": None, "kernel": dominant["kernel"], "kernel_us": dominant["avg_us"],
                      "alg_bytes_per_launch": dominant["alg_bytes_per_launch"]} if dominant else None),
        "kernels": kernels or None,
        "kernel_source": "rocprofv3 --kernel-trace child run of this workload (3 calls)" if kernels else None,
        "verified_vs_libjpeg_turbo": verified,
    }


# demo.ipynb's 14 classifiers (their input shapes, classifier[SHAPE]) and depth_range
DEMO_CLASSIFIERS = [(224, 224)] * 9 + [(331, 331)] + [(299, 299)] * 3 + [(240, 240)]


def run_plan(args, torch, rank):
    """The stage plan: the demo's 14 classifiers x 5 depths
    of _get_img_batch over a folder of 8K JPEG files, driven the way
    ClassifierProcessor drives it -- for each depth a pool of 14 classifier
    threads, each walking the folder's batches (classifying_tools.py:546-551,
    414-419, 339-346) -- through wicca_amd.StagePlan with the folder's batches
    known (each batch computed once, in one native call, the next batch
    started while the current one runs).  value = steady-state ms per batch of
    that loop.  Beside it: one synchronous plan call (wicca_image_stage_plan_u8)
    and the per-call file stage run 70 times (the reference's structure).
    Files are distinct and on disk (a temporary directory); outputs are host arrays."""
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor

    from oracle import jpeg_pil
    from wicca_amd import _lib
    from wicca_amd.plan import StagePlan
    lib = _lib.load()
    B = 25 if args.images == 128 else args.images
    H, W = args.height, args.width
    depths = [int(x) for x in args.depths.split(",")] if args.depths != "1,2,3,4,5,6" else [2, 3, 4, 5, 6]
    NB = 1 if args.kernel_only else max(1, args.plan_batches)
    blobs_all = distinct_jpegs(args, NB * B, H, W)
    blobs = blobs_all[:B]
    keep = [np.frombuffer(b, np.uint8) for b in blobs]
    ptrs = (ctypes.c_void_p * B)(*[k.ctypes.data for k in keep])
    sizes = (ctypes.c_int64 * B)(*[k.size for k in keep])
    shapes = list(dict.fromkeys(DEMO_CLASSIFIERS))
    res = [_lib.pinned_empty((B, h, w, 3)) for (w, h) in shapes]  # as get_img_matrix allocates them
    ico = [[_lib.pinned_empty((B, h, w, 3)) for _ in depths] for (w, h) in shapes]
    c_shapes = (ctypes.c_int64 * (2 * len(shapes)))(*[v for sh in shapes for v in sh])
    c_depths = (ctypes.c_int * len(depths))(*depths)
    c_res = (ctypes.c_void_p * len(shapes))(*[r.ctypes.data for r in res])
    c_ico = (ctypes.c_void_p * (len(shapes) * len(depths)))(*[a.ctypes.data for row in ico for a in row])

    def plan():
        _lib.check(lib.wicca_image_stage_plan_u8(ptrs, sizes, B, c_shapes, len(shapes), c_depths, len(depths), 1, 0,
                                                 args.interpolation, c_res, c_ico, -1, None))

    for _ in range(max(1, args.warmup)):
        plan()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan()
    plan_s = (time.perf_counter() - t0) / args.steps
    if args.kernel_only:
        return {"kernel_only": True, "ms_per_step": round(plan_s * 1e3, 3)}

    # the folder on disk, in _classify's batches
    tmp = tempfile.mkdtemp(prefix="wicca_plan_", dir="/tmp")
    try:
        batches = []
        for b in range(NB):
            paths = []
            for i in range(B):
                p = os.path.join(tmp, f"{b:03d}_{i:03d}.jpg")
                with open(p, "wb") as f:
                    f.write(blobs_all[b * B + i])
                paths.append(p)
            batches.append(paths)

        def loop(ahead, copy=True):
            sp = StagePlan(DEMO_CLASSIFIERS, depths, args.interpolation, batches=batches, ahead=ahead, copy=copy)
            done = []  # when each batch's computation finished (s from the loop start)
            compute = sp._compute

            def timed(*a, **kw):
                compute(*a, **kw)
                done.append(time.perf_counter() - t)
            sp._compute = timed

            def classify(shape, d):
                for paths in batches:
                    imgs, icons = sp.get_img_batch(paths, shape, d)
                    assert imgs.shape == (B, shape[1], shape[0], 3) and icons.shape == imgs.shape
            t = time.perf_counter()
            for d in depths:  # process_classifiers: depth by depth, a pool of classifier tasks each
                with ThreadPoolExecutor(max_workers=len(DEMO_CLASSIFIERS)) as ex:
                    list(ex.map(lambda shp: classify(shp, d), DEMO_CLASSIFIERS))
            wall = time.perf_counter() - t
            sp.close()
            done.sort()
            stats = dict(sp.stats)
            stats["first_batch_ms"] = round(done[0] * 1e3, 2) if done else None
            stats["steady_ms_per_batch"] = (round((done[-1] - done[0]) / (len(done) - 1) * 1e3, 3)
                                            if len(done) > 1 else None)
            return wall, stats

        loop(2, copy=False)  # warm: workspaces, the pinned pool, the page cache
        # the timed loop three times, the median reported (the host side --
        # parse, de-stuffing, 14 classifier threads -- varies run to run)
        runs = sorted((loop(2, copy=False) for _ in range(3)), key=lambda r: r[0])
        loop_wall, loop_stats = runs[1]
        loop_stats["runs_ms_per_batch"] = [round(r[0] / NB * 1e3, 3) for r in runs]
        loop_stats["runs_steady_ms_per_batch"] = [r[1].get("steady_ms_per_batch") for r in runs]
        serial_wall, _ = loop(0, copy=False)
        copy_wall, _ = loop(2, copy=True)
        # the plan's outputs for batch 0 through the StagePlan path against the per-call stage
        sp = StagePlan(DEMO_CLASSIFIERS, depths, args.interpolation)
        got0 = {(sh, d): sp.get_img_batch(batches[0], sh, d) for sh in shapes for d in depths}
        sp.close()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    pc = {sh: (np.empty((B, sh[1], sh[0], 3), np.uint8), np.empty((B, sh[1], sh[0], 3), np.uint8))
          for sh in shapes}

    def per_call(sh, d):
        r, c = pc[sh]
        _lib.check(lib.wicca_image_icon_stage_u8(ptrs, sizes, B, d, 1, 0, sh[0], sh[1], args.interpolation,
                                                 r.ctypes.data, c.ctypes.data, -1, None))

    loop_s = float("nan")
    if not args.plan_no_loop:
        per_call(shapes[0], depths[0])
        t0 = time.perf_counter()
        for d in depths:
            for sh in DEMO_CLASSIFIERS:
                per_call(sh, d)
        loop_s = time.perf_counter() - t0
    verified = None
    if not args.no_verify:
        verified = True
        for si, sh in enumerate(shapes):
            for di, d in enumerate(depths):
                per_call(sh, d)
                r, c = pc[sh]
                verified &= bool(np.array_equal(res[si], r) and np.array_equal(ico[si][di], c))
                verified &= bool(np.array_equal(got0[(sh, d)][0], r) and np.array_equal(got0[(sh, d)][1], c))
        if not verified:
            raise SystemExit("plan bench verification FAILED")
    pairs = len(DEMO_CLASSIFIERS) * len(depths)
    mpix = B * H * W / 1e6
    per_batch = loop_wall / NB
    # per-kernel rooflines of one plan call (rocprofv3 kernel trace of a child run)
    kstats = None if args.no_kernel_trace else kernel_trace_child(
        args, ["--config", "plan", "--steps", "3", "--warmup", "1", "--images", str(B), "--height", str(H),
               "--width", str(W), "--quality", str(args.quality), "--plan-no-loop", "--depths",
               ",".join(map(str, depths))])
    img_b = B * H * W * 3
    icon_b = sum(B * -(-H >> d) * -(-W >> d) * 3 for d in depths)
    out_src_b = sum(B * w * h * 3 for (w, h) in shapes)
    # the icon planes the area kernel's icon launch reads (INTER_AREA downscales
    # in both dimensions to some shape) and the icon resizes it writes
    area_icons = [(d, sh) for d in depths for sh in shapes
                  if sh[0] <= -(-W >> d) and sh[1] <= -(-H >> d)]
    icon_read_b = sum(B * -(-H >> d) * -(-W >> d) * 3 for d in sorted({d for d, _ in area_icons}))
    icon_out_b = sum(B * w * h * 3 for _, (w, h) in area_icons)
    kernels = kernel_rooflines(kstats, [
        ("haar_multi_ragged_kernel (icons, every depth)", "haar_multi_ragged_kernel", img_b + icon_b,
         "decoded images read once + every depth's icons written"),
        ("plan_area_wave_kernel (INTER_AREA resizes: icon launch + source launch)", "plan_area",
         img_b + out_src_b + icon_read_b + icon_out_b,
         "decoded images and the downscaled depths' icons read once, every area resize written", 2),
    ])
    dominant = max(kernels, key=lambda e: e["avg_us"], default=None)
    cpu = None if args.no_cpu_baseline else plan_cpu_baseline(args, blobs, shapes, depths)
    return {
        "metric": "ms per batch for the demo's 14 classifiers x depths of _get_img_batch (stage plan)",
        "value": round(per_batch * 1e3, 3), "unit": "ms", "n_gpus": 1, "steps": NB, "warmup": 1,
        "ms_per_step": round(per_batch * 1e3, 3), "higher_is_better": False, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": f"{NB * B} distinct synthetic 8K scenes encoded by libjpeg-turbo (q{args.quality}, 4:2:0), "
                "files on disk (page cache); every output lands in host memory inside the timed region",
        "config": {"workload": f"{NB} batches x {B} x {W}x{H} JPEG files, shapes {shapes} (14 classifiers), "
                               f"depths {depths}; StagePlan(batches=...) under ClassifierProcessor's loop "
                               "(per depth a pool of 14 classifier threads walking the batches)",
                   "images": B, "batches": NB, "classifiers": len(DEMO_CLASSIFIERS), "depths": depths,
                   "pairs": pairs},
        "loop_stats": loop_stats,
        "steady_ms_per_batch": loop_stats.get("steady_ms_per_batch"),
        "steady_what": "(last batch computed - first batch computed) / (batches - 1) in the timed loop: "
                       "the pipeline's rate without its fill; value is the whole loop / batches (median of "
                       "three timed loops, all three in loop_stats)",
        "outputs": "StagePlan(copy=False): every classifier of a (shape, depth) gets the batch's one cached "
                   "pair of arrays, read-only",
        "no_overlap": {"ms_per_batch": round(serial_wall / NB * 1e3, 3),
                       "what": "the same loop with StagePlan(ahead=0): each batch computed only when requested"},
        "private_copies": {"ms_per_batch": round(copy_wall / NB * 1e3, 3),
                           "what": "the same loop with StagePlan(copy=True): every request gets its own writable "
                                   "copy, as np.stack gives (~665 MB of host memcpy per batch)"},
        "single_call": {"ms_per_batch": round(plan_s * 1e3, 3), "decoded_MP_per_s": round(mpix / plan_s, 1),
                        "what": "one synchronous wicca_image_stage_plan_u8 call on one batch (files in memory)"},
        "per_call_loop": {"ms_per_batch": round(loop_s * 1e3, 3) if loop_s == loop_s else None,
                          "what": f"wicca_image_icon_stage_u8 once per (classifier, depth): {pairs} calls, "
                                  "each decoding, resizing and iconing the whole batch (the reference's structure)"},
        "speedup_vs_per_call": round(loop_s / per_batch, 2) if loop_s == loop_s else None,
        "verified_vs_per_call": verified,
        "roofline": ({"bound": "hbm", **{k: dominant[k] for k in ("achieved", "peak", "unit", "frac")},
                      "traffic": None, "kernel": dominant["kernel"], "kernel_us": dominant["avg_us"],
                      "alg_bytes_per_launch": dominant["alg_bytes_per_launch"]} if dominant else None),
        "kernels": kernels or None,
        "kernel_source": "rocprofv3 --kernel-trace child run of one plan call x 3" if kernels else None,
        "cpu_baseline": cpu,
    }


def plan_cpu_baseline(args, blobs, shapes, depths):
    """The reference's per-batch CPU cost, sampled: for one file, libjpeg-turbo's
    decode (Pillow: the library cv2.imread wraps), the INTER_AREA source resize
    per classifier shape and the icon resize per (shape, depth) by
    oracle/area_cpu.c (OpenCV's resize.cpp area tables and arithmetic order in
    C at -O3, byte-identical to oracle/resize_cv.py -- cv2 itself is absent; the
    icon upscales of the deep depths, OpenCV's bilinear path, through the NumPy
    restatement: small images), and the Haar icon per depth by the NumPy port
    (the reference's HaarCoder is NumPy); extrapolated to the reference's
    structure, which recomputes the whole chain for every file, classifier and
    depth (classifying_tools.py:312-323 under :339-346, :414-419, :546-551)."""
    from oracle import c_oracle, haar_numpy, jpeg_pil
    from oracle import resize_cv as R
    B = len(blobs)

    def area(img, sh):
        out = c_oracle.area_resize(img, sh) if args.interpolation == R.INTER_AREA else None
        return out if out is not None else R.resize(img, sh, args.interpolation)
    t = time.perf_counter()
    img = jpeg_pil.decode_rgb(blobs[0])
    t_dec = time.perf_counter() - t
    t_src, t_ico = {}, {}
    icons = {}
    for sh in shapes:
        t = time.perf_counter()
        out = area(img, sh)
        t_src[sh] = time.perf_counter() - t
        if sh == shapes[0] and not np.array_equal(out, R.resize(img, sh, args.interpolation)):
            raise SystemExit("plan cpu baseline: compiled INTER_AREA differs from resize_cv")
    t_haar = {}
    for d in depths:
        t = time.perf_counter()
        icons[d] = haar_numpy.get_small_copy(img, d)
        t_haar[d] = time.perf_counter() - t
    for sh in shapes:
        for d in depths:
            t = time.perf_counter()
            area(icons[d], sh)
            t_ico[(sh, d)] = time.perf_counter() - t
    per_file = sum(t_dec + t_src[sh] + t_haar[d] + t_ico[(sh, d)] for sh in DEMO_CLASSIFIERS for d in depths)
    sampled = t_dec + sum(t_src.values()) + sum(t_haar.values()) + sum(t_ico.values())
    return {"value": round(per_file * B * 1e3, 1), "unit": "ms", "cores": 1, "kind": "port",
            "sample": f"one {img.shape[1]}x{img.shape[0]} file: Pillow decode {t_dec * 1e3:.0f} ms, INTER_AREA "
                      f"source resizes in C (oracle/area_cpu.c, -O3, checked against resize_cv on this file) "
                      f"{sum(t_src.values()) * 1e3:.0f} ms for {len(shapes)} shapes, haar_numpy "
                      f"{sum(t_haar.values()) * 1e3:.0f} ms for {len(depths)} depths, icon resizes "
                      f"{sum(t_ico.values()) * 1e3:.0f} ms ({sampled:.2f} s sampled); extrapolated to {B} files x "
                      f"{len(DEMO_CLASSIFIERS)} classifiers x {len(depths)} depths, single thread",
            "per_file_ms": round(per_file * 1e3, 1),
            "per_file_parts_ms": {"decode": round(t_dec * 1e3, 1),
                                  "source_resize": {f"{w}x{h}": round(v * 1e3, 1) for (w, h), v in t_src.items()},
                                  "haar": {str(d): round(v * 1e3, 1) for d, v in t_haar.items()},
                                  "icon_resizes": round(sum(t_ico.values()) * 1e3, 1)}}


def run_raster(args, torch, rank):
    """load_image for PNG / BMP files (data_loader.py:53; ClassifierProcessor
    counts .png / .bmp, classifying_tools.py:162): B files of the configs[2]
    size decoded in one wicca_image_decode_u8 call into device RGB (PNG:
    inflate + row reconstruction on host threads, pixel conversion on the
    device; BMP: rows copied, converted on the device), then the file-based
    caller stage.  The CPU baseline is Pillow's decoder of the same files
    (zlib + its own unfilter for PNG, as libpng under cv2.imread)."""
    import io
    from concurrent.futures import ThreadPoolExecutor

    from PIL import Image

    from oracle import jpeg_pil
    from wicca_amd import _lib
    lib = _lib.load()
    fmt = args.config
    B = 25 if args.images == 128 else args.images
    H, W, D = args.height, args.width, args.depth
    srcs = [jpeg_pil.test_image("scene", H, W, 40 + k) for k in range(4)]
    distinct = []
    for img in srcs:
        b = io.BytesIO()
        Image.fromarray(img).save(b, "PNG" if fmt == "png" else "BMP")
        distinct.append(b.getvalue())
    blobs = [distinct[i % 4] for i in range(B)]
    keep = [np.frombuffer(b, np.uint8) for b in blobs]
    ptrs = (ctypes.c_void_p * B)(*[k.ctypes.data for k in keep])
    sizes = (ctypes.c_int64 * B)(*[k.size for k in keep])
    pitch = (W * 3 + 127) // 128 * 128
    dev = torch.empty(B * H * pitch, dtype=torch.uint8, device="cuda")
    dsts = (ctypes.c_void_p * B)(*[dev.data_ptr() + i * H * pitch for i in range(B)])
    pitches = (ctypes.c_int64 * B)(*([pitch] * B))
    stream = torch.cuda.Stream()
    sh = ctypes.c_void_p(stream.cuda_stream)

    def decode():
        _lib.check(lib.wicca_image_decode_u8(ptrs, sizes, B, dsts, pitches, 1, 1, -1, sh, None))
        stream.synchronize()

    steps = max(1, args.steps // 4) if fmt == "png" else args.steps  # PNG calls take ~0.5 s
    for _ in range(min(args.warmup, 1) if fmt == "png" else args.warmup):
        decode()
    t0 = time.perf_counter()
    for _ in range(steps):
        decode()
    dec_s = (time.perf_counter() - t0) / steps
    verified = None
    if not args.no_verify:
        for i in range(min(B, 4)):
            got = dev[i * H * pitch:(i + 1) * H * pitch].view(H, pitch)[:, :W * 3].cpu().numpy().reshape(H, W, 3)
            verified = bool(np.array_equal(got, srcs[i])) and verified is not False
        if not verified:
            raise SystemExit(f"{fmt} bench verification FAILED")
    shape = tuple(int(x) for x in args.shape.split(","))
    res = np.empty((B, shape[1], shape[0], 3), np.uint8)
    ico = np.empty_like(res)

    def stage():
        _lib.check(lib.wicca_image_icon_stage_u8(ptrs, sizes, B, D, 1, 0, shape[0], shape[1],
                                                 args.interpolation, res.ctypes.data, ico.ctypes.data, -1, None))

    stage()
    t0 = time.perf_counter()
    for _ in range(steps):
        stage()
    stage_s = (time.perf_counter() - t0) / steps
    # a loader loop: wicca_image_icon_stage_async with one batch in flight ahead
    # (a PNG / BMP batch's stage runs on a host thread of its own)
    outs = [(res, ico), (np.empty_like(res), np.empty_like(ico))]

    def issue_stage(k):
        t = ctypes.c_int64(0)
        r, c = outs[k % 2]
        _lib.check(lib.wicca_image_icon_stage_async(ptrs, sizes, B, D, 1, 0, shape[0], shape[1], args.interpolation,
                                                    r.ctypes.data, c.ctypes.data, -1, ctypes.byref(t)))
        return t.value

    pipe_steps = max(2, steps)
    t0 = time.perf_counter()
    prev = issue_stage(0)
    for k in range(1, pipe_steps):
        cur = issue_stage(k)
        _lib.check(lib.wicca_image_stage_wait(prev))
        prev = cur
    _lib.check(lib.wicca_image_stage_wait(prev))
    stage_pipe_s = (time.perf_counter() - t0) / pipe_steps
    mpix = B * H * W / 1e6

    def pil(b):
        im = Image.open(io.BytesIO(b))
        return np.asarray(im.convert("RGB"))

    n1, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 3.0 and n1 < 8:
        pil(blobs[n1 % 4])
        n1 += 1
    single = n1 * H * W / 1e6 / (time.perf_counter() - t0)
    threads = min(16, len(os.sched_getaffinity(0)))
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(pil, blobs[:threads]))
        t0 = time.perf_counter()
        list(ex.map(pil, blobs))
        pool = B * H * W / 1e6 / (time.perf_counter() - t0)
    import PIL
    return {
        "metric": f"megapixels/sec {fmt.upper()} decode (load_image) into device RGB", "value": round(mpix / dec_s, 1),
        "unit": "MP/s", "n_gpus": 1, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(dec_s * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic scenes written by Pillow {PIL.__version__} "
                f"({'PNG, zlib level 6, adaptive filters' if fmt == 'png' else '24-bit BMP'}), files in host "
                "memory; decoded into device RGB (decoded rows cross PCIe inside the timed region)",
        "config": {"workload": f"{B} x {W}x{H} {fmt.upper()} files per call", "images": B,
                   "mean_file_MB": round(sum(len(b) for b in blobs) / B / 1e6, 2)},
        "file_stage": {"ms_per_batch": round(stage_s * 1e3, 3), "MP_per_s": round(mpix / stage_s, 1),
                       "what": f"decode + cv2.resize to {shape} + icon depth {D} + icon resize, "
                               "outputs to host (classifying_tools.py:312-323)"},
        "file_stage_pipelined": {"ms_per_batch": round(stage_pipe_s * 1e3, 3),
                                 "MP_per_s": round(mpix / stage_pipe_s, 1),
                                 "what": "the same stage through wicca_image_icon_stage_async, one batch in "
                                         "flight ahead (the next batch's host inflate overlaps)"},
        "cpu_baseline": {"value": round(pool, 1), "unit": "MP/s", "cores": threads, "kind": "port",
                         "sample": f"Pillow {PIL.__version__} decode + convert('RGB') of the same files, "
                                   f"ThreadPoolExecutor({threads}), {B} files",
                         "single_thread_value": round(single, 1)},
        "roofline": None, "verified_vs_source_pixels": verified,
    }


def run_multi(args, torch, rank):
    """All depths of configs[2]'s sweep from ONE read of the batch
    (wicca_haar_ll_u8_multi_uniform), against one launch per depth."""
    from wicca_amd import _lib
    lib = _lib.load()
    B, H, W, C = args.images, args.height, args.width, args.channels
    depths = [int(x) for x in args.depths.split(",")]
    pitch = (W * C + 15) // 16 * 16
    src = torch.empty(B * H * pitch, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sh = ctypes.c_void_p(stream.cuda_stream)
    _lib.check(lib.wicca_synth_u8(ctypes.c_void_p(src.data_ptr()), B, H, W, C, pitch, H * pitch,
                                  args.seed * 1000003 + rank, -1, sh))
    outs, ptrs, pitches, strides, dims = [], [], [], [], []
    for d in depths:
        oh, ow = -(-H >> d), -(-W >> d)
        op = (ow * C + 15) // 16 * 16
        o = torch.empty(B * oh * op, dtype=torch.uint8, device="cuda")
        outs.append(o)
        ptrs.append(o.data_ptr())
        pitches.append(op)
        strides.append(oh * op)
        dims.append((oh, ow))
    nd = len(depths)
    c_d = (ctypes.c_int * nd)(*depths)
    c_p = (ctypes.c_void_p * nd)(*ptrs)
    c_pi = (ctypes.c_int64 * nd)(*pitches)
    c_s = (ctypes.c_int64 * nd)(*strides)

    def multi():
        _lib.check(lib.wicca_haar_ll_u8_multi_uniform(
            ctypes.c_void_p(src.data_ptr()), B, H, W, C, pitch, H * pitch, c_d, nd, args.border,
            0, c_p, c_pi, c_s, -1, sh))

    def separate():
        for i, d in enumerate(depths):
            _lib.check(lib.wicca_haar_ll_u8_uniform(
                ctypes.c_void_p(src.data_ptr()), B, H, W, C, pitch, H * pitch, d, args.border, 0,
                ctypes.c_void_p(ptrs[i]), pitches[i], strides[i], -1, sh))

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3, e0.elapsed_time(e1) / args.steps

    sep_wall, sep_dev = timed(separate)
    sep_icons = [o.clone() for o in outs]
    multi_wall, multi_dev = timed(multi)
    same = all(torch.equal(a, b) for a, b in zip(sep_icons, outs))
    if not same and not args.no_verify:  # --no-verify: timing-only experiment builds
        raise SystemExit("multi-depth icons differ from per-depth icons")
    mp = B * H * W / 1e6
    in_bytes = B * H * W * C
    return {
        "metric": BASELINE["metric"],
        "value": round(mp / (multi_wall / 1e3), 1), "unit": "MP/s (all depths per pixel)",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(multi_wall, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (on-device splitmix64 images, HBM-resident before timing)",
        "config": {"workload": f"{B} x {W}x{H}x{C}, icons at depths {depths} per step "
                               "(BASELINE configs[2] sweep) from one read",
                   "depths": depths, "images_per_gpu": B},
        "separate_depths_ms": round(sep_wall, 4),
        "speedup_vs_separate": round(sep_wall / multi_wall, 3),
        "input_read_GBps_equiv": round(in_bytes / (multi_dev / 1e3) / 1e9, 1),
        "identical_to_separate": same,
    }


def spawn_ranks(n: int) -> int:
    """``bench.py --gpus N`` without a launcher: start N ranks (one per GPU)
    through ``torch.distributed.run`` as a CHILD process and return its exit
    code.  This parent never touches the GPU (no torch import, no HIP call)
    and never execs, so the children initialise the devices themselves."""
    import socket
    import subprocess
    with socket.socket() as s:  # a free rendezvous port on the loopback
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch "
                         "one rank per GPU (or pass --gpus N alone and bench.py starts them)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:  # launcher check only (tests/test_bench_launch.py): no GPU, no torch
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world}), flush=True)
        return

    import torch
    # one rank per GPU; the modulo only matters for a rehearsal with more ranks
    # than GPUs (WICCA_BENCH_BACKEND=gloo), never for the driver's runs
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("WICCA_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()

    from wicca_amd import _lib
    lib = _lib.load()
    if _lib.device_count() < 1:
        raise SystemExit("no HIP device visible")
    if args.config == "multi":
        out = run_multi(args, torch, rank)
        if rank == 0:
            print(json.dumps(out), flush=True)
        return
    if args.config == "jpeg":
        out = run_jpeg(args, torch, rank)
        if rank == 0:
            print(json.dumps(out), flush=True)
        return
    if args.config == "plan":
        out = run_plan(args, torch, rank)
        if rank == 0:
            print(json.dumps(out), flush=True)
        return
    if args.config in ("png", "bmp"):
        out = run_raster(args, torch, rank)
        if rank == 0:
            print(json.dumps(out), flush=True)
        return
    if args.config == "stage":
        out = run_stage(args, torch, rank)
        if rank == 0:
            print(json.dumps(out), flush=True)
        return
    if args.config == "ragged":
        out = run_ragged(args, torch, rank)
        if rank == 0:
            print(json.dumps(out), flush=True)
        return
    if args.config == "tiled":
        out = run_tiled(args, torch, dist, world, rank, local_rank)
        if out is not None:
            print(json.dumps(out), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    B, H, W, C, D = args.images, args.height, args.width, args.channels, args.depth
    pitch = (W * C + 15) // 16 * 16
    r = 1 << D
    oh, ow = -(-H // r), -(-W // r)
    opitch = (ow * C + 15) // 16 * 16
    src = torch.empty(B * H * pitch, dtype=torch.uint8, device="cuda")
    dst = torch.empty(B * oh * opitch, dtype=torch.uint8, device="cuda")
    # a dedicated (non-null) stream: the C ABI launches on it and the HIP
    # events below are recorded on the same stream
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sh = ctypes.c_void_p(stream.cuda_stream)
    assert sh.value, "expected a non-null HIP stream"
    # device-resident synthetic batch; rank r owns images [r*B, (r+1)*B)
    _lib.check(lib.wicca_synth_u8(ctypes.c_void_p(src.data_ptr()), B, H, W, C, pitch, H * pitch,
                                  args.seed * 1000003 + rank, -1, sh))

    def step():
        _lib.check(lib.wicca_haar_ll_u8_uniform(
            ctypes.c_void_p(src.data_ptr()), B, H, W, C, pitch, H * pitch, D, args.border, 0,
            ctypes.c_void_p(dst.data_ptr()), opitch, oh * opitch, -1, sh))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    barrier()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # one kernel launch per step

    if dist is not None:
        t = torch.tensor([wall, kernel_ms], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, kernel_ms = float(t[0]), float(t[1])

    # every rank checks its own last image (REPLICATE and CONSTANT k = 77)
    # against the NumPy port outside the timed region; the pass/fail flags are
    # reduced over ranks, so an N-rank line says verified only if all N passed
    verified = None
    checked = []
    if not args.no_verify:
        from oracle import haar_numpy
        from wicca_amd.synth import synth_image
        ok = True
        # the first, a middle and the last image of the rank's batch (REPLICATE)
        for i in sorted({0, B // 2, B - 1}):
            img = synth_image(args.seed * 1000003 + rank, i, H, W, C)
            ref = haar_numpy.get_small_copy(img, D, args.border)
            got = dst.view(B, oh, opitch)[i, :, :ow * C].cpu().numpy().reshape(oh, ow, C)
            ok = ok and bool(np.array_equal(got, ref))
            checked.append(i)
        one = torch.empty(oh * opitch, dtype=torch.uint8, device="cuda")
        _lib.check(lib.wicca_haar_ll_u8_uniform(
            ctypes.c_void_p(src.data_ptr() + i * H * pitch), 1, H, W, C, pitch, H * pitch, D, 0, 77,
            ctypes.c_void_p(one.data_ptr()), opitch, oh * opitch, -1, sh))
        got_k = one.view(oh, opitch)[:, :ow * C].cpu().numpy().reshape(oh, ow, C)
        ok = ok and bool(np.array_equal(got_k, haar_numpy.get_small_copy(img, D, 0, 77)))
        n_ok = 1 if ok else 0
        if dist is not None:
            t = torch.tensor([n_ok], dtype=torch.int64,
                             device="cuda" if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            n_ok = int(t[0])
        verified = n_ok == world
        if not verified:
            raise SystemExit(f"bench verification FAILED on {world - n_ok} of {world} ranks: "
                             "icon differs from the NumPy port")

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    ms_per_step = wall / args.steps * 1e3
    mpix = world * B * H * W / 1e6
    value = mpix / (ms_per_step / 1e3)
    alg_bytes = B * (H * W * C + oh * ow * C)  # per launch: u8 read once + u8 icon write
    achieved = alg_bytes / (kernel_ms / 1e3) / 1e9
    workload_key = f"b{B}_{W}x{H}x{C}_d{D}"
    kernel = lib.wicca_kernel_name(D, C, 0).decode()
    # live HBM bytes: rank 0 (every rank runs the same per-GPU workload) starts
    # two single-process PMC child runs on its own device after the timed
    # region and the verification; the committed summary is only the fallback
    sweep = None
    if world == 1 and not args.no_sweep:
        sweep = run_sweep(args, torch, lib, src, B, H, W, C, pitch, stream, sh, args.seed * 1000003 + rank)
    del src, dst
    torch.cuda.empty_cache()
    # this run's rocprofv3 kernel trace of the same workload (a child run):
    # the launch durations beside the HIP-event ones
    trace = None
    if world == 1 and not args.no_kernel_trace:
        trace = kernel_trace_grid(args, ["--steps", "5", "--warmup", "1", "--images", str(B), "--height", str(H),
                                         "--width", str(W), "--channels", str(C), "--depth", str(D),
                                         "--border", str(args.border), "--seed", str(args.seed)]
                                  + (["--no-sweep"] if sweep is None else []))
    if sweep is not None:
        for e in sweep:
            hit = trace_lookup(trace, e["kernel"], -1 if e["config"] == "configs[1]" else 0)
            e["rocprof_avg_us"] = round(hit[1], 1) if hit else None
    pmc = live_pmc(args, kernel) if not args.no_live_pmc else None
    pmc_source = ("live (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child runs of this per-GPU workload"
                  + (" on rank 0's device)" if world > 1 else ")")) if pmc else None
    if pmc is None:
        pmc = read_pmc(args.pmc, workload_key)
        pmc_source = f"committed summary {os.path.relpath(args.pmc, REPO)} (not this run)" if pmc else None
    traffic = round(pmc["hbm_bytes_per_launch"]) if pmc else None

    out = {
        "metric": BASELINE["metric"],
        "value": round(value, 1),
        "unit": "MP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (on-device splitmix64 images, HBM-resident before timing)",
        "config": {
            "workload": f"{B} x {W}x{H}x{C} uint8 images per GPU, Haar LL depth {D}, "
                        f"{'REPLICATE' if args.border == 1 else 'CONSTANT'} border "
                        "(BASELINE.json configs[2] at the metric's depth)",
            "images_per_gpu": B, "height": H, "width": W, "channels": C, "depth": D,
            "parallelism": f"image-parallel x{world} (no collectives)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": kernel,
            "kernel_ms": round(kernel_ms, 4),
            "alg_bytes_per_launch": alg_bytes,
            "pmc_source": pmc_source,
            "rocprof_avg_us": None,
            "rocprof_launches": None,
        },
        "sweep": sweep,
        "cpu_baseline": None,
        "verified_vs_numpy_port": verified,
        "verified_ranks": world if verified else None,
        "verified_images_per_rank": checked if verified else None,
    }
    hit = trace_lookup(trace, kernel, 0)
    if hit:
        out["roofline"]["rocprof_launches"], out["roofline"]["rocprof_avg_us"] = hit[0], round(hit[1], 1)
        out["roofline"]["rocprof_source"] = ("rocprofv3 --kernel-trace child run of this workload "
                                             "(5 timed steps + the sweep's launches)")
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
