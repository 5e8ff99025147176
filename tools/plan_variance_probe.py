"""Run-to-run variance of the StagePlan loop (diagnostic, GPU box): the plan
bench's folder of distinct 8K JPEG batches and its ClassifierProcessor-shaped
loop (ahead 2, copy=False), repeated; per loop the steady rate and, per batch,
when its issue started / ended (host read, parse, de-stuffing, uploads queued)
and when its wait returned (device work and output copies done), relative to
the loop start.  A slow loop then shows whether one batch stalled or every
batch slowed, and in which phase.
Usage: python tools/plan_variance_probe.py [loops] [batches] [aheads, e.g. 2,3]"""
import argparse
import os
import shutil
import sys
import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def cgroup_stat():
    """(nr_throttled, throttled_usec) of this process's cgroup (v2 cpu.stat; v1 cpu.stat), or None."""
    for path in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            with open(path) as f:
                kv = dict(line.split() for line in f if len(line.split()) == 2)
            thr = int(kv.get("throttled_usec", int(kv.get("throttled_time", 0)) // 1000))
            return int(kv.get("nr_throttled", 0)), thr
        except (OSError, ValueError):
            continue
    return None


def cpu_quota():
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f, open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as g:
            return f.read().strip() + " " + g.read().strip()
    except OSError:
        return "unknown"


def main():
    import resource

    import bench
    from wicca_amd import plan as P
    loops = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    aheads = [int(a) for a in (sys.argv[3] if len(sys.argv) > 3 else "2").split(",")]
    args = argparse.Namespace(quality=90)
    B, H, W = 25, 4320, 7680
    depths = [2, 3, 4, 5, 6]
    blobs = bench.distinct_jpegs(args, nb * B, H, W)
    tmp = tempfile.mkdtemp(prefix="wicca_var_", dir="/tmp")
    lock = threading.Lock()
    log = []
    orig_async = P.get_img_matrix_async

    def timed_async(*a, **kw):
        t1 = time.perf_counter()
        call = orig_async(*a, **kw)
        call._probe_t = (t1, time.perf_counter())  # plain attributes: no reference cycle keeps the outputs alive
        return call
    orig_wait = P.MatrixCall.wait

    def timed_wait(self):
        r = orig_wait(self)
        t = getattr(self, "_probe_t", None)
        if t is not None:
            with lock:
                log.append((t[0], t[1], time.perf_counter(), threading.get_ident()))
        return r
    P.get_img_matrix_async = timed_async
    P.MatrixCall.wait = timed_wait
    reads = []
    orig_read = P._read

    def timed_read(*a, **kw):
        t1 = time.perf_counter()
        r = orig_read(*a, **kw)
        with lock:
            reads.append(time.perf_counter() - t1)
        return r
    P._read = timed_read
    try:
        batches = []
        for b in range(nb):
            paths = []
            for i in range(B):
                p = os.path.join(tmp, f"{b:03d}_{i:03d}.jpg")
                with open(p, "wb") as f:
                    f.write(blobs[b * B + i])
                paths.append(p)
            batches.append(paths)
        print(f"cgroup cpu quota: {cpu_quota()}; affinity {len(os.sched_getaffinity(0))} CPUs", flush=True)
        for rep in range(loops * len(aheads) + 1):
            ahead = aheads[(rep - 1) % len(aheads)] if rep else aheads[0]
            log.clear()
            reads.clear()
            st0 = cgroup_stat()
            ru0 = resource.getrusage(resource.RUSAGE_SELF)
            sp = P.StagePlan(bench.DEMO_CLASSIFIERS, depths, batches=batches, ahead=ahead, copy=False)
            t0 = time.perf_counter()
            for d in depths:
                def classify(shape):
                    for paths in batches:
                        sp.get_img_batch(paths, shape, d)
                with ThreadPoolExecutor(len(bench.DEMO_CLASSIFIERS)) as ex:
                    list(ex.map(classify, bench.DEMO_CLASSIFIERS))
            wall = time.perf_counter() - t0
            ru1 = resource.getrusage(resource.RUSAGE_SELF)
            st1 = cgroup_stat()
            sp.close()
            cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
            thr = (f"throttled {st1[0] - st0[0]} times, {(st1[1] - st0[1]) / 1e3:.1f} ms" if st0 and st1 else "no cpu.stat")
            ev = sorted((a - t0, b - t0, c - t0) for a, b, c, _ in log)
            done = sorted(c for _, _, c in ev)
            steady = (done[-1] - done[0]) / (len(done) - 1) if len(done) > 1 else 0.0
            tag = "warm" if rep == 0 else f"loop {rep} ahead {ahead}"
            print(f"{tag}: {1e3 * wall / nb:.2f} ms per batch, steady {1e3 * steady:.2f}; CPU {cpu_s / wall:.1f} cores; "
                  f"{thr}; "
                  f"issue ms {' '.join(f'{1e3 * (b - a):.1f}' for a, b, _ in ev)}; "
                  f"of which file reads ms {' '.join(f'{1e3 * r:.1f}' for r in reads)}; "
                  f"done gaps ms {' '.join(f'{1e3 * (y - x):.1f}' for x, y in zip(done, done[1:]))}", flush=True)
    finally:
        P.get_img_matrix_async = orig_async
        P.MatrixCall.wait = orig_wait
        P._read = orig_read
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
