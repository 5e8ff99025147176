#!/usr/bin/env python3
"""In-process A/B of libwicca_hip.so variants (interleaved rounds, same data, one device).

    python tools/ab.py --libs tools/variants/lib_a.so tools/variants/lib_b.so \
        --depths 1 3 5 --rounds 5

Every variant is loaded with its own ctypes handle (RTLD_LOCAL), so each keeps
its own kernels; all share one HIP runtime and one synthetic batch.  Reports the
median and min over rounds of achieved GB/s (algorithmic bytes / kernel time).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--depths", nargs="+", type=int, default=[5])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--images", type=int, default=128)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--border", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--ragged", type=float, default=0.0,
                    help="> 0: a ragged batch, H, W drawn from [ragged * size, size], one "
                         "wicca_haar_ll_u8_batch call with device descriptors")
    ap.add_argument("--ragged-align", type=int, default=16, help="row pitch alignment (bytes)")
    ap.add_argument("--ragged-wmult", type=int, default=1,
                    help="round ragged widths down to a multiple of this many pixels")
    ap.add_argument("--ragged-hmult", type=int, default=1,
                    help="round ragged heights down to a multiple of this many rows")
    ap.add_argument("--multi", default="",
                    help="comma-separated depth list: time wicca_haar_ll_u8_multi_uniform (K5) "
                         "instead of single depths (uniform batch)")
    ap.add_argument("--pitch-pad", type=int, default=0,
                    help="uniform batch: bytes added to the 16-B aligned row pitch")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the identical-icons check (ablation builds compute garbage)")
    args = ap.parse_args()

    import torch
    from wicca_amd import _lib as L
    L.load()  # preload the shared runtime + bind the default library
    libs = {}
    for path in args.libs:
        h = ctypes.CDLL(os.path.abspath(path))
        for name, (res, argt) in L.SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, argt
        libs[os.path.basename(path)] = h

    B, H, W, C = args.images, args.height, args.width, args.channels
    import numpy as np
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sh = ctypes.c_void_p(stream.cuda_stream)
    first = next(iter(libs.values()))
    if args.ragged > 0:
        rng = np.random.default_rng(0)
        Hs = [int(x) // args.ragged_hmult * args.ragged_hmult
              for x in rng.integers(int(H * args.ragged), H + 1, B)]
        Ws = [int(x) // args.ragged_wmult * args.ragged_wmult
              for x in rng.integers(int(W * args.ragged), W + 1, B)]
        al = args.ragged_align
        pitches = [(w * C + al - 1) // al * al for w in Ws]
    else:
        Hs, Ws = [H] * B, [W] * B
        pitches = [(W * C + 15) // 16 * 16 + args.pitch_pad] * B
    offs = np.concatenate([[0], np.cumsum([p * h for p, h in zip(pitches, Hs)])]).astype(np.int64)
    src = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda")
    for i in range(B):
        if args.ragged > 0 or i == 0:
            n_i = 1 if args.ragged > 0 else B
            assert first.wicca_synth_u8(ctypes.c_void_p(src.data_ptr() + int(offs[i])), n_i, Hs[i],
                                        Ws[i], C, pitches[i], Hs[i] * pitches[i], i, -1, sh) == 0
    pitch = pitches[0]
    results = []
    if args.multi:
        ds = [int(x) for x in args.multi.split(",")]
        outs, c_p, c_pi, c_s = [], [], [], []
        alg = B * H * W * C
        for d in ds:
            oh, ow = -(-H // (1 << d)), -(-W // (1 << d))
            op = (ow * C + 15) // 16 * 16
            outs.append(torch.empty(B * oh * op, dtype=torch.uint8, device="cuda"))
            c_p.append(outs[-1].data_ptr())
            c_pi.append(op)
            c_s.append(oh * op)
            alg += B * oh * ow * C
        arr_d = (ctypes.c_int * len(ds))(*ds)
        arr_p = (ctypes.c_void_p * len(ds))(*c_p)
        arr_pi = (ctypes.c_int64 * len(ds))(*c_pi)
        arr_s = (ctypes.c_int64 * len(ds))(*c_s)
        samples = {k: [] for k in libs}
        for rnd in range(args.rounds):
            for name, h in libs.items():
                def mstep():
                    rc = h.wicca_haar_ll_u8_multi_uniform(
                        ctypes.c_void_p(src.data_ptr()), B, H, W, C, pitch, H * pitch, arr_d, len(ds),
                        args.border, 0, arr_p, arr_pi, arr_s, -1, sh)
                    assert rc == 0, rc
                for _ in range(2):
                    mstep()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.steps):
                    mstep()
                e1.record(stream)
                e1.synchronize()
                samples[name].append(alg / (e0.elapsed_time(e1) / args.steps / 1e3) / 1e9)
        for name, v in samples.items():
            row = {"lib": name, "depths": ds, "median_gbs": round(statistics.median(v), 1),
                   "min_gbs": round(min(v), 1), "max_gbs": round(max(v), 1), "rounds": len(v)}
            results.append(row)
            print(json.dumps(row), flush=True)
        args.depths = []
    for D in args.depths:
        r = 1 << D
        oh, ow = -(-H // r), -(-W // r)
        align = int(os.environ.get("WICCA_AB_OPITCH_ALIGN", "16"))  # icon row pitch alignment
        opitch = (ow * C + align - 1) // align * align
        dst = torch.empty(B * oh * opitch, dtype=torch.uint8, device="cuda")
        alg = sum(h * w * C + (-(-h // r)) * (-(-w // r)) * C for h, w in zip(Hs, Ws))
        descs = (L.ImageDesc * B)()
        for i in range(B):
            descs[i] = L.ImageDesc(src.data_ptr() + int(offs[i]), dst.data_ptr() + i * oh * opitch,
                                   Hs[i], Ws[i], pitches[i], opitch)
        ref = None
        samples = {k: [] for k in libs}
        for rnd in range(args.rounds):
            for name, h in libs.items():
                def step():
                    if args.ragged > 0:
                        rc = h.wicca_haar_ll_u8_batch(descs, B, C, D, args.border, 0, 1, 1, -1, sh)
                        assert rc == 0, rc
                        return
                    rc = h.wicca_haar_ll_u8_uniform(
                        ctypes.c_void_p(src.data_ptr()), B, H, W, C, pitch, H * pitch, D,
                        args.border, 0, ctypes.c_void_p(dst.data_ptr()), opitch, oh * opitch,
                        -1, sh)
                    assert rc == 0, rc
                for _ in range(2):
                    step()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.steps):
                    step()
                e1.record(stream)
                e1.synchronize()
                ms = e0.elapsed_time(e1) / args.steps
                samples[name].append(alg / (ms / 1e3) / 1e9)
                if rnd == 0 and not args.no_check:  # variants must produce identical icons
                    got = dst.clone()
                    if ref is None:
                        ref = got
                    elif not torch.equal(ref, got):
                        raise SystemExit(f"{name}: icons differ from {next(iter(libs))} at D={D}")
        for name, v in samples.items():
            row = {"lib": name, "depth": D, "median_gbs": round(statistics.median(v), 1),
                   "min_gbs": round(min(v), 1), "max_gbs": round(max(v), 1), "rounds": len(v)}
            results.append(row)
            print(json.dumps(row), flush=True)
        del dst
    if args.out:
        with open(args.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
