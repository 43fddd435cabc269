#!/usr/bin/env python3
"""Bandwidth of the gfx950 data-plane kernels vs the HBM roof and vs PyTorch equivalents.

Interleaved rounds in one process (A/B noise), random data, 128 MiB per operand by default.
Bytes counted are the minimum each op must move: reduce2 3S, copy 2S, multi-k (k+1)S,
prepare-dual 3S, checksum S.  Prints one JSON line per kernel.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from rabit_amd import ops  # noqa: E402

HBM_SPEC_TBPS = 8.0  # MI355X HBM3E spec; the achievable peak is measured in each run (below)


def timeit(fn, reps, inner):
    """median / best GPU time of one call.  Each sample brackets `inner` back-to-back calls with
    events: the host enqueues faster than the GPU drains them, so the per-call host overhead of
    the Python / ctypes wrappers (which would otherwise sit between the start event and the
    kernel) is hidden, for the rabit and the torch calls alike."""
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        start.record()
        for _ in range(inner):
            fn()
        end.record()
        end.synchronize()
        times.append(start.elapsed_time(end) * 1e-3 / inner)
    times.sort()
    return times[len(times) // 2], times[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--inner", type=int, default=10, help="calls per timed sample")
    ap.add_argument("--only", default="", help="comma-separated substrings of kernel names")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = args.mb * (1 << 20) // 4
    S = n * 4
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.rand(n, generator=g, device=dev)
    b = torch.rand(n, generator=g, device=dev)
    out = torch.empty_like(a)
    out2 = torch.empty_like(a)
    srcs = [torch.rand(n // 4, generator=g, device=dev) for _ in range(8)]
    out_small = torch.empty(n // 4, device=dev)
    ai = torch.randint(0, 1 << 30, (n,), generator=g, device=dev, dtype=torch.int32)
    bi = torch.randint(0, 1 << 30, (n,), generator=g, device=dev, dtype=torch.int32)
    # bf16 operands of the same byte size (fp32 accumulation inside the kernels)
    ah = torch.rand(2 * n, generator=g, device=dev).to(torch.bfloat16)
    bh = torch.rand(2 * n, generator=g, device=dev).to(torch.bfloat16)
    srcs_h = [torch.rand(n // 2, generator=g, device=dev).to(torch.bfloat16) for _ in range(8)]
    out_small_h = torch.empty(n // 2, device=dev, dtype=torch.bfloat16)
    sums = torch.zeros(2, dtype=torch.int64, device=dev)
    cases = {
        "rabit_reduce_sum_f32": (lambda: ops.reduce_(a, b, ops.SUM), 3 * S),
        "torch_add_f32": (lambda: a.add_(b), 3 * S),
        "rabit_reduce_max_f32": (lambda: ops.reduce_(a, b, ops.MAX), 3 * S),
        "rabit_reduce_bitor_i32": (lambda: ops.reduce_(ai, bi, ops.BITOR), 3 * S),
        "torch_bitwise_or_i32": (lambda: ai.bitwise_or_(bi), 3 * S),
        "rabit_copy": (lambda: ops.copy(out, a), 2 * S),
        "rabit_prepare_copy": (lambda: ops.prepare(out, a, ops.PREP_COPY), 2 * S),
        "torch_copy": (lambda: out.copy_(a), 2 * S),
        "rabit_prepare_square_dual": (lambda: ops.prepare(out, a, ops.PREP_SQUARE, dst2=out2), 3 * S),
        "torch_square_two_outputs": (lambda: (torch.mul(a, a, out=out), out2.copy_(out)), 4 * S),
        "rabit_multi8_sum_f32": (lambda: ops.reduce_multi(out_small, srcs, ops.SUM), 9 * S // 4),
        "torch_stack_sum8_f32": (lambda: torch.sum(torch.stack(srcs), dim=0, out=out_small),
                                 9 * S // 4),
        "rabit_checksum": (lambda: ops.checksum(a, out=sums), S),
        "torch_sum_f32": (lambda: torch.sum(a), S),
        "rabit_reduce_sum_bf16": (lambda: ops.reduce_(ah, bh, ops.SUM), 3 * S),
        "torch_add_bf16": (lambda: ah.add_(bh), 3 * S),
        "rabit_multi8_sum_bf16": (lambda: ops.reduce_multi(out_small_h, srcs_h, ops.SUM), 9 * S // 4),
        "torch_stack_sum8_bf16": (lambda: torch.sum(torch.stack(srcs_h), dim=0, out=out_small_h),
                                  9 * S // 4),
    }
    if args.only:
        keys = args.only.split(",")
        cases = {k: v for k, v in cases.items() if any(q in k for q in keys)}
    results = {k: [] for k in cases}
    for _ in range(args.rounds):
        for name, (fn, nbytes) in cases.items():
            med, best = timeit(fn, args.reps, args.inner)
            results[name].append((med, best, nbytes))
    rows = []
    for name, vals in results.items():
        med = sorted(v[0] for v in vals)[len(vals) // 2]
        best = min(v[1] for v in vals)
        nbytes = vals[0][2]
        rows.append((name, med, best, nbytes))
    # the roof every percentage refers to: the best median bandwidth any streaming case (ours or
    # torch's) reached in this run, so no figure can exceed 100 %; the 8 TB/s spec alongside
    peak = max(nb / med for _, med, _, nb in rows)
    for name, med, best, nbytes in rows:
        rec = {"kernel": name, "mib_per_operand": args.mb, "inner": args.inner,
               "median_us": round(med * 1e6, 1),
               "best_us": round(best * 1e6, 1), "GBps": round(nbytes / med / 1e9, 1),
               "pct_of_measured_peak": round(100 * nbytes / med / peak, 1),
               "measured_peak_GBps": round(peak / 1e9, 1),
               "pct_of_hbm_spec": round(100 * nbytes / med / 1e12 / HBM_SPEC_TBPS, 1)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
