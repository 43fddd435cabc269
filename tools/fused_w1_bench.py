"""Fused vs classic direct two-shot allreduce at world 1 (VERDICT r2 "what's next" #2).

One rank, one GPU, no contention: world-1 device ops are routed through a one-peer direct group
(rabit_device_world1_transport=1), so every kernel of the direct path runs (stage copy, flag
barriers, reduce, gather — or the single fused launch) with nothing else on the GPU.  This
separates the fused kernel's own cost from the CU sharing of ranks that share one GPU.

    python tools/fused_w1_bench.py [--sizes 1M,4M,16M,128M] [--reps 20] [--forms classic,fused]

Prints one JSON line per (form, size): median / min op time in us, and the classic form's
per-phase hipEvent times.  Run it under rocprofv3 --kernel-trace for the kernel view.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_size(s):
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    if s[-1] in mult:
        return int(float(s[:-1]) * mult[s[-1]])
    return int(s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1M,4M,16M,128M")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--forms", default="classic,fused")
    ap.add_argument("--port", type=int, default=9391)
    ap.add_argument("params", nargs="*", help="extra rabit name=value parameters")
    args = ap.parse_args()

    import torch

    import rabit_amd as rabit
    from rabit_amd.tracker import RabitTracker

    tracker = RabitTracker("127.0.0.1", 1, port=args.port, print_fn=lambda m: None).start(1)
    rabit.init(args.params, lib="base", rabit_tracker_uri="127.0.0.1",
               rabit_tracker_port=tracker.port, rabit_task_id=0, rabit_world_size=1,
               rabit_world1_fastpath=0, rabit_device_world1_transport=1,
               rabit_device_algo="direct", rabit_device=0)
    dev = torch.device("cuda", 0)
    sizes = [parse_size(s) for s in args.sizes.split(",")]
    rabit.allreduce(torch.ones(1024, device=dev), rabit.SUM)  # brings the direct group up
    for form in args.forms.split(","):
        fused = form == "fused"
        assert rabit.set_device_transport(rabit.TRANSPORT_DIRECT, fused=fused), "no direct group"
        for nbytes in sizes:
            x = torch.arange(nbytes // 4, device=dev, dtype=torch.float32).remainder_(1000)
            want = x.clone()
            for _ in range(3):
                rabit.allreduce(x, rabit.SUM)
            torch.cuda.synchronize()
            assert torch.equal(x, want), (form, nbytes)
            before = rabit.stats()
            times = []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rabit.allreduce(x, rabit.SUM)
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t0)
            st = rabit.stats()
            if not fused:
                # per-phase hipEvent times in a separate pass (the events cost time themselves)
                rabit.set_phase_timing(True)
                for _ in range(5):
                    rabit.allreduce(x, rabit.SUM)
                torch.cuda.synchronize()
                st = dict(st, direct_phase_us=rabit.stats().get("direct_phase_us"))
                rabit.set_phase_timing(False)
            times.sort()
            rec = {"form": form, "bytes": nbytes, "median_us": round(times[len(times) // 2] * 1e6, 1),
                   "min_us": round(times[0] * 1e6, 1), "reps": args.reps,
                   "fused_chunks": st["fused_chunks"] - before["fused_chunks"],
                   "fused_grid": st["fused_grid"], "result_ok": bool(torch.equal(x, want))}
            if not fused and st.get("direct_phase_us"):
                rec["phase_us"] = {k: round(v, 1) for k, v in st["direct_phase_us"].items()}
            print(json.dumps(rec), flush=True)
    rabit.finalize()
    tracker.join(30)


if __name__ == "__main__":
    main()
