"""Where BASELINE config 5's iteration time goes at N ranks (torchrun launch, bench.py's init).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/config5_probe.py

Phases, each rank in lock step (device synchronised + host allreduce) before every timed rep,
median over reps, max over ranks, in microseconds:
  sum_clean      256 MiB robust allreduce before any checkpoint of this size
  ckpt_iter      allreduce + model update + checkpoint_tensors (caller's stream only)
  sum_after      the allreduce alone again, after the checkpoints (mirrors drained first)
  sum_after_log  the same with the result log cleared first (checkpoint(None))
Rank 0 prints one JSON line; XR_ENV lists extra rabit_* parameters (a=b,c=d).
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import rabit_amd as rabit
    from rabit_amd.torchrun import init_from_env

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = local_rank % torch.cuda.device_count()
    torch.cuda.set_device(gpu)
    extra = dict(kv.split("=", 1) for kv in os.environ.get("XR_ENV", "").split(",") if "=" in kv)
    ctx = init_from_env(lib="standard", rabit_world1_fastpath=0, rabit_device=gpu, **extra)
    dev = torch.device("cuda", gpu)
    reps = int(os.environ.get("XR_REPS", "5"))
    n = (256 << 20) // 4
    grad = torch.rand(n, device=dev).mul_(1e-3)
    model = torch.zeros(n, device=dev)

    def timed(fn, device_wide=True):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
            t0 = time.perf_counter()
            fn()
            if device_wide:
                torch.cuda.synchronize()
            else:
                torch.cuda.current_stream().synchronize()
            ts.append(time.perf_counter() - t0)
        per_rep = [round(t * 1e6, 1) for t in ts]
        med = float(rabit.allreduce(np.array([float(np.median(ts))]), rabit.MAX)[0])
        return round(med * 1e6, 1), per_rep

    it = [0]

    def step(ckpt):
        rabit.allreduce(grad, rabit.SUM)
        model.add_(grad, alpha=-1e-3)
        if ckpt:
            it[0] += 1
            rabit.checkpoint_tensors({"w": model}, meta={"it": it[0]})

    out = {"world": rabit.get_world_size()}
    rabit.allreduce(grad, rabit.SUM)
    out["sum_clean"] = timed(lambda: step(False))
    step(True)
    out["ckpt_iter"] = timed(lambda: step(True), device_wide=False)
    out["ckpt_iter_drained"] = timed(lambda: step(True))
    out["sum_after"] = timed(lambda: step(False))
    rabit.checkpoint(None)
    out["sum_after_log"] = timed(lambda: step(False))
    st = rabit.stats()
    out["stats"] = {k: st.get(k) for k in ("device_direct", "device_rccl", "n_checkpoint",
                                           "mirrors", "mirrors_deferred", "log_reserved_bytes",
                                           "log_spilled_bytes")}
    if rabit.get_rank() == 0:
        print(json.dumps(out), flush=True)
    ctx.finalize()


if __name__ == "__main__":
    main()
