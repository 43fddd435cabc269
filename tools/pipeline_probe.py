"""A few 128 MiB robust allreduces on one direct form, for kernel traces (one rocprofv3 per rank,
torchrun-style environment as tools/prof_world2.sh sets it).

    RANK=0 LOCAL_RANK=0 WORLD_SIZE=2 ... python tools/pipeline_probe.py pipelined

Rank 0 prints one JSON line: median op time over the ranks' slowest (us) and the form's stats."""
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

    mode = sys.argv[1] if len(sys.argv) > 1 else "pipelined"
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = local_rank % torch.cuda.device_count()
    torch.cuda.set_device(gpu)
    ctx = init_from_env(lib="standard", rabit_device=gpu, rabit_device_direct_mode=mode,
                        rabit_device_fused=0)
    dev = torch.device("cuda", gpu)
    x = torch.full(((128 << 20) // 4,), float(rabit.get_rank() + 1), device=dev)
    rabit.allreduce(x, rabit.SUM)
    ts = []
    for _ in range(5):
        x.fill_(float(rabit.get_rank() + 1))
        torch.cuda.synchronize()
        rabit.allreduce(np.zeros(1, dtype=np.int32), rabit.SUM)
        t0 = time.perf_counter()
        rabit.allreduce(x, rabit.SUM)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    world = rabit.get_world_size()
    assert bool((x == world * (world + 1) / 2).all().item()), float(x[0])
    med = float(rabit.allreduce(np.array([float(np.median(ts))]), rabit.MAX)[0])
    st = rabit.stats()
    if rabit.get_rank() == 0:
        print(json.dumps({"mode": mode, "world": world, "t_us": round(med * 1e6, 1),
                          "pipelined_ops": st.get("pipelined_ops"),
                          "pipelined_rounds": st.get("pipelined_rounds"),
                          "push_chunks": st.get("push_chunks")}), flush=True)
    ctx.finalize()


if __name__ == "__main__":
    main()
