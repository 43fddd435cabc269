"""What the asynchronous host mirror of a device checkpoint costs the training step it overlaps.

One world-1 robust engine per setting of rabit_device_mirror_ctas (0 = hipMemcpyAsync, whose
D2H blit kernel puts a workgroup on every CU; N = the narrow copy kernel with N workgroups).
Per setting, medians over reps of:
  gemm_us      20 bf16 8192^3 matmuls alone (the "training step")
  mirror_us    checkpoint_tensors of a 256 MiB model until the device is idle (snapshot + D2H)
  overlap_us   checkpoint, then the 20 matmuls; until the caller's stream is done
  overlap_all  the same, until the device is idle (mirror included)

    python tools/mirror_probe.py            # all settings, one subprocess each
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(ctas, prio="normal", engine=None, mirror="always", reps=5):
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    import rabit_amd as rabit
    from rabit_amd.tracker import RabitTracker

    tr = RabitTracker("127.0.0.1", 1, port=9391, port_end=9491, print_fn=lambda m: None).start(1)
    rabit.init(rabit_tracker_uri="127.0.0.1", rabit_tracker_port=tr.port, rabit_task_id=0,
               rabit_world_size=1, rabit_world1_fastpath=0, rabit_device=0,
               rabit_device_ckpt_mirror=mirror, rabit_device_mirror_ctas=ctas,
               rabit_device_mirror_priority=prio,
               **({"rabit_device_mirror_engine": engine} if engine else {}))
    model = torch.rand((256 << 20) // 4, device="cuda")
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    c = torch.empty_like(a)

    def gemms():
        for _ in range(20):
            torch.matmul(a, b, out=c)

    gemms()
    rabit.checkpoint_tensors({"w": model}, meta=0)
    torch.cuda.synchronize()
    out = {"gemm_us": [], "mirror_us": [], "overlap_us": [], "overlap_all_us": []}
    for i in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gemms()
        torch.cuda.synchronize()
        out["gemm_us"].append(time.perf_counter() - t0)
        time.sleep(0.02)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rabit.checkpoint_tensors({"w": model}, meta=i)
        torch.cuda.synchronize()
        out["mirror_us"].append(time.perf_counter() - t0)
        time.sleep(0.02)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rabit.checkpoint_tensors({"w": model}, meta=i)
        gemms()
        torch.cuda.current_stream().synchronize()
        out["overlap_us"].append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        out["overlap_all_us"].append(time.perf_counter() - t0)
    res = {k: round(float(np.median(v)) * 1e6, 1) for k, v in out.items()}
    res["mirror_ctas"] = ctas
    res["priority"] = prio
    res["engine"] = engine or ("kernel" if ctas > 0 else "hip")
    res["mirror"] = mirror
    res["hsa_enable_sdma"] = os.environ.get("HSA_ENABLE_SDMA")
    res["stats_mirrors"] = rabit.stats().get("ckpt_mirrors")
    res["stats_engine"] = rabit.stats().get("ckpt_mirror_engine")
    print("MIRROR " + json.dumps(res), flush=True)
    rabit.finalize()
    tr.join(10)


def main():
    if len(sys.argv) > 1:
        one(int(sys.argv[1]), sys.argv[2] if len(sys.argv) > 2 else "normal",
            sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != "-" else None,
            sys.argv[4] if len(sys.argv) > 4 else "always")
        return
    # "N", "N:sdma" (HSA_ENABLE_SDMA=1 for that run: the runtime may move the D2H copy to a
    # DMA engine instead of a blit kernel), "N:low" (mirror stream of the lowest priority) or
    # "0:engine=sdma" (rabit_device_mirror_engine); ":off" takes no mirror at all (baseline)
    settings = os.environ.get("MIRROR_SETTINGS", "0,4,8,16,32,64").split(",")
    for setting in settings:
        ctas = int(setting.split(":")[0])
        env = dict(os.environ)
        if setting.endswith(":sdma"):
            env["HSA_ENABLE_SDMA"] = "1"
        prio = "low" if setting.endswith(":low") else "normal"
        engine = setting.split("engine=")[1].split(":")[0] if "engine=" in setting else "-"
        mirror = "off" if setting.endswith(":off") else "always"
        r = subprocess.run([sys.executable, __file__, str(ctas), prio, engine, mirror],
                           capture_output=True, text=True, timeout=300, env=env)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("MIRROR ")]
        if r.returncode != 0 or not lines:
            print("ctas=%d failed rc=%d\n%s" % (ctas, r.returncode, r.stderr[-2000:]), flush=True)
            sys.exit(1)
        print(lines[0], flush=True)


if __name__ == "__main__":
    main()
