"""bench.py's run-time guards (CPU): the deadline watcher names the phase and exits non-zero
before the headline exists; once the headline is measured, a stuck side measurement still ends
the run with exactly one JSON line on rank 0 (flagged) and exit status 0."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(body, timeout=60):
    code = "import sys, time; sys.path.insert(0, %r); import bench\n%s" % (ROOT, body)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=timeout)


def test_deadline_before_headline_fails():
    p = _run("bench.phase('timed')\nbench.start_deadline(1, 0, 100)\ntime.sleep(30)")
    assert p.returncode == 3
    assert "phase 'timed'" in p.stderr
    assert p.stdout.strip() == ""


def test_stuck_side_measurement_still_prints_headline():
    p = _run("bench.start_deadline(100, 0, 1)\n"
             "bench.HEADLINE.update(rec={'metric': 'm', 'value': 1.0}, t=time.time())\n"
             "bench.phase('variant direct-push-fused/torch')\ntime.sleep(30)")
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["value"] == 1.0
    assert "direct-push-fused" in rec["post_headline_failure"]


def test_headline_printed_once_and_only_on_rank0():
    p = _run("bench.start_deadline(100, 0, 2)\n"
             "bench.HEADLINE.update(rec={'metric': 'm', 'value': 2.0}, t=time.time())\n"
             "bench.emit_headline()\nbench.phase('finalize')\ntime.sleep(30)")
    assert p.returncode == 0
    assert len([ln for ln in p.stdout.splitlines() if ln.startswith("{")]) == 1
    p = _run("bench.start_deadline(100, 1, 1)\n"
             "bench.HEADLINE.update(rec={'metric': 'm'}, t=time.time(), rank=1)\ntime.sleep(30)")
    assert p.returncode == 0
    assert p.stdout.strip() == ""


def test_headline_value_is_busbw_above_one_rank():
    """BASELINE.json's metric is the allreduce bus bandwidth: `value` is busbw at N > 1 (the
    whole-job aggregate is a separate field); at N = 1 busbw is 0 by definition and `value` is
    the algbw, labelled as such"""
    import importlib
    sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    size = 128 << 20
    for n in (2, 4, 8):
        bw = bench.bandwidths(n, size, 1e-3)
        assert bw["value"] == bw["busbw_GBps"] and bw["value_is"] == "busbw_GBps"
        assert abs(bw["busbw_GBps"] - bw["algbw_GBps"] * 2 * (n - 1) / n) < 0.02
        assert abs(bw["aggregate_GBps"] - n * bw["algbw_GBps"]) < 0.05 * n
    one = bench.bandwidths(1, size, 1e-3)
    assert one["busbw_GBps"] == 0.0 and one["value"] == one["algbw_GBps"]
    assert one["value_is"].startswith("algbw")


def test_ft_tax_fields_cpu():
    """measure_ft_tax's arithmetic on a stand-in engine (CPU): ft_tax = robust step - base op,
    dual-store and host-wait costs relative to the base op, times max over ranks"""
    import importlib
    import types
    import numpy as np
    sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    clock = {"t": 0.0}
    cost = {0: 100e-6, 1: 130e-6, 2: 90e-6}
    rabit = types.SimpleNamespace(PROBE_BASE=0, PROBE_DUAL_STORE=1, PROBE_NO_WAIT=2, SUM=2, MAX=0)

    def probe(x, op, mode):
        clock["t"] += cost[mode]
    rabit.probe_allreduce = probe
    rabit.allreduce = lambda a, op: np.asarray(a)
    torch = types.SimpleNamespace(cuda=types.SimpleNamespace(synchronize=lambda: None))
    real = bench.time.perf_counter
    bench.time.perf_counter = lambda: clock["t"]
    try:
        ft = bench.measure_ft_tax(rabit, torch, None, 10, 150e-6)
    finally:
        bench.time.perf_counter = real
    assert ft["base_us"] == 100.0 and ft["dual_store_us"] == 130.0 and ft["no_host_wait_us"] == 90.0
    assert ft["ft_tax_us"] == 50.0 and abs(ft["ft_tax_pct"] - 33.3) < 0.1
    assert ft["dual_store_cost_us"] == 30.0 and ft["host_wait_cost_us"] == 10.0


def test_bench_torchrun_busbw_and_config5():
    """GPU: bench.py under torch.distributed.run with 2 ranks sharing the box's GPU (the direct
    transport carries the data): the headline `value` is the busbw, and the extras carry
    BASELINE config 5 (256 MiB sum + checkpoint every iteration, and its overhead)"""
    import pytest
    pytest.importorskip("torch")
    import socket
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                          "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--steps", "3", "--warmup", "1", "--variants", "0"],
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["collective"] is True
    assert rec["value"] == rec["busbw_GBps"] > 0 and rec["value_is"] == "busbw_GBps", rec
    assert rec["sum_tdiff_speed_MiBps"] > 0 and rec["aggregate_GBps"] > rec["value"]
    assert "post_headline_failure" not in rec, rec["post_headline_failure"]
    ex = rec["extras"]
    assert ex["config5_iter_us"] > 0 and ex["config5_sum_only_iter_us"] > 0, ex
    assert "config5_ckpt_overhead_us" in ex, ex
    # the fault-tolerance tax of the headline op and the reference speed_test's whole line
    ft = ex["ft_tax"]
    assert "error" not in ft, ft
    for k in ("base_us", "dual_store_us", "no_host_wait_us", "robust_us", "ft_tax_us",
              "ft_tax_pct", "dual_store_cost_us", "host_wait_cost_us"):
        assert k in ft, (k, ft)
    assert ft["base_us"] > 0 and ft["robust_us"] > 0, ft
    st = ex["speed_test"]
    for k in ("max_tdiff", "sum_tdiff", "bcast_tdiff"):
        assert st[k]["speed_MiBps"] > 0 and st[k]["mean_s"] > 0, st
    assert st["tot_tdiff"]["mean_s"] > 0, st


test_bench_torchrun_busbw_and_config5.pytestmark = [__import__("pytest").mark.gpu]
