"""examples/dp_train.py: fault-tolerant data-parallel MLP training.  A worker killed in the
middle of a step resumes from the last checkpoint and replays the missed gradient allreduces;
the final weights are bit-identical to the run without failures (CPU ranks here; the GPU
variant with HBM buckets and device checkpoints is in test_gpu_models.py)."""
import os
import re
import sys


from rabit_amd.launcher import LocalJob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "examples", "dp_train.py")


def run_dp_train(n, attempts, extra, env=None):
    job = LocalJob([sys.executable, SCRIPT, "--steps", "12", "lib=mock"] + list(extra), n,
                   attempts, capture=True, timeout=240, print_fn=lambda m: None, env=env)
    rc = job.run()
    out = "".join("".join(o) for o in job.outputs)
    assert rc == 0, out[-4000:]
    digests = set(re.findall(r"DPTRAIN OK weights=([0-9a-f]+)", out))
    assert len(digests) == 1 and out.count("DPTRAIN OK") == n, out[-3000:]
    return digests.pop(), job, out


def test_dp_train_failure_is_invisible(native_build):
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    clean, _, _ = run_dp_train(3, 1, [], env=env)
    failed, job, out = run_dp_train(3, 3, ["mock=1,2,1,0", "mock=2,3,0,0"], env=env)
    assert sum(a - 1 for a in job.attempts) >= 2, "kill points did not fire"
    assert "resumed at version" in out
    assert failed == clean
