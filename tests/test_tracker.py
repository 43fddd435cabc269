"""Tracker topology and launcher behaviour."""
import os
import re
import subprocess
import sys

import pytest

from rabit_amd.launcher import LocalJob
from rabit_amd.tracker import link_map, tree_neighbours

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 7, 8, 10, 16, 31, 64])
def test_link_map_invariants(n):
    tree, parent, ring = link_map(n)
    assert sorted(tree) == list(range(n))
    # ring is relabelled to rank order
    for r in range(n):
        assert ring[r] == ((r - 1) % n, (r + 1) % n)
    # the tree is symmetric, connected, with one root
    roots = [r for r in range(n) if parent[r] == -1]
    assert roots == [0]
    for r in range(n):
        for q in tree[r]:
            assert r in tree[q]
        if parent[r] != -1:
            assert parent[r] in tree[r]
    edges = sum(len(v) for v in tree.values()) // 2
    assert edges == n - 1
    seen, stack = {0}, [0]
    while stack:
        for q in tree[stack.pop()]:
            if q not in seen:
                seen.add(q)
                stack.append(q)
    assert len(seen) == n


def test_ring_mostly_follows_tree():
    # the DFS ring should reuse tree edges (short hops) for most ring steps
    tree, _, ring = link_map(15)
    shared = sum(1 for r in range(15) if ring[r][1] in tree[r])
    assert shared >= 8


def test_heap_neighbours():
    assert tree_neighbours(0, 5) == [1, 2]
    assert tree_neighbours(1, 5) == [0, 3, 4]
    assert tree_neighbours(4, 5) == [1]


def test_launcher_restarts_failing_worker(tmp_path):
    flag = tmp_path / "died"
    script = tmp_path / "w.py"
    script.write_text(
        "import os, sys\n"
        "t = int(os.environ['DMLC_TASK_ID']); a = int(os.environ['DMLC_NUM_ATTEMPT'])\n"
        "sys.path.insert(0, %r)\n"
        "import rabit_amd as rabit\n"
        "if t == 1 and a == 0:\n"
        "    open(%r, 'w').write('x'); sys.exit(3)\n"
        "rabit.init(); rabit.finalize()\n" % (ROOT, str(flag)))
    job = LocalJob([sys.executable, str(script)], 2, 3, timeout=60, print_fn=lambda m: None)
    assert job.run() == 0
    assert flag.exists() and job.attempts == [1, 2]


def test_launcher_restarts_on_reported_exit(tmp_path):
    """a worker that reports its exit code on the launcher's exit pipe is replaced at once, while
    it is still tearing down (here: sleeping 3 s before it really exits)"""
    script = tmp_path / "w.py"
    script.write_text(
        "import os, sys, time\n"
        "t = int(os.environ['DMLC_TASK_ID']); a = int(os.environ['DMLC_NUM_ATTEMPT'])\n"
        "if t == 1 and a == 0:\n"
        "    fd = int(os.environ['XRABIT_EXIT_FD'].split(':')[0])\n"
        "    open(%r, 'w').write(repr(time.time()))\n"
        "    os.write(fd, b'7\\n'); time.sleep(3); sys.exit(7)\n"
        "if t == 1:\n"
        "    open(%r, 'w').write(repr(time.time()))\n"
        % (str(tmp_path / "died"), str(tmp_path / "again")))
    job = LocalJob([sys.executable, str(script)], 2, 3, timeout=60, print_fn=lambda m: None)
    job.tracker.start = lambda n: None  # no rabit.init in this worker: no tracker needed
    job.tracker.join = lambda t: None
    assert job.run() == 0
    died = float((tmp_path / "died").read_text())
    again = float((tmp_path / "again").read_text())
    assert again - died < 2.0, again - died
    assert job.attempts == [1, 2] and job.reported_exits == [[], [7]]


def test_mock_kill_reports_exit_code(tmp_path):
    """the native mock kill shuts its sockets and reports its code on the exit pipe
    (csrc/src/core/exit.h) before it _Exits; the job still ends with the exact result"""
    script = tmp_path / "w.py"
    script.write_text(
        "import sys\n"
        "sys.path.insert(0, %r)\n"
        "import numpy as np\n"
        "import rabit_amd as rabit\n"
        "rabit.init(sys.argv[1:], lib='mock')\n"
        "v, _ = rabit.load_checkpoint()\n"
        "x = rabit.allreduce(np.ones(4) * (rabit.get_rank() + 1), rabit.SUM)\n"
        "assert x[0] == 3, x\n"
        "rabit.finalize()\n" % ROOT)
    job = LocalJob([sys.executable, str(script), "mock=1,0,0,0"], 2, 3, timeout=60,
                   print_fn=lambda m: None)
    assert job.run() == 0
    assert job.reported_exits == [[], [254]] and job.attempts == [1, 2]


def test_launcher_cli_basic_example(native_build):
    out = subprocess.run([sys.executable, "-m", "rabit_amd.launcher", "-n", "3", "--",
                          os.path.join(native_build, "basic")], capture_output=True, text=True,
                         timeout=60, cwd=ROOT)
    assert out.returncode == 0, out.stderr
    # Max then Sum of a[i] = rank + i over 3 ranks (doc/guide.md semantics)
    assert out.stdout.count("after-allreduce-max: a={2, 3, 4}") == 3
    assert out.stdout.count("after-allreduce-sum: a={6, 9, 12}") == 3


def test_examples_broadcast_and_lazy(native_build):
    out = subprocess.run([sys.executable, "-m", "rabit_amd.launcher", "-n", "2", "--",
                          os.path.join(native_build, "broadcast")], capture_output=True,
                         text=True, timeout=60, cwd=ROOT)
    assert out.returncode == 0 and out.stdout.count('after-broadcast: s="hello world"') == 2
    out = subprocess.run([sys.executable, "-m", "rabit_amd.launcher", "-n", "2", "--",
                          os.path.join(native_build, "lazy_allreduce")], capture_output=True,
                         text=True, timeout=60, cwd=ROOT)
    assert out.returncode == 0
    assert out.stdout.count("run prepare function") == 2
    assert out.stdout.count("after-allreduce-sum: a={2, 4, 6}") == 2


def test_cpp_unit_tests(native_build):
    out = subprocess.run([os.path.join(native_build, "unit_tests")], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert " 0 failed" in out.stdout


def test_speed_test_cpu(native_build):
    out = subprocess.run([sys.executable, "-m", "rabit_amd.launcher", "-n", "4", "--",
                          os.path.join(native_build, "speed_test"), "100000", "5"],
                         capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode == 0, out.stderr
    assert "sum_tdiff-speed" in out.stdout and "bcast_tdiff-speed" in out.stdout


def test_launcher_ssh_cluster(tmp_path):
    """--cluster ssh: workers placed host by host (consecutive ranks share a node), started
    through the ssh command with an explicit environment (the stand-in gives them a clean one),
    LOCAL_RANK / LOCAL_WORLD_SIZE per node, and a killed worker restarted on its host."""
    from rabit_amd.launcher import SSHJob, parse_host_file, place_workers

    hf = tmp_path / "hosts"
    hf.write_text("# test cluster\nnodeA:2\nnodeB slots=3\n")
    hosts = parse_host_file(str(hf))
    assert hosts == [("nodeA", 2), ("nodeB", 3)]
    assert place_workers(hosts, 4) == [("nodeA", 0, 2), ("nodeA", 1, 2), ("nodeB", 0, 2),
                                       ("nodeB", 1, 2)]
    with pytest.raises(ValueError):
        place_workers(hosts, 6)
    fake = os.path.join(ROOT, "tests", "scripts", "fake_ssh.sh")
    worker = os.path.join(ROOT, "tests", "scripts", "ssh_worker.py")
    flag = tmp_path / "killed"
    # task 3 dies once before rabit.init (a lost node process); the launcher restarts it
    cmd = [sys.executable, "-c",
           "import os, sys, runpy\n"
           "if os.environ['DMLC_TASK_ID'] == '3' and not os.path.exists(%r):\n"
           "    open(%r, 'w').write('x'); sys.exit(7)\n"
           "sys.argv = [%r]; runpy.run_path(%r, run_name='__main__')\n"
           % (str(flag), str(flag), worker, worker)]
    job = SSHJob(cmd, hosts, 4, num_attempt=2, host_ip="127.0.0.1", tracker_port=9391,
                 timeout=120, capture=True, print_fn=lambda m: None, ssh=[fake, "-o", "X=y"],
                 workdir=str(tmp_path))
    assert job.run() == 0, "".join("".join(o) for o in job.outputs)[-3000:]
    out = "".join("".join(o) for o in job.outputs)
    seen = sorted(re.findall(r"SSHW rank=(\d) host=(\w+) local=(\d)/(\d)", out))
    assert seen == [("0", "nodeA", "0", "2"), ("1", "nodeA", "1", "2"), ("2", "nodeB", "0", "2"),
                    ("3", "nodeB", "1", "2")], out[-3000:]
    assert job.attempts == [1, 1, 1, 2]


def test_launcher_mpi_cluster(tmp_path):
    """--cluster mpi: one mpirun of the worker shim, which maps the MPI rank variables to the
    rabit worker environment (task id, LOCAL_RANK per node) and runs the command."""
    fake = os.path.join(ROOT, "tests", "scripts", "fake_mpirun.sh")
    worker = os.path.join(ROOT, "tests", "scripts", "ssh_worker.py")
    out = subprocess.run([sys.executable, "-m", "rabit_amd.launcher", "--cluster", "mpi",
                          "--mpirun", fake, "--host-ip", "127.0.0.1", "--port", "9411", "-n", "4",
                          "--timeout", "120", "--", sys.executable, worker],
                         capture_output=True, text=True, timeout=180, cwd=str(tmp_path),
                         env=dict(os.environ, PYTHONPATH=ROOT))
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    seen = sorted(re.findall(r"SSHW rank=(\d) host=\w+ local=(\d)/(\d)", out.stdout))
    assert seen == [("0", "0", "2"), ("1", "1", "2"), ("2", "0", "2"), ("3", "1", "2")], out.stdout


def test_shim_env_schedulers():
    from rabit_amd.launcher import shim_env
    e = shim_env({"SLURM_PROCID": "5", "SLURM_LOCALID": "1", "SLURM_NTASKS_PER_NODE": "8(x2)"},
                 "10.0.0.1", 9091, 16)
    assert (e["DMLC_TASK_ID"], e["LOCAL_RANK"], e["LOCAL_WORLD_SIZE"]) == ("5", "1", "8")
    assert e["DMLC_TRACKER_URI"] == "10.0.0.1" and e["rabit_world_size"] == "16"
    e = shim_env({"PMI_RANK": "2", "MPI_LOCALRANKID": "0", "LOCAL_RANK": "3"}, "h", 1, 4)
    assert e["DMLC_TASK_ID"] == "2" and e["LOCAL_RANK"] == "3"  # an explicit LOCAL_RANK wins
    with pytest.raises(RuntimeError):
        shim_env({}, "h", 1, 4)


def test_launcher_ssh_kill_reaches_remote_worker(tmp_path):
    """killing an ssh job ends the remote workers too: each remote shell watches its session's
    stdin, which the launcher holds open, and terminates its worker on EOF"""
    import time
    from rabit_amd.launcher import SSHJob

    fake = os.path.join(ROOT, "tests", "scripts", "fake_ssh.sh")
    pidfile = tmp_path / "pids"
    cmd = [sys.executable, "-c",
           "import os, time\n"
           "open(%r, 'a').write('%%d\\n' %% os.getpid())\n"
           "time.sleep(300)\n" % str(pidfile)]
    job = SSHJob(cmd, [("nodeA", 2)], 2, host_ip="127.0.0.1", tracker_port=9421,
                 ssh=[fake], workdir=str(tmp_path), print_fn=lambda m: None)
    job.tracker.start(2)
    import threading
    threads = [threading.Thread(target=job._run_worker, args=(i,), daemon=True) for i in range(2)]
    for t in threads:
        t.start()
    deadline = time.time() + 30
    while time.time() < deadline and (not pidfile.exists() or
                                      len(pidfile.read_text().split()) < 2):
        time.sleep(0.1)
    pids = [int(x) for x in pidfile.read_text().split()]
    assert len(pids) == 2
    job.kill()

    def alive(pid):
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            return False
        # a zombie (exited, not yet reaped by its shell) counts as gone
        with open("/proc/%d/stat" % pid) as f:
            return f.read().split(")")[-1].split()[0] != "Z"

    deadline = time.time() + 15
    while time.time() < deadline and any(alive(p) for p in pids):
        time.sleep(0.1)
    assert not any(alive(p) for p in pids), "remote workers survived the launcher's kill"
