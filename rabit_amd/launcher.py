"""Job launcher with restart-on-failure (the role of `dmlc-submit --cluster local|ssh|mpi`,
which the reference's test/test.mk and guide use; plus Slurm).

Starts a tracker, spawns `num_workers` copies of a command with the DMLC_* environment and
restarts any worker that exits with a non-zero status, up to `num_attempt` times, passing the
attempt number in DMLC_NUM_ATTEMPT (the mock engine keys its kill points on it).  This is how
the fault-tolerance scenarios of the reference's test/test.mk run on one machine.

    python -m rabit_amd.launcher -n 10 --num-attempt 20 -- ./model_recover 10000 mock=0,0,1,0

Multi-node jobs (`--cluster ssh --host-file hosts`): workers are started over ssh on the hosts
of the file, `host[:slots]` or `host slots=N` per line.  Ranks fill each host's slots before the
next host, so ranks that share a node are consecutive (their ring links and the direct device
transport stay on xGMI); every worker gets LOCAL_RANK / LOCAL_WORLD_SIZE for its node, from
which the device plane picks its GPU (one process per GPU).  The tracker listens on --host-ip,
by default this host's address.  A remote worker ends with its ssh session, so a killed
launcher leaves nothing running on the hosts.

    python -m rabit_amd.launcher --cluster ssh --host-file hosts -n 16 -- python train.py

Under an MPI launcher or Slurm (`--cluster mpi` / `--cluster slurm`) the job's processes belong
to `mpirun` / `srun`: the launcher runs the tracker and one `mpirun -n N` (or `srun -n N`) of a
small worker shim, which maps the scheduler's rank variables (OMPI_COMM_WORLD_RANK, PMI_RANK,
PMIX_RANK, SLURM_PROCID and their local-rank counterparts) to DMLC_TASK_ID and LOCAL_RANK and
runs the command as its child.  As with dmlc-submit's mpi mode, restarts are the scheduler's
business there, not the launcher's.

    python -m rabit_amd.launcher --cluster mpi -n 16 --mpi-args "--hostfile hosts" -- ./prog
"""
from __future__ import annotations

import argparse
import os
import select
import shlex
import socket
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

from .tracker import RabitTracker


class LocalJob:
    """Run a rabit job of local worker processes."""

    def __init__(self, cmd: Sequence[str], num_workers: int, num_attempt: int = 1,
                 env: Optional[Dict[str, str]] = None, host_ip: str = "127.0.0.1",
                 tracker_port: int = 9091, timeout: Optional[float] = None,
                 capture: bool = False, print_fn=None):
        self.cmd = list(cmd)
        self.n = num_workers
        self.num_attempt = num_attempt
        self.env = dict(env or {})
        self.timeout = timeout
        self.capture = capture
        self.tracker = RabitTracker(host_ip, num_workers, tracker_port, print_fn=print_fn)
        self.returncodes: List[Optional[int]] = [None] * num_workers
        self.attempts: List[int] = [0] * num_workers
        self.outputs: List[List[str]] = [[] for _ in range(num_workers)]
        self._procs: List[Optional[subprocess.Popen]] = [None] * num_workers
        self._dying: List[subprocess.Popen] = []  # reported their exit, not yet reaped
        # exit codes workers reported on their exit pipe (each restarted without waiting)
        self.reported_exits: List[List[int]] = [[] for _ in range(num_workers)]
        self._lock = threading.Lock()
        self._stop = False

    def _worker_env(self, task: int, attempt: int) -> Dict[str, str]:
        e = dict(os.environ)
        # workers can import rabit_amd without installing it
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
        e.update(self.env)
        e.update(self.tracker.worker_envs())
        e.update({
            "DMLC_TASK_ID": str(task),
            "DMLC_ROLE": "worker",
            "DMLC_NUM_ATTEMPT": str(attempt),
            "DMLC_NUM_WORKER": str(self.n),
            "rabit_world_size": str(self.n),
        })
        return e

    def _spawn(self, task: int, attempt: int) -> subprocess.Popen:
        # the exit pipe: a worker that fails by itself writes its exit code here before it
        # _Exits (csrc/src/core/exit.h), so the restart need not wait for the kernel to tear
        # down a process that holds GPU memory (~0.2 s, on the survivors' recovery path)
        env = self._worker_env(task, attempt)
        rfd, wfd = os.pipe()
        env["XRABIT_EXIT_FD"] = "%d:%d" % (wfd, os.fstat(wfd).st_ino)
        try:
            p = subprocess.Popen(
                self.cmd, env=env, pass_fds=(wfd,),
                stdout=subprocess.PIPE if self.capture else None,
                stderr=subprocess.STDOUT if self.capture else None,
                text=self.capture)
        except BaseException:
            os.close(rfd)
            raise
        finally:
            os.close(wfd)
        p.exit_pipe = rfd
        return p

    @staticmethod
    def _wait_exit(p: subprocess.Popen) -> Tuple[int, bool]:
        """(exit code, whether the process may still be tearing down): the code the worker
        reported on its exit pipe, else its status once it has ended"""
        rfd = getattr(p, "exit_pipe", None)
        if rfd is None:
            return p.wait(), False
        try:
            buf = b""
            while True:
                ready, _, _ = select.select([rfd], [], [], 0.1)
                if ready:
                    chunk = os.read(rfd, 64)
                    if not chunk:  # every writer closed: the process has ended
                        return p.wait(), False
                    buf += chunk
                    if b"\n" in buf:
                        line = buf.split(b"\n", 1)[0].strip()
                        code = int(line) if line.lstrip(b"-").isdigit() else 1
                        if code != 0:
                            return code, True
                elif p.poll() is not None:
                    return p.returncode, False
        finally:
            os.close(rfd)

    def _drain(self, task: int, p: subprocess.Popen):
        for line in p.stdout:
            self.outputs[task].append(line)

    def _reap(self, p: subprocess.Popen, reader: Optional[threading.Thread]):
        p.wait()
        if reader is not None:
            reader.join()
        with self._lock:
            if p in self._dying:
                self._dying.remove(p)

    def _run_worker(self, task: int):
        attempt = 0
        while True:
            with self._lock:
                if self._stop:
                    return
                p = self._spawn(task, attempt)
                self._procs[task] = p
            reader = None
            if self.capture:
                reader = threading.Thread(target=self._drain, args=(task, p), daemon=True)
                reader.start()
            rc, dying = self._wait_exit(p)
            self.attempts[task] = attempt + 1
            attempt += 1
            if dying:
                self.reported_exits[task].append(rc)
            if dying and rc != 0 and attempt < self.num_attempt:
                # restart now; the old process finishes dying (and is reaped) meanwhile
                with self._lock:
                    self._dying.append(p)
                threading.Thread(target=self._reap, args=(p, reader), daemon=True).start()
                continue
            p.wait()
            if reader is not None:
                reader.join()
            if rc == 0:
                self.returncodes[task] = 0
                return
            if attempt >= self.num_attempt:
                self.returncodes[task] = rc
                return
            time.sleep(0.01)  # (a restart is on the recovery critical path of the survivors)

    def run(self) -> int:
        self.tracker.start(self.n)
        threads = [threading.Thread(target=self._run_worker, args=(i,), daemon=True)
                   for i in range(self.n)]
        for t in threads:
            t.start()
        deadline = None if self.timeout is None else time.time() + self.timeout
        for t in threads:
            t.join(None if deadline is None else max(0.0, deadline - time.time()))
        if any(t.is_alive() for t in threads):
            self.kill()
            tail = ""
            if self.capture:
                for t in threads:
                    t.join(5)
                tail = "\n".join("--- worker %d ---\n%s" % (i, "".join(o[-40:]))
                                 for i, o in enumerate(self.outputs))
            raise TimeoutError("rabit job did not finish within %s s\n%s" % (self.timeout, tail))
        failed = [rc for rc in self.returncodes if rc != 0]
        if not failed:
            self.tracker.join(30)
        return 0 if not failed else (failed[0] or 1)

    def kill(self):
        with self._lock:
            self._stop = True
            for p in list(self._procs) + list(self._dying):
                if p is not None and p.poll() is None:
                    p.kill()


def parse_host_file(path: str) -> List[Tuple[str, int]]:
    """`host`, `host:slots` or `host slots=N` per line ('#' starts a comment)"""
    hosts = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if not line:
                continue
            slots = 1
            parts = line.split()
            host = parts[0]
            for opt in parts[1:]:
                if opt.startswith("slots="):
                    slots = int(opt[len("slots="):])
            if ":" in host:
                host, n = host.rsplit(":", 1)
                slots = int(n)
            if slots < 1:
                raise ValueError("%s: host %s has no slots" % (path, host))
            hosts.append((host, slots))
    if not hosts:
        raise ValueError("%s lists no hosts" % path)
    return hosts


def place_workers(hosts: Sequence[Tuple[str, int]], n: int) -> List[Tuple[str, int, int]]:
    """(host, local_rank, local_world) of each task: every host's slots are filled before the
    next host's, so the ranks of one node are consecutive"""
    total = sum(s for _, s in hosts)
    if n > total:
        raise ValueError("%d workers but the host file has %d slots" % (n, total))
    out: List[Tuple[str, int, int]] = []
    for host, slots in hosts:
        k = min(slots, n - len(out))
        out.extend((host, i, k) for i in range(k))
        if len(out) == n:
            break
    return out


class SSHJob(LocalJob):
    """A rabit job whose workers run on remote hosts over ssh (dmlc-submit --cluster ssh).

    The worker's environment is not inherited across ssh: the DMLC_* / rabit_* variables, the
    tracker address, LOCAL_RANK / LOCAL_WORLD_SIZE and the --env pairs are exported explicitly
    in the remote shell, which changes to `workdir` (the launch directory by default, assumed
    to be shared or replicated) before running the command.  A worker whose ssh session ends
    with a non-zero status is restarted on the same host, like a local one."""

    def __init__(self, cmd: Sequence[str], hosts: Sequence[Tuple[str, int]], num_workers: int,
                 num_attempt: int = 1, env: Optional[Dict[str, str]] = None,
                 host_ip: Optional[str] = None, tracker_port: int = 9091,
                 timeout: Optional[float] = None, capture: bool = False, print_fn=None,
                 ssh: Sequence[str] = ("ssh", "-o", "StrictHostKeyChecking=no",
                                       "-o", "BatchMode=yes"),
                 workdir: Optional[str] = None):
        super().__init__(cmd, num_workers, num_attempt, env, host_ip or default_host_ip(),
                         tracker_port, timeout, capture, print_fn)
        self.placement = place_workers(hosts, num_workers)
        self.ssh = list(ssh)
        self.workdir = workdir or os.getcwd()

    def _remote_env(self, task: int, attempt: int) -> Dict[str, str]:
        host, local_rank, local_world = self.placement[task]
        e = {k: v for k, v in self._worker_env(task, attempt).items()
             if k.startswith(("DMLC_", "rabit_", "XRABIT_")) or k == "PYTHONPATH"}
        e.update(self.env)
        e.update({"LOCAL_RANK": str(local_rank), "LOCAL_WORLD_SIZE": str(local_world)})
        return e

    def remote_command(self, task: int, attempt: int) -> str:
        """The remote shell line: the worker runs in the background with stdin from /dev/null,
        and a watcher reads the session's stdin (kept open by the launcher) until EOF, then
        terminates the worker.  A killed launcher or a dropped connection therefore ends the
        remote worker too, instead of leaving it behind on its host."""
        exports = " ".join("%s=%s" % (k, shlex.quote(v))
                           for k, v in sorted(self._remote_env(task, attempt).items()))
        worker = "env %s %s" % (exports, " ".join(shlex.quote(c) for c in self.cmd))
        return ("cd %s || exit 1; exec 3<&0; %s </dev/null & w=$!; "
                "( cat <&3 >/dev/null 2>&1; kill -TERM $w 2>/dev/null ) >/dev/null 2>&1 & "
                "exec 3<&-; wait $w" % (shlex.quote(self.workdir), worker))

    def _spawn(self, task: int, attempt: int) -> subprocess.Popen:
        host = self.placement[task][0]
        return subprocess.Popen(
            self.ssh + [host, self.remote_command(task, attempt)],
            stdin=subprocess.PIPE,  # held open: its EOF tells the remote watcher to stop
            stdout=subprocess.PIPE if self.capture else None,
            stderr=subprocess.STDOUT if self.capture else None,
            text=self.capture)

    def kill(self):
        with self._lock:
            self._stop = True
            for p in self._procs:
                if p is not None and p.poll() is None:
                    if p.stdin is not None:
                        p.stdin.close()
                    p.kill()


_RANK_VARS = ("OMPI_COMM_WORLD_RANK", "PMIX_RANK", "PMI_RANK", "SLURM_PROCID")
_LOCAL_RANK_VARS = ("OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "SLURM_LOCALID")
_LOCAL_SIZE_VARS = ("OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "SLURM_NTASKS_PER_NODE")


def _first(env: Dict[str, str], names: Sequence[str]) -> Optional[str]:
    for k in names:
        if env.get(k, "") != "":
            return env[k]
    return None


def shim_env(env: Dict[str, str], tracker: str, port: int, world: int) -> Dict[str, str]:
    """the rabit worker environment of a process started by mpirun / srun"""
    task = _first(env, _RANK_VARS)
    if task is None:
        raise RuntimeError("no MPI/Slurm rank variable (%s) in the environment"
                           % ", ".join(_RANK_VARS))
    out = dict(env)
    out.update({"DMLC_TRACKER_URI": tracker, "DMLC_TRACKER_PORT": str(port),
                "DMLC_TASK_ID": task, "DMLC_ROLE": "worker",
                "DMLC_NUM_ATTEMPT": env.get("DMLC_NUM_ATTEMPT", "0"),
                "DMLC_NUM_WORKER": str(world), "rabit_world_size": str(world)})
    local = _first(env, _LOCAL_RANK_VARS)
    if local is not None and "LOCAL_RANK" not in env:
        out["LOCAL_RANK"] = local
    size = _first(env, _LOCAL_SIZE_VARS)
    if size is not None and "LOCAL_WORLD_SIZE" not in env:
        out["LOCAL_WORLD_SIZE"] = size.split("(")[0]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return out


def run_shim(argv: Sequence[str]) -> int:
    """worker side of --cluster mpi|slurm: `--shim URI PORT WORLD -- cmd...`"""
    tracker, port, world = argv[0], int(argv[1]), int(argv[2])
    cmd = list(argv[3:])
    if cmd and cmd[0] == "--":
        cmd = cmd[1:]
    return subprocess.call(cmd, env=shim_env(dict(os.environ), tracker, port, world))


class SchedulerJob:
    """A rabit job whose processes are started by mpirun or srun (see the module docstring)"""

    def __init__(self, cmd: Sequence[str], num_workers: int, launcher: Sequence[str],
                 host_ip: Optional[str] = None, tracker_port: int = 9091,
                 timeout: Optional[float] = None, print_fn=None):
        self.cmd = list(cmd)
        self.n = num_workers
        self.launcher = list(launcher)
        self.timeout = timeout
        self.tracker = RabitTracker(host_ip or default_host_ip(), num_workers, tracker_port,
                                    print_fn=print_fn)

    def command(self) -> List[str]:
        return self.launcher + [sys.executable, "-m", "rabit_amd.launcher", "--shim",
                                self.tracker.host_ip, str(self.tracker.port), str(self.n),
                                "--"] + self.cmd

    def run(self) -> int:
        self.tracker.start(self.n)
        rc = subprocess.call(self.command(), timeout=self.timeout)
        if rc == 0:
            self.tracker.join(30)
        return rc


def default_host_ip() -> str:
    """an address of this host other peers can reach (the tracker binds and advertises it)"""
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect(("10.255.255.255", 1))  # no packet is sent: picks the outgoing interface
            return s.getsockname()[0]
    except OSError:
        return socket.gethostbyname(socket.gethostname())


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] == "--shim":
        sys.exit(run_shim(argv[1:]))
    ap = argparse.ArgumentParser(description="launch an xrabit job (local, ssh, mpi or slurm)")
    ap.add_argument("-n", "--num-workers", type=int, required=True)
    ap.add_argument("--num-attempt", "--local-num-attempt", type=int, default=1,
                    help="restarts allowed per worker (fault-tolerance tests)")
    ap.add_argument("--cluster", choices=["local", "ssh", "mpi", "slurm"], default="local")
    ap.add_argument("--mpi-args", default="", help="--cluster mpi: extra mpirun arguments")
    ap.add_argument("--mpirun", default="mpirun", help="--cluster mpi: the MPI launcher")
    ap.add_argument("--srun", default="srun", help="--cluster slurm: the Slurm launcher")
    ap.add_argument("--host-file", help="--cluster ssh: host[:slots] per line")
    ap.add_argument("--ssh", default="ssh -o StrictHostKeyChecking=no -o BatchMode=yes",
                    help="--cluster ssh: the ssh command (host and remote command appended)")
    ap.add_argument("--workdir", default=None,
                    help="--cluster ssh: directory the remote workers start in (default: cwd)")
    ap.add_argument("--host-ip", default=None,
                    help="tracker address (default 127.0.0.1 local, this host's address ssh)")
    ap.add_argument("--port", type=int, default=9091)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for every worker")
    ap.add_argument("command", nargs=argparse.REMAINDER)
    args = ap.parse_args(argv)
    cmd = args.command[1:] if args.command and args.command[0] == "--" else args.command
    if not cmd:
        ap.error("missing worker command")
    env = dict(kv.split("=", 1) for kv in args.env)
    if args.cluster in ("mpi", "slurm"):
        if args.cluster == "mpi":
            launcher = shlex.split(args.mpirun) + ["-n", str(args.num_workers)] + \
                shlex.split(args.mpi_args)
        else:
            launcher = shlex.split(args.srun) + ["-n", str(args.num_workers)]
        job = SchedulerJob(cmd, args.num_workers, launcher, args.host_ip, args.port, args.timeout)
        sys.exit(job.run())
    if args.cluster == "ssh":
        if not args.host_file:
            ap.error("--cluster ssh needs --host-file")
        job = SSHJob(cmd, parse_host_file(args.host_file), args.num_workers, args.num_attempt,
                     env, args.host_ip, args.port, args.timeout, ssh=shlex.split(args.ssh),
                     workdir=args.workdir)
    else:
        job = LocalJob(cmd, args.num_workers, args.num_attempt, env,
                       args.host_ip or "127.0.0.1", args.port, args.timeout)
    rc = job.run()
    sys.exit(rc)


if __name__ == "__main__":
    main()
