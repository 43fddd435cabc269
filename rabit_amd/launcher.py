"""Local job launcher with restart-on-failure (the role of `dmlc-submit --cluster local`).

Starts a tracker, spawns `num_workers` copies of a command with the DMLC_* environment and
restarts any worker that exits with a non-zero status, up to `num_attempt` times, passing the
attempt number in DMLC_NUM_ATTEMPT (the mock engine keys its kill points on it).  This is how
the fault-tolerance scenarios of the reference's test/test.mk run on one machine.

    python -m rabit_amd.launcher -n 10 --num-attempt 20 -- ./model_recover 10000 mock=0,0,1,0
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Sequence

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

    def _run_worker(self, task: int):
        attempt = 0
        while True:
            with self._lock:
                if self._stop:
                    return
                p = subprocess.Popen(
                    self.cmd, env=self._worker_env(task, attempt),
                    stdout=subprocess.PIPE if self.capture else None,
                    stderr=subprocess.STDOUT if self.capture else None,
                    text=self.capture)
                self._procs[task] = p
            if self.capture:
                for line in p.stdout:
                    self.outputs[task].append(line)
            rc = p.wait()
            self.attempts[task] = attempt + 1
            if rc == 0:
                self.returncodes[task] = 0
                return
            attempt += 1
            if attempt >= self.num_attempt:
                self.returncodes[task] = rc
                return
            time.sleep(0.05)

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
            for p in self._procs:
                if p is not None and p.poll() is None:
                    p.kill()


def main(argv=None):
    ap = argparse.ArgumentParser(description="launch a local xrabit job")
    ap.add_argument("-n", "--num-workers", type=int, required=True)
    ap.add_argument("--num-attempt", "--local-num-attempt", type=int, default=1,
                    help="restarts allowed per worker (fault-tolerance tests)")
    ap.add_argument("--host-ip", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9091)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for every worker")
    ap.add_argument("command", nargs=argparse.REMAINDER)
    args = ap.parse_args(argv)
    cmd = args.command[1:] if args.command and args.command[0] == "--" else args.command
    if not cmd:
        ap.error("missing worker command")
    env = dict(kv.split("=", 1) for kv in args.env)
    job = LocalJob(cmd, args.num_workers, args.num_attempt, env, args.host_ip, args.port,
                   args.timeout)
    rc = job.run()
    sys.exit(rc)


if __name__ == "__main__":
    main()
