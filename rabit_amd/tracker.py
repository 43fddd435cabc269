"""Rabit tracker: rank assignment, tree/ring topology and link brokering.

The reference delegates this to the external dmlc-core tracker;
this is a fresh implementation of the same wire protocol, so both xrabit workers and the
reference's workers can talk to it.  Protocol (all integers are little-endian int32, a string
is an int32 length followed by the bytes):

    worker -> magic(0xff99); tracker -> magic
    worker -> rank, world_size, task_id, command
    command "print":    worker -> message
    command "shutdown": (nothing more)
    command "start" / "recover":
        tracker -> rank, parent_rank, world_size, n_tree_neighbours, neighbours..., ring_prev,
                   ring_next
        loop:   worker -> n_good, good_ranks...
                tracker -> n_connect, n_accept, then n_connect x (host, port, rank)
                worker -> n_errors          (loop again while n_errors != 0)
        worker -> listen_port

Topology: a binary-heap tree; the ring is a depth-first walk of that tree whose last subtree
is walked in reverse (so consecutive ring members are mostly tree neighbours), and ranks are
relabelled so the ring is 0 -> 1 -> ... -> n-1 -> 0, which the ring collectives require
(reference allreduce_base.cc:787-789).
"""
from __future__ import annotations

import logging
import socket
import struct
import threading
import time
from typing import Dict, List, Optional, Tuple

MAGIC = 0xFF99
log = logging.getLogger("rabit_amd.tracker")


# ----------------------------------------------------------------------------- wire helpers
class _Conn:
    def __init__(self, sock: socket.socket):
        self.sock = sock

    def recv_all(self, n: int) -> bytes:
        chunks = []
        while n > 0:
            b = self.sock.recv(n)
            if not b:
                raise ConnectionError("worker closed the connection")
            chunks.append(b)
            n -= len(b)
        return b"".join(chunks)

    def recv_int(self) -> int:
        return struct.unpack("@i", self.recv_all(4))[0]

    def send_int(self, v: int) -> None:
        self.sock.sendall(struct.pack("@i", v))

    def recv_str(self) -> str:
        n = self.recv_int()
        return self.recv_all(n).decode() if n > 0 else ""

    def send_str(self, s: str) -> None:
        b = s.encode()
        self.send_int(len(b))
        self.sock.sendall(b)


# ----------------------------------------------------------------------------- topology
def tree_neighbours(rank: int, n: int) -> List[int]:
    """Neighbours of `rank` in a binary heap of n nodes (parent first)."""
    out = []
    if rank > 0:
        out.append((rank - 1) // 2)
    for child in (2 * rank + 1, 2 * rank + 2):
        if child < n:
            out.append(child)
    return out


def _ring_order(n: int) -> List[int]:
    """DFS over the heap; the last child's subtree is emitted reversed so the walk ends next
    to the root and the ring closes on a short hop."""

    def walk(r: int) -> List[int]:
        children = [c for c in (2 * r + 1, 2 * r + 2) if c < n]
        seq = [r]
        for i, c in enumerate(children):
            sub = walk(c)
            if i == len(children) - 1:
                sub.reverse()
            seq.extend(sub)
        return seq

    return walk(0)


def link_map(n: int) -> Tuple[Dict[int, List[int]], Dict[int, int], Dict[int, Tuple[int, int]]]:
    """(tree neighbours, parent, (ring prev, ring next)) per rank, relabelled so that the ring
    order is the rank order."""
    order = _ring_order(n)
    relabel = {old: new for new, old in enumerate(order)}
    tree: Dict[int, List[int]] = {}
    parent: Dict[int, int] = {}
    ring: Dict[int, Tuple[int, int]] = {}
    for old in range(n):
        new = relabel[old]
        tree[new] = [relabel[x] for x in tree_neighbours(old, n)]
        parent[new] = relabel[(old - 1) // 2] if old > 0 else -1
        ring[new] = ((new - 1) % n, (new + 1) % n)
    return tree, parent, ring


# ----------------------------------------------------------------------------- tracker
class _Worker:
    def __init__(self, conn: _Conn, host: str):
        self.conn = conn
        self.host = host
        self.rank = -1
        self.world_size = -1
        self.task_id = "NULL"
        self.cmd = ""
        self.port = -1
        self.pending_accepts = 0

    def handshake(self) -> None:
        magic = self.conn.recv_int()
        if magic != MAGIC:
            raise ConnectionError("bad magic 0x%x from %s" % (magic, self.host))
        self.conn.send_int(MAGIC)
        self.rank = self.conn.recv_int()
        self.world_size = self.conn.recv_int()
        self.task_id = self.conn.recv_str()
        self.cmd = self.conn.recv_str()


class RabitTracker:
    """Tracker server.  `start()` serves in a background thread; `join()` waits until every
    worker has sent "shutdown"."""

    def __init__(self, host_ip: str = "127.0.0.1", n_workers: int = 0, port: int = 9091,
                 port_end: int = 9999, print_fn=None):
        self.host_ip = host_ip
        self.n_workers = n_workers
        self.print_fn = print_fn or (lambda msg: print(msg, end="" if msg.endswith("\n") else "\n",
                                                       flush=True))
        self.sock = None
        # SO_REUSEADDR lets two trackers starting at once both bind a free port; only the first
        # listen() succeeds, so a listen that fails moves on to the next port as well
        for p in range(port, port_end):
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            try:
                s.bind((host_ip, p))
                s.listen(256)
            except OSError:
                s.close()
                continue
            self.sock, self.port = s, p
            break
        if self.sock is None:
            raise OSError("no free tracker port in [%d, %d)" % (port, port_end))
        self.thread: Optional[threading.Thread] = None
        self.error: Optional[BaseException] = None
        self.start_time = None
        self.end_time = None
        self.messages: List[str] = []

    def worker_envs(self) -> Dict[str, str]:
        return {"DMLC_TRACKER_URI": self.host_ip, "DMLC_TRACKER_PORT": str(self.port)}

    # -- main loop -----------------------------------------------------------------------
    def _assign(self, w: _Worker, rank: int, wait_conn: Dict[int, _Worker], tree, parent, ring):
        w.rank = rank
        nbrs = set(tree[rank])
        prev_r, next_r = ring[rank]
        c = w.conn
        c.send_int(rank)
        c.send_int(parent[rank])
        c.send_int(len(tree))
        c.send_int(len(nbrs))
        for r in sorted(nbrs):
            c.send_int(r)
        for r in (prev_r, next_r):
            if r != -1 and r != rank:
                nbrs.add(r)
                c.send_int(r)
            else:
                c.send_int(-1)
        while True:
            ngood = c.recv_int()
            good = {c.recv_int() for _ in range(ngood)}
            assert good.issubset(nbrs), "worker reports links outside its neighbourhood"
            bad = sorted(nbrs - good)
            connect = [r for r in bad if r in wait_conn]
            c.send_int(len(connect))
            c.send_int(len(bad) - len(connect))
            for r in connect:
                c.send_str(wait_conn[r].host)
                c.send_int(wait_conn[r].port)
                c.send_int(r)
            if c.recv_int() != 0:
                continue
            w.port = c.recv_int()
            for r in connect:
                wait_conn[r].pending_accepts -= 1
                if wait_conn[r].pending_accepts == 0:
                    del wait_conn[r]
            w.pending_accepts = len(bad) - len(connect)
            if w.pending_accepts > 0:
                wait_conn[rank] = w
            return

    def _serve(self):
        n = self.n_workers
        shutdown: Dict[int, bool] = {}
        wait_conn: Dict[int, _Worker] = {}
        job_map: Dict[str, int] = {}
        pending: List[_Worker] = []
        todo: List[int] = []
        maps = None
        while maps is None or len(shutdown) != n:
            fd, addr = self.sock.accept()
            w = _Worker(_Conn(fd), addr[0])
            try:
                w.handshake()
            except (ConnectionError, OSError) as e:
                log.warning("dropping connection from %s: %s", addr[0], e)
                fd.close()
                continue
            if w.cmd == "print":
                msg = w.conn.recv_str()
                self.messages.append(msg)
                self.print_fn(msg)
                fd.close()
                continue
            if w.cmd == "shutdown":
                assert w.rank >= 0 and w.rank not in shutdown, "duplicate shutdown"
                shutdown[w.rank] = True
                log.debug("rank %d shut down", w.rank)
                fd.close()
                continue
            assert w.cmd in ("start", "recover"), "unknown command %r" % w.cmd
            if maps is None:
                if w.world_size > 0:
                    n = w.world_size
                assert n > 0, "world size unknown: pass n_workers or rabit_world_size"
                self.n_workers = n
                maps = link_map(n)
                todo = list(range(n))
            elif w.world_size > 0:
                assert w.world_size == n, "inconsistent world size %d vs %d" % (w.world_size, n)
            if w.cmd == "recover":
                assert w.rank >= 0, "recover without a rank"
            rank = w.rank
            if rank < 0 and w.task_id != "NULL" and w.task_id in job_map:
                rank = job_map[w.task_id]
            if rank >= 0:
                self._assign(w, rank, wait_conn, *maps)
                if rank in todo:
                    todo.remove(rank)
                fd.close()
                continue
            # batch assignment once every expected worker connected: stable order by host,
            # then by numeric task id (so torchrun RANK == rabit rank on one host)
            pending.append(w)
            if len(pending) == len(todo):

                def key(x: _Worker):
                    t = x.task_id
                    return (x.host, 0, int(t), "") if t.lstrip("-").isdigit() else (x.host, 1, 0, t)

                pending.sort(key=key)
                for pw in pending:
                    r = todo.pop(0)
                    if pw.task_id != "NULL":
                        job_map[pw.task_id] = r
                    self._assign(pw, r, wait_conn, *maps)
                    pw.conn.sock.close()
                pending = []
                if not todo and self.start_time is None:
                    self.start_time = time.time()
                    log.info("all %d workers started", n)
        self.end_time = time.time()

    def _run(self):
        try:
            self._serve()
        except BaseException as e:  # noqa: BLE001 - surfaced through join()
            self.error = e
            log.exception("tracker failed")
        finally:
            self.sock.close()

    def start(self, n_workers: Optional[int] = None) -> "RabitTracker":
        if n_workers is not None:
            self.n_workers = n_workers
        self.thread = threading.Thread(target=self._run, name="rabit-tracker", daemon=True)
        self.thread.start()
        return self

    def join(self, timeout: Optional[float] = None) -> bool:
        assert self.thread is not None
        self.thread.join(timeout)
        if self.error is not None:
            raise RuntimeError("tracker failed: %r" % (self.error,))
        return not self.thread.is_alive()

    def alive(self) -> bool:
        return self.thread is not None and self.thread.is_alive()


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="xrabit tracker")
    ap.add_argument("-n", "--num-workers", type=int, required=True)
    ap.add_argument("--host-ip", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9091)
    args = ap.parse_args(argv)
    t = RabitTracker(args.host_ip, args.num_workers, args.port).start()
    print("DMLC_TRACKER_URI=%s DMLC_TRACKER_PORT=%d" % (t.host_ip, t.port), flush=True)
    t.join()


if __name__ == "__main__":
    main()
