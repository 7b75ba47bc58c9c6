"""Out-of-band control plane for the multi-rank bootstrap (no torch, no GPU).

The ranks of one node exchange a few small host objects before and around a
solve: the RCCL unique id (gk_comm_unique_id), every rank's device-exchange
IPC handle (gk_xchg_handle), agreement flags (did every rank's self-test /
warmup pass?) and the max-over-ranks timing.  INTEGRATION.md leaves that
transport to the caller ("shared out of band"); this is the one bench.py and
the multi-rank tests use -- plain TCP on the loopback interface between
processes of one node, so a rank process never imports torch and runs the
library on the HIP runtime and RCCL it was built against.

Rendezvous: rank 0 listens on an ephemeral 127.0.0.1 port and publishes
(port, authkey) in a file named by the launch (MASTER_ADDR, MASTER_PORT and
the launcher's pid, which torch.distributed.run's ranks share); the other
ranks poll for that file and connect.  Every collective is a gather to rank 0
followed by a broadcast of the result, in rank order, so all ranks see
identical values.
"""
from __future__ import annotations

import os
import secrets
import tempfile
import time
from multiprocessing import AuthenticationError
from multiprocessing.connection import Client, Listener


def launch_key() -> str:
    """Identifies one multi-rank launch on this node (same on all its ranks)."""
    return "_".join([os.environ.get("MASTER_ADDR", "127.0.0.1"), os.environ.get("MASTER_PORT", "0"),
                     os.environ.get("TORCHELASTIC_RUN_ID", ""), str(os.getppid())]).replace("/", "_")


class Ctl:
    """A gather/broadcast control plane over TCP between the ranks of one node."""

    def __init__(self, rank: int, world: int, key: str | None = None, timeout: float = 300.0,
                 rdzv_dir: str | None = None):
        self.rank, self.world = rank, world
        self.timeout = timeout
        self._peers = []  # rank 0: connections of ranks 1..world-1, in rank order
        self._conn = None  # ranks > 0: connection to rank 0
        self._listener = None
        self._file = os.path.join(rdzv_dir or tempfile.gettempdir(), f"gk_ctl_{key or launch_key()}")
        if world == 1:
            return
        if rank == 0:
            auth = secrets.token_bytes(16)
            self._listener = Listener(("127.0.0.1", 0), authkey=auth)
            port = self._listener.address[1]
            tmp = self._file + f".{os.getpid()}.tmp"
            with open(tmp, "w") as f:
                f.write(f"{port} {auth.hex()}\n")
            os.replace(tmp, self._file)  # atomic: a reader sees all of it or nothing
            sock = getattr(getattr(self._listener, "_listener", None), "_socket", None)
            if sock is not None:
                sock.settimeout(timeout)  # accept() raises instead of waiting forever for a dead rank
            got = {}
            deadline = time.monotonic() + timeout
            while len(got) < world - 1:
                if time.monotonic() > deadline:
                    raise TimeoutError(f"control plane: {world - 1 - len(got)} rank(s) never connected")
                c = self._listener.accept()
                r = c.recv()
                got[int(r)] = c
            self._peers = [got[r] for r in range(1, world)]
        else:
            deadline = time.monotonic() + timeout
            last = None
            while True:
                try:
                    port, auth = open(self._file).read().split()
                    self._conn = Client(("127.0.0.1", int(port)), authkey=bytes.fromhex(auth))
                    self._conn.send(rank)
                    break
                except (OSError, ValueError, EOFError, AuthenticationError) as e:  # not published yet / a stale file
                    last = e
                    if time.monotonic() > deadline:
                        raise TimeoutError(f"control plane: rank {rank} could not reach rank 0 ({last})") from e
                    time.sleep(0.05)

    # -------------------------------------------------------------- collectives
    def allgather(self, obj) -> list:
        """Every rank's object, in rank order, on every rank."""
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            vals = [obj] + [c.recv() for c in self._peers]
            for c in self._peers:
                c.send(vals)
            return vals
        self._conn.send(obj)
        return self._conn.recv()

    def bcast(self, obj, root: int = 0):
        return self.allgather(obj if self.rank == root else None)[root]

    def allreduce(self, x, op: str = "sum"):
        vals = self.allgather(x)
        if op == "min":
            return min(vals)
        if op == "max":
            return max(vals)
        s = vals[0]
        for v in vals[1:]:
            s = s + v
        return s

    def barrier(self) -> None:
        self.allgather(None)

    def close(self) -> None:
        for c in self._peers:
            c.close()
        if self._conn is not None:
            self._conn.close()
        if self._listener is not None:
            self._listener.close()
            try:
                os.unlink(self._file)
            except OSError:
                pass
        self._peers, self._conn, self._listener = [], None, None
