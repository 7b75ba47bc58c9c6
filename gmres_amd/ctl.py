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
"port token pid" in a file named by the launch (MASTER_ADDR, MASTER_PORT and
the launcher's pid, which torch.distributed.run's ranks share); the other
ranks poll for that file, skip it while the pid it names is not alive (a file
left by a crashed launch), connect and present the token, which rank 0 checks
before it counts the rank.

Authentication comes before any deserialisation: the hello is raw
bytes -- the 32-character token and the rank as a 4-byte integer -- compared
with hmac.compare_digest, and rank 0 answers with raw bytes too; only links
that passed it ever carry pickles.  The rendezvous file is created mode 0600,
and a joining rank uses it only if this user owns it, so neither the token nor
the port can be read or planted by another local user.  Every collective is a gather to rank 0 followed by
a broadcast of the result, in rank order, so all ranks see identical values.

Every wait is bounded (round 5): the connect,
the hello, and every receive of a collective time out after `timeout` seconds
(GK_CTL_TIMEOUT overrides the default) with a TimeoutError that names the rank
that never answered, so a live-but-stuck peer cannot block the others forever.
"""
from __future__ import annotations

import hmac
import os
import pickle
import secrets
import socket
import struct
import tempfile
import time

_HDR = struct.Struct("!Q")
_HELLO = struct.Struct("!32sI")  # token (32 hex characters), rank
_ACK = b"OK"


def launch_key() -> str:
    """Identifies one multi-rank launch on this node (same on all its ranks)."""
    return "_".join([os.environ.get("MASTER_ADDR", "127.0.0.1"), os.environ.get("MASTER_PORT", "0"),
                     os.environ.get("TORCHELASTIC_RUN_ID", ""), str(os.getppid())]).replace("/", "_")


def default_timeout() -> float:
    return float(os.environ.get("GK_CTL_TIMEOUT", "300"))


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


class _Link:
    """One length-prefixed pickle stream over a connected socket; every receive
    bounded by the socket timeout."""

    def __init__(self, sock: socket.socket, who: str):
        self.sock, self.who = sock, who

    def send(self, obj) -> None:
        data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        self.sock.sendall(_HDR.pack(len(data)) + data)

    def _exact(self, n: int, timeout: float) -> bytes:
        buf = bytearray()
        self.sock.settimeout(timeout)
        while len(buf) < n:
            try:
                chunk = self.sock.recv(n - len(buf))
            except socket.timeout as e:
                raise TimeoutError(f"control plane: no message from {self.who} within {timeout:.0f} s") from e
            if not chunk:
                raise ConnectionError(f"control plane: {self.who} closed the connection")
            buf += chunk
        return bytes(buf)

    def recv(self, timeout: float):
        (n,) = _HDR.unpack(self._exact(_HDR.size, timeout))
        return pickle.loads(self._exact(n, timeout))

    def send_raw(self, data: bytes) -> None:
        self.sock.sendall(data)

    def recv_raw(self, n: int, timeout: float) -> bytes:
        return self._exact(n, timeout)

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


class Ctl:
    """A gather/broadcast control plane over TCP between the ranks of one node."""

    def __init__(self, rank: int, world: int, key: str | None = None, timeout: float | None = None,
                 rdzv_dir: str | None = None):
        self.rank, self.world = rank, world
        self.timeout = default_timeout() if timeout is None else float(timeout)
        self._peers: list[_Link] = []  # rank 0: links to ranks 1..world-1, in rank order
        self._conn: _Link | None = None  # ranks > 0: link to rank 0
        self._listener: socket.socket | None = None
        self._file = os.path.join(rdzv_dir or tempfile.gettempdir(), f"gk_ctl_{key or launch_key()}")
        if world == 1:
            return
        deadline = time.monotonic() + self.timeout
        if rank == 0:
            self._serve(deadline)
        else:
            self._join(deadline)

    def _serve(self, deadline: float) -> None:
        token = secrets.token_hex(16)
        ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        ls.bind(("127.0.0.1", 0))
        ls.listen(self.world)
        self._listener = ls
        tmp = self._file + f".{os.getpid()}.tmp"
        fd = os.open(tmp, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o600)  # owner-only: the token is a secret
        with os.fdopen(fd, "w") as f:
            f.write(f"{ls.getsockname()[1]} {token} {os.getpid()}\n")
        os.replace(tmp, self._file)  # atomic: a reader sees all of it or nothing
        got: dict[int, _Link] = {}
        while len(got) < self.world - 1:
            left = deadline - time.monotonic()
            if left <= 0:
                missing = sorted(set(range(1, self.world)) - set(got))
                raise TimeoutError(f"control plane: rank(s) {missing} never connected")
            ls.settimeout(left)
            try:
                s, _ = ls.accept()
            except socket.timeout:
                continue
            link = _Link(s, "a connecting rank")
            try:  # raw bytes: nothing is unpickled before the token matched
                tok, r = _HELLO.unpack(link.recv_raw(_HELLO.size, min(10.0, max(left, 0.1))))
            except (TimeoutError, ConnectionError, struct.error):
                link.close()  # not one of ours (or too slow to say hello): drop it
                continue
            if not (hmac.compare_digest(tok, token.encode()) and 0 < r < self.world and r not in got):
                link.close()
                continue
            link.who = f"rank {r}"
            link.send_raw(_ACK)
            got[r] = link
        self._peers = [got[r] for r in range(1, self.world)]

    def _join(self, deadline: float) -> None:
        last = None
        while True:
            try:
                st = os.stat(self._file)
                if st.st_uid != os.getuid() or (st.st_mode & 0o077):
                    raise ValueError(f"rendezvous file {self._file} is not this user's private file")
                port, token, pid = open(self._file).read().split()
                if not _pid_alive(int(pid)):
                    raise ValueError(f"rendezvous file of a dead rank 0 (pid {pid})")
                left = max(0.1, deadline - time.monotonic())
                s = socket.create_connection(("127.0.0.1", int(port)), timeout=min(5.0, left))
                link = _Link(s, "rank 0")
                link.send_raw(_HELLO.pack(token.encode(), self.rank))
                if link.recv_raw(len(_ACK), min(10.0, left)) != _ACK:
                    link.close()
                    raise ConnectionError("rank 0 refused the hello")
                self._conn = link
                return
            except (OSError, ValueError, EOFError, TimeoutError, ConnectionError, pickle.UnpicklingError) as e:
                last = e  # not published yet / a stale file / rank 0 still binding
                if time.monotonic() > deadline:
                    raise TimeoutError(f"control plane: rank {self.rank} could not reach rank 0 ({last})") from e
                time.sleep(0.05)

    # -------------------------------------------------------------- collectives
    def allgather(self, obj) -> list:
        """Every rank's object, in rank order, on every rank.  A rank that does not
        answer within the timeout raises TimeoutError naming it."""
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            vals = [obj] + [c.recv(self.timeout) for c in self._peers]
            for c in self._peers:
                c.send(vals)
            return vals
        self._conn.send(obj)
        return self._conn.recv(self.timeout)

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
