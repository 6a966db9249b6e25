"""Host-side process group for multi-rank runs, without torch.

One process per GPU loads librspl.so (the system ROCm HIP runtime).  Importing torch into the same
process would load torch's bundled HIP runtime beside it (seen to abort at interpreter exit with a
double free), so the ranks' host control plane -- barrier, max-over-ranks timing, the rank census,
the RCCL id broadcast and host-staged all-reduces -- runs over plain TCP sockets instead: rank 0 is
the hub (MASTER_ADDR:MASTER_PORT, 127.0.0.1 by default), the other ranks connect to it.

Only data crosses the wire: length-prefixed raw byte strings (numpy float64 buffers, the RCCL id) and
JSON documents (ranks, timings, census rows); nothing received is ever executed or unpickled.  Every
collective is an all-gather through the hub, so each rank sees the contributions in rank order and
sums formed in rank order are bitwise identical on all ranks.
"""
import json
import os
import socket
import struct
import time

import numpy as np

_MAX_MSG = 1 << 31


def _send(sock, data: bytes):
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 20))
        if not chunk:
            raise ConnectionError("host group: a rank closed its connection")
        buf += chunk
    return bytes(buf)


def _recv(sock) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    if n > _MAX_MSG:
        raise ValueError(f"host group: message of {n} bytes refused")
    return _recv_exact(sock, n)


class HostGroup:
    def __init__(self, rank=None, world=None, addr=None, port=None, timeout=300.0):
        self.rank = int(os.environ.get("RANK", 0)) if rank is None else rank
        self.world = int(os.environ.get("WORLD_SIZE", 1)) if world is None else world
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("RSPL_HOSTGROUP_PORT", 0)) or int(os.environ.get("MASTER_PORT", 29500))
            if "RSPL_HOSTGROUP_PORT" not in os.environ and "TORCHELASTIC_RUN_ID" in os.environ:
                port += 1  # under torch.distributed.run the launcher's own store holds MASTER_PORT
        self.timeout = timeout
        self.peers = {}
        self.hub = None
        if self.world == 1:
            return
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(timeout)
            try:
                while len(self.peers) < self.world - 1:
                    conn, _ = srv.accept()
                    conn.settimeout(timeout)
                    r = json.loads(_recv(conn))
                    if not isinstance(r, int) or not 0 < r < self.world or r in self.peers:
                        conn.close()
                        raise ConnectionError(f"host group: unexpected rank hello {r!r}")
                    self.peers[r] = conn
            except socket.timeout:
                raise TimeoutError(f"host group: {len(self.peers) + 1} of {self.world} ranks came up") from None
            finally:
                srv.close()
        else:
            t0 = time.time()
            while True:
                try:
                    self.hub = socket.create_connection((addr, port), timeout=timeout)
                    break
                except OSError:
                    if time.time() - t0 > timeout:
                        raise TimeoutError(f"host group: rank {self.rank} cannot reach rank 0 at {addr}:{port}")
                    time.sleep(0.1)
            self.hub.settimeout(timeout)
            _send(self.hub, json.dumps(self.rank).encode())

    def all_gather_bytes(self, data: bytes):
        """[bytes of rank 0, bytes of rank 1, ...] on every rank."""
        if self.world == 1:
            return [bytes(data)]
        if self.rank == 0:
            rows = [bytes(data)] + [b""] * (self.world - 1)
            for r, conn in self.peers.items():
                rows[r] = _recv(conn)
            for conn in self.peers.values():
                for row in rows:
                    _send(conn, row)
            return rows
        _send(self.hub, bytes(data))
        return [_recv(self.hub) for _ in range(self.world)]

    def all_gather(self, obj):
        """JSON-serialisable obj of every rank, in rank order."""
        return [json.loads(b) for b in self.all_gather_bytes(json.dumps(obj).encode())]

    def barrier(self):
        self.all_gather_bytes(b"")

    def allreduce_max(self, x: float) -> float:
        return max(self.all_gather(float(x)))

    def broadcast_bytes(self, data: bytes, src=0) -> bytes:
        return self.all_gather_bytes(data if self.rank == src else b"")[src]

    def allreduce_sum_(self, arr: np.ndarray):
        """In-place float64 sum over the ranks, formed in rank order (identical bits on every rank)."""
        a = np.ascontiguousarray(arr, np.float64)
        rows = [np.frombuffer(b, np.float64) for b in self.all_gather_bytes(a.tobytes())]
        if any(r.size != a.size for r in rows):
            raise ValueError("host group: all-reduce of arrays of different sizes")
        acc = rows[0].copy()
        for r in rows[1:]:
            acc += r
        arr[...] = acc.reshape(arr.shape)
        return arr

    def close(self):
        for c in list(self.peers.values()) + ([self.hub] if self.hub else []):
            try:
                c.close()
            except OSError:
                pass
        self.peers, self.hub = {}, None
