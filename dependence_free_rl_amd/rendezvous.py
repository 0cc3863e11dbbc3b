"""Torch-free rendezvous for a one-process-per-GPU job on one node.

The job's only data-path exchange is RCCL inside libxylo_hip.so (the gradient
all-reduce).  Before RCCL exists, rank 0's 128-byte ``ncclUniqueId`` has to
reach every rank; the benchmark also needs a barrier and a max-over-ranks of
its wall time.  Those three host steps go over a star of plain TCP sockets
(rank 0 listens), so no framework with its own bundled HIP / RCCL runtime is
ever loaded into the process (torch ships libamdhip64 / librccl under the same
sonames as /opt/rocm; a process that loaded torch first would make
libxylo_hip bind those copies instead).

Address: MASTER_ADDR (default 127.0.0.1); port: XH_RDZV_PORT, else
MASTER_PORT + 1 (torch.distributed.run's own store listens on MASTER_PORT).
"""
import os
import socket
import struct
import time


def _send(sock, payload):
    sock.sendall(struct.pack("<Q", len(payload)) + payload)


def _recv_exact(sock, n):
    out = bytearray()
    while len(out) < n:
        chunk = sock.recv(n - len(out))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        out += chunk
    return bytes(out)


def _recv(sock):
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class Rendezvous:
    """Star rendezvous: rank 0 accepts world-1 connections."""

    def __init__(self, rank, world, addr=None, port=None, timeout=300.0):
        self.rank, self.world = rank, world
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("XH_RDZV_PORT") or
                       int(os.environ.get("MASTER_PORT", "29500")) + 1)
        self.peers = []  # rank 0: sockets of ranks 1..world-1 in rank order
        self.sock = None
        if world == 1:
            return
        deadline = time.monotonic() + timeout
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            srv.settimeout(timeout)
            by_rank = {}
            try:
                while len(by_rank) < world - 1:
                    conn, _ = srv.accept()
                    conn.settimeout(timeout)
                    (r,) = struct.unpack("<i", _recv_exact(conn, 4))
                    if r <= 0 or r >= world or r in by_rank:
                        conn.close()
                        raise RuntimeError("rendezvous: unexpected rank %d" % r)
                    by_rank[r] = conn
            finally:
                srv.close()
            self.peers = [by_rank[r] for r in range(1, world)]
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.2)
            s.settimeout(timeout)
            s.sendall(struct.pack("<i", rank))
            self.sock = s

    def broadcast(self, payload=None):
        """Rank 0's bytes to every rank (returned on all)."""
        if self.world == 1:
            return payload
        if self.rank == 0:
            for p in self.peers:
                _send(p, payload)
            return payload
        return _recv(self.sock)

    def gather(self, payload):
        """Every rank's bytes, in rank order, on rank 0 (None elsewhere)."""
        if self.world == 1:
            return [payload]
        if self.rank == 0:
            return [payload] + [_recv(p) for p in self.peers]
        _send(self.sock, payload)
        return None

    def allreduce_max(self, value):
        """max over ranks of a float, returned on every rank."""
        vals = self.gather(struct.pack("<d", float(value)))
        out = None
        if self.rank == 0:
            out = struct.pack("<d", max(struct.unpack("<d", v)[0] for v in vals))
        return struct.unpack("<d", self.broadcast(out))[0]

    def barrier(self):
        self.gather(b"")
        self.broadcast(b"")

    def close(self):
        for p in self.peers:
            p.close()
        if self.sock:
            self.sock.close()
        self.peers, self.sock = [], None
