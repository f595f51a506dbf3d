"""Salamander packet connection -- the ``obfsPacketConn`` wrapper on MI355X.

Mirrors ``extras/obfs/conn.go`` over a UDP socket, through
``include/hyobfs_conn.h``:

=========================================  ==========================================
reference (Go)                             here
=========================================  ==========================================
``WrapPacketConnSalamander(conn, psk)``    ``wrap_packet_conn_salamander(sock, psk)``
(salamander.go:51-57, conn.go:56-71)       / ``SalamanderPacketConn(sock, obfuscator)``
``ReadFrom(p)`` (conn.go:73-88)            ``read_from(bufsize) -> (payload, addr)``
``WriteTo(p, addr)`` (conn.go:90-99)       ``write_to(p, addr) -> len(p)``
``Close()`` (conn.go:101-103)              ``close()`` (closes the socket)
``LocalAddr()`` (conn.go:105-107)          ``local_addr()``
``Set{,Read,Write}Deadline``               ``set_deadline(t)`` / ``set_read_deadline(t)`` /
(conn.go:109-119)                          ``set_write_deadline(t)`` (absolute ``time.time()``
                                           seconds, None = none), or ``settimeout(seconds)``
``SetReadBuffer`` / ``SetWriteBuffer``     ``set_read_buffer`` / ``set_write_buffer``
(new) batched receive / send               ``read_batch(n)`` / ``write_batch(msgs)``
(new) coalescing per-datagram calls        ``set_coalescing(max_batch, max_wait_us)``,
                                           ``flush()``, ``stats()``
=========================================  ==========================================

Kept reference behaviour: ``read_from`` drops datagrams that fail to
deobfuscate and reads again; ``write_to`` of a payload longer than 2040 bytes
sends an EMPTY datagram and still returns ``len(p)``.  A timeout raises
``TimeoutError`` (the Go deadline error); other socket errors raise ``OSError``.
"""
from __future__ import annotations

import ctypes
import errno
import os
import socket
import struct
import threading

from . import _lib
from ._lib import HyobfsDgram, check
from .salamander import UDP_BUFFER_SIZE, SalamanderObfuscator

_AF_INET6_LEN = 28
_AF_INET_LEN = 16


def _sockaddr(addr, family: int) -> bytes:
    """struct sockaddr_in / sockaddr_in6 for a Python socket address."""
    if family == socket.AF_INET:
        host, port = addr
        return struct.pack("=H", socket.AF_INET) + struct.pack("!H", port) + socket.inet_pton(
            socket.AF_INET, host) + b"\0" * 8
    if family == socket.AF_INET6:
        host, port = addr[0], addr[1]
        flow = addr[2] if len(addr) > 2 else 0
        scope = addr[3] if len(addr) > 3 else 0
        return (struct.pack("=H", socket.AF_INET6) + struct.pack("!HI", port, flow)
                + socket.inet_pton(socket.AF_INET6, host) + struct.pack("=I", scope))
    raise ValueError(f"unsupported address family {family}")


def _pyaddr(raw: bytes):
    """Python socket address of a struct sockaddr; None for an empty one."""
    if len(raw) < 2:
        return None
    fam = struct.unpack_from("=H", raw)[0]
    if fam == socket.AF_INET:
        port = struct.unpack_from("!H", raw, 2)[0]
        return socket.inet_ntop(socket.AF_INET, raw[4:8]), port
    if fam == socket.AF_INET6:
        port, flow = struct.unpack_from("!HI", raw, 2)
        scope = struct.unpack_from("=I", raw, 24)[0]
        return socket.inet_ntop(socket.AF_INET6, raw[8:24]), port, flow, scope
    return raw


def _check_conn(status: int, what: str) -> None:
    """A status call on the connection: HYOBFS_ERR_CLOSED is Go's net.ErrClosed."""
    if status == _lib.HYOBFS_ERR_CLOSED:
        raise OSError(errno.EBADF, f"{what}: use of closed connection")
    check(status, what)


def _raise_errno(what: str):
    e = ctypes.get_errno()
    if e in (errno.EAGAIN, errno.EWOULDBLOCK, errno.ETIMEDOUT):
        raise TimeoutError(e, f"{what}: i/o timeout")
    raise OSError(e, f"{what}: {os.strerror(e)}")


class SalamanderPacketConn:
    """obfsPacketConn over a bound UDP socket; the obfuscator runs on the GPU.

    The connection takes over the socket (``close()`` closes it, like the
    reference's Close).  ``batch`` bounds the datagrams per batched call.
    """

    def __init__(self, sock: socket.socket, obfuscator: SalamanderObfuscator, batch: int = 1024):
        if sock.type != socket.SOCK_DGRAM:
            raise ValueError("need a UDP (SOCK_DGRAM) socket")
        self._lib = _lib.load()
        self._sock = sock
        self._family = sock.family
        self._ob = obfuscator          # keeps the context alive
        self._timeout = sock.gettimeout()
        sock.setblocking(True)         # timeouts go through SO_RCVTIMEO, the fd stays blocking
        if self._timeout is not None:
            self.settimeout(self._timeout)
        h = ctypes.c_void_p()
        self._closed = False
        self._close_lock = threading.Lock()
        check(self._lib.hyobfs_conn_wrap(sock.fileno(), obfuscator._h, batch, ctypes.byref(h)), "hyobfs_conn_wrap")
        self._h = h
        self.batch = batch

    # ------------------------------------------------------------ lifecycle
    def close(self) -> None:
        """Close (conn.go:101-103): the C side sends what a coalescing connection
        accepted, wakes blocked calls and closes the socket.  Calls made during or
        after close raise OSError(EBADF) (Go: net.ErrClosed); the handle is freed
        only when this object goes away (hyobfs_conn_free), so threads still
        inside a call never touch freed memory.  A second close raises too."""
        with self._close_lock:         # one closer detaches the socket; the others get EBADF
            if self._closed:
                raise OSError(errno.EBADF, "close: use of closed connection")
            self._closed = True
            self._sock.detach()        # the C side owns and closes the fd
        _check_conn(self._lib.hyobfs_conn_close(self._h), "close")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        if not self._closed:
            self.close()

    def __del__(self):
        h = getattr(self, "_h", None)
        if not h:
            return
        try:
            if not self._closed:
                self.close()
        except Exception:
            pass
        self._h = None
        self._lib.hyobfs_conn_free(h)   # nobody can be inside a call: this object is unreachable

    # ------------------------------------------------------------ net.PacketConn
    def local_addr(self):
        return self._sock.getsockname()

    def fileno(self) -> int:
        return self._sock.fileno()

    def settimeout(self, seconds: float | None) -> None:
        """SetDeadline as a relative timeout (None = block forever)."""
        us = 0 if seconds is None else max(1, int(seconds * 1e6))
        tv = struct.pack("ll", us // 1_000_000, us % 1_000_000)
        self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVTIMEO, tv)
        self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_SNDTIMEO, tv)
        self._timeout = seconds

    def set_read_deadline(self, t: float | None) -> None:
        """SetReadDeadline: absolute time (time.time() seconds) or None; applies to blocked reads too."""
        _check_conn(self._lib.hyobfs_conn_set_read_deadline(self._h, 0 if t is None else max(1, int(t * 1e9))),
                    "set_read_deadline")

    def set_write_deadline(self, t: float | None) -> None:
        """SetWriteDeadline: absolute time (time.time() seconds) or None."""
        _check_conn(self._lib.hyobfs_conn_set_write_deadline(self._h, 0 if t is None else max(1, int(t * 1e9))),
                    "set_write_deadline")

    def set_deadline(self, t: float | None) -> None:
        """SetDeadline: both deadlines."""
        self.set_read_deadline(t)
        self.set_write_deadline(t)

    def set_read_buffer(self, nbytes: int) -> None:
        self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, nbytes)

    def set_write_buffer(self, nbytes: int) -> None:
        self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, nbytes)

    def read_from(self, bufsize: int = UDP_BUFFER_SIZE):
        """ReadFrom (conn.go:73-88): (payload, addr) of the next valid datagram."""
        # per-call buffers: several threads may read one connection at once
        buf = ctypes.create_string_buffer(max(bufsize, 1))
        addr = ctypes.create_string_buffer(128)
        al = ctypes.c_uint32(128)
        n = self._lib.hyobfs_conn_read_from(self._h, buf, bufsize, addr, ctypes.byref(al))
        if n < 0:
            _raise_errno("read")
        return buf.raw[:n], _pyaddr(addr.raw[: al.value])

    def write_to(self, p, addr) -> int:
        """WriteTo (conn.go:90-99): returns len(p); > 2040 bytes sends an empty datagram."""
        p = bytes(p)
        sa = _sockaddr(addr, self._family)
        n = self._lib.hyobfs_conn_write_to(self._h, p or None, len(p), sa, len(sa))
        if n < 0:
            _raise_errno("write")
        return n

    # ------------------------------------------------------------ coalescing
    def set_coalescing(self, max_batch: int = 1024, max_wait_us: int = 50) -> None:
        """Serve the per-datagram write_to / read_from from GPU batches (include/hyobfs_conn.h,
        hyobfs_conn_set_coalescing): write_to returns once the datagram is queued; many
        threads may call both.  The batched calls are unavailable afterwards."""
        _check_conn(self._lib.hyobfs_conn_set_coalescing(self._h, max_batch, max_wait_us), "set_coalescing")

    def flush(self) -> None:
        """Wait until every datagram write_to accepted was handed to the socket."""
        _check_conn(self._lib.hyobfs_conn_flush(self._h), "flush")

    def stats(self) -> dict:
        out = (ctypes.c_uint64 * 6)()
        check(self._lib.hyobfs_conn_stats(self._h, out), "stats")
        return dict(zip(("accepted", "tx_batches", "tx_errors", "received", "rx_batches", "rx_dropped"), out))

    # ------------------------------------------------------------ batched
    def read_batch(self, n: int, bufsize: int = UDP_BUFFER_SIZE):
        """Up to ``n`` valid datagrams from one recvmmsg + one GPU batch (blocks for the first)."""
        n = min(n, self.batch)
        msgs = (HyobfsDgram * n)()
        bufs = ctypes.create_string_buffer(n * bufsize)
        base = ctypes.addressof(bufs)
        for i in range(n):
            msgs[i].buf = base + i * bufsize
            msgs[i].cap = bufsize
        k = self._lib.hyobfs_conn_read_batch(self._h, msgs, n)
        if k < 0:
            _raise_errno("read_batch")
        out = []
        for i in range(k):
            m = msgs[i]
            out.append((ctypes.string_at(m.buf, m.len), _pyaddr(bytes(m.addr)[: m.addrlen])))
        return out

    def write_batch(self, datagrams) -> int:
        """Send [(payload, addr), ...] with one GPU batch per ``batch`` datagrams."""
        datagrams = list(datagrams)
        n = len(datagrams)
        if n == 0:
            return 0
        msgs = (HyobfsDgram * n)()
        keep = []
        for i, (p, addr) in enumerate(datagrams):
            b = ctypes.create_string_buffer(bytes(p), max(len(p), 1))
            keep.append(b)
            msgs[i].buf = ctypes.addressof(b)
            msgs[i].len = len(p)
            sa = _sockaddr(addr, self._family)
            ctypes.memmove(msgs[i].addr, sa, len(sa))
            msgs[i].addrlen = len(sa)
        k = self._lib.hyobfs_conn_write_batch(self._h, msgs, n)
        if k < 0:
            _raise_errno("write_batch")
        return k


def wrap_packet_conn_salamander(sock: socket.socket, psk: bytes, device: int = 0,
                                batch: int = 1024) -> SalamanderPacketConn:
    """WrapPacketConnSalamander (salamander.go:51-57) on HIP device ``device``."""
    return SalamanderPacketConn(sock, SalamanderObfuscator(psk, device), batch=batch)
