"""Loopback-UDP scenarios for SalamanderPacketConn (extras/obfs/conn.go semantics).

Shared by the CPU-emulated tier (tests/emu/run_case.py conn) and the GPU tier
(tests/test_gpu_parity.py).  Wire bytes are checked against the oracle
(oracle/salamander_ref.py); the reference's own conn behaviour being checked is
cited per step.
"""
import errno
import socket

import numpy as np

from hysteria_amd.conn import SalamanderPacketConn, _sockaddr
from hysteria_amd.salamander import SalamanderObfuscator
from oracle import salamander_ref as ref

PSK = b"conn_test_password"


def _udp():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    s.settimeout(10.0)
    return s


def _payload(rng, n):
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes()


def run_conn_scenarios(device: int = 0, batch: int = 64, n_batch: int = 200):
    rng = np.random.default_rng(7)
    sa, sb, raw = _udp(), _udp(), _udp()
    oa, ob = SalamanderObfuscator(PSK, device), SalamanderObfuscator(PSK, device)
    oa.seed(11)
    ca, cb = SalamanderPacketConn(sa, oa, batch=batch), SalamanderPacketConn(sb, ob, batch=batch)
    a_addr, b_addr, r_addr = ca.local_addr(), cb.local_addr(), raw.getsockname()
    try:
        # WriteTo -> ReadFrom round trip (conn.go:73-99)
        for n in (1, 9, 100, 1200, 2040):
            p = _payload(rng, n)
            assert ca.write_to(p, b_addr) == n
            got, addr = cb.read_from()
            assert got == p and addr == a_addr, n

        # wire bytes = salt || p ^ BLAKE2b-256(PSK||salt) (salamander.go:59-72)
        for n in (0, 1, 31, 32, 33, 1350, 2040):
            p = _payload(rng, n)
            ca.write_to(p, r_addr)
            wire, addr = raw.recvfrom(4096)
            assert addr == a_addr and len(wire) == n + 8
            assert wire == ref.obfuscate(PSK, p, wire[:8], n + 8), n

        # a zero-length payload goes out as an 8-byte datagram, which Deobfuscate
        # rejects (len <= 8, salamander.go:75-77): the reader drops it and reads on
        ca.write_to(b"", b_addr)
        mark = _payload(rng, 77)
        ca.write_to(mark, b_addr)
        assert cb.read_from()[0] == mark

        # > 2040 bytes: Obfuscate returns 0 and WriteTo sends an EMPTY datagram,
        # still reporting len(p) (conn.go:92-98) ...
        big = _payload(rng, 2041)
        assert ca.write_to(big, r_addr) == 2041
        wire, _ = raw.recvfrom(4096)
        assert wire == b""
        # ... and ReadFrom returns an empty read for it (n <= 0 branch, conn.go:77-80)
        assert ca.write_to(big, b_addr) == 2041
        got, addr = cb.read_from()
        assert got == b"" and addr == a_addr

        # invalid datagrams are dropped and the read goes on (conn.go:86)
        raw.sendto(b"12345", b_addr)
        raw.sendto(b"12345678", b_addr)
        p = _payload(rng, 200)
        raw.sendto(ref.obfuscate(PSK, p, b"\x01" * 8, 208), b_addr)   # too big for a 100-byte buffer
        q = _payload(rng, 60)
        raw.sendto(ref.obfuscate(PSK, q, b"\x02" * 8, 68), b_addr)
        got, addr = cb.read_from(100)
        assert got == q and addr == r_addr
        # a datagram from the oracle side deobfuscates on the GPU side
        raw.sendto(ref.obfuscate(PSK, p, b"saltsalt", 208), b_addr)
        assert cb.read_from()[0] == p

        # batched: WriteBatch -> oracle on the wire
        lens = [int(x) for x in rng.integers(0, 2100, n_batch)]
        lens[:4] = [0, 2040, 2041, 9]
        pays = [_payload(rng, n) for n in lens]
        sent = 0
        for i in range(0, n_batch, 32):   # stay inside the loopback socket buffer
            grp = pays[i:i + 32]
            sent += ca.write_batch([(p, r_addr) for p in grp])
            for p in grp:
                wire, addr = raw.recvfrom(4096)
                assert addr == a_addr
                if len(p) > 2040:
                    assert wire == b""
                else:
                    assert wire == ref.obfuscate(PSK, p, wire[:8], len(p) + 8)
        assert sent == n_batch

        # batched: WriteBatch -> ReadBatch; invalid datagrams (the 8-byte salt-only
        # one of an empty payload, junk) are dropped, and an empty datagram (the
        # > 2040-byte quirk) is a 0-byte entry, as ReadFrom returns it (conn.go:77-80)
        def seen(p):
            return p if len(p) <= 2040 else b""
        expect = [seen(p) for p in pays if len(p) >= 1]
        got = []
        for i in range(0, n_batch, 32):
            grp = pays[i:i + 32]
            assert ca.write_batch([(p, b_addr) for p in grp]) == len(grp)
            raw.sendto(b"x" * 8, b_addr)   # junk between groups
            want = sum(1 for p in grp if len(p) >= 1)
            have = 0
            while have < want:
                msgs = cb.read_batch(64)
                for m, addr in msgs:
                    assert addr == a_addr
                got.extend(m for m, _ in msgs)
                have += len(msgs)
        assert got == expect

        # ReadBatch takes oracle-made datagrams too
        qs = [_payload(rng, int(n)) for n in rng.integers(9, 1500, 20)]
        for j, q in enumerate(qs):
            raw.sendto(ref.obfuscate(PSK, q, bytes([j]) * 8, len(q) + 8), b_addr)
        got = []
        while len(got) < len(qs):
            got += [m for m, _ in cb.read_batch(64)]
        assert got == qs

        # SetReadDeadline: an idle read times out
        cb.settimeout(0.2)
        try:
            cb.read_from()
            raise AssertionError("read did not time out")
        except TimeoutError:
            pass
        try:
            cb.read_batch(8)
            raise AssertionError("read_batch did not time out")
        except TimeoutError:
            pass
    finally:
        ca.close()
        cb.close()
        raw.close()
        oa.close()
        ob.close()


def run_coalesce_scenarios(device: int = 0, writers: int = 8, per_writer: int = 300, readers: int = 4,
                           max_batch: int = 64, max_wait_us: int = 200, idle_timeout: float = 3.0):
    """Coalescing mode (hyobfs_conn_set_coalescing): many threads calling the
    per-datagram WriteTo / ReadFrom of one connection share GPU batches.  Every
    datagram arrives exactly once with the reference's per-datagram semantics
    (conn.go:73-99): wire bytes equal the oracle's, invalid datagrams are
    dropped, an empty datagram is a 0-byte read, a > 2040-byte payload goes out
    as an empty datagram, the read deadline holds."""
    import threading
    rng = np.random.default_rng(17)
    sa, sb, raw = _udp(), _udp(), _udp()
    for s in (sa, sb, raw):
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 32 << 20)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 32 << 20)
    oa, ob = SalamanderObfuscator(PSK, device), SalamanderObfuscator(PSK, device)
    ca, cb = SalamanderPacketConn(sa, oa, batch=max_batch), SalamanderPacketConn(sb, ob, batch=max_batch)
    ca.set_coalescing(max_batch, max_wait_us)
    cb.set_coalescing(max_batch, max_wait_us)
    a_addr, b_addr, r_addr = ca.local_addr(), cb.local_addr(), raw.getsockname()
    try:
        # the batched calls belong to the coalescer now
        for call in (lambda: ca.write_batch([(b"x", b_addr)]), lambda: cb.read_batch(4)):
            try:
                call()
                raise AssertionError("batched call allowed in coalescing mode")
            except OSError as e:
                assert e.errno == errno.EBUSY

        # many writers -> many readers: each payload carries (writer, seq); lengths
        # include 0 (an 8-byte datagram the reader drops) and 2041 (an empty datagram)
        def payload(w, i):
            n = [0, 1, 9, 100, 1200, 2040, 2041, 31][i % 8] if i < 16 else 16 + (w * 131 + i * 17) % 1400
            head = bytes([w]) + i.to_bytes(3, "little")
            return (head * (n // 4 + 1))[:n]
        expect = {}
        for w in range(writers):
            for i in range(per_writer):
                p = payload(w, i)
                if len(p) == 0:
                    continue                      # salt-only datagram: dropped by the reader
                key = p if len(p) <= 2040 else b""
                expect[key] = expect.get(key, 0) + 1
        total = sum(expect.values())
        got, lock = {}, threading.Lock()
        cb.settimeout(idle_timeout)   # readers left over once every datagram arrived end on this

        def reader():
            while True:
                with lock:
                    if sum(got.values()) >= total:
                        return
                try:
                    m, addr = cb.read_from()
                except TimeoutError:
                    return
                assert addr == a_addr
                with lock:
                    got[m] = got.get(m, 0) + 1

        def writer(w):
            for i in range(per_writer):
                p = payload(w, i)
                assert ca.write_to(p, b_addr) == len(p)

        rt = [threading.Thread(target=reader) for _ in range(readers)]
        wt = [threading.Thread(target=writer, args=(w,)) for w in range(writers)]
        for t in rt + wt:
            t.start()
        for t in wt:
            t.join()
        ca.flush()
        for t in rt:
            t.join()
        if got != expect:
            extra = {(k[:8].hex(), len(k)): (v, expect.get(k)) for k, v in got.items() if expect.get(k) != v}
            miss = {(k[:8].hex(), len(k)): (v, got.get(k)) for k, v in expect.items() if got.get(k) != v}
            raise AssertionError((sum(got.values()), total, list(extra.items())[:5], list(miss.items())[:5]))
        st = ca.stats()
        assert st["accepted"] == writers * per_writer and st["tx_errors"] == 0 and st["tx_batches"] >= 1

        # wire bytes against the oracle (coalescing writer -> plain socket)
        sent = [_payload(rng, n) for n in (0, 1, 33, 1200, 2040, 2041)]
        for p in sent:
            ca.write_to(p, r_addr)
        ca.flush()
        seen = []
        for _ in sent:
            wire, addr = raw.recvfrom(4096)
            assert addr == a_addr
            seen.append(wire)
        for p in sent:   # one batch: sendmmsg keeps the order
            wire = seen.pop(0)
            if len(p) > 2040:
                assert wire == b""
            else:
                assert wire == ref.obfuscate(PSK, p, wire[:8], len(p) + 8), len(p)

        # plain socket -> coalescing reader: junk dropped, empty datagram = 0-byte read
        raw.sendto(b"12345678", b_addr)
        q = _payload(rng, 60)
        raw.sendto(ref.obfuscate(PSK, q, b"\x02" * 8, 68), b_addr)
        raw.sendto(b"", b_addr)
        assert cb.read_from() == (q, r_addr)
        assert cb.read_from() == (b"", r_addr)
        assert cb.stats()["rx_dropped"] >= 1
        # SetReadDeadline: an idle read times out
        cb.settimeout(0.2)
        try:
            cb.read_from()
            raise AssertionError("read did not time out")
        except TimeoutError:
            pass
    finally:
        ca.close()
        cb.close()
        raw.close()
        oa.close()
        ob.close()


def run_lifecycle_scenarios(device: int = 0, n: int = 200, max_batch: int = 64, max_wait_us: int = 100000):
    """Close() and error paths of both modes (include/hyobfs_conn.h):
      * close() without flush() on a coalescing connection still sends every
        datagram write_to accepted (the flusher runs before the socket closes);
      * close() while other threads are blocked in read_from / write_to wakes
        them with EBADF (coalescing and plain mode; conn.go:101-103 Close of the
        inner conn unblocks a pending ReadFrom);
      * a send that fails after write_to queued its datagram (coalescing) is
        reported by the NEXT write_to as -1 with that errno, then cleared.
    A long max_wait_us keeps the datagrams queued until close() or flush()."""
    import threading
    import time
    rng = np.random.default_rng(23)
    oa = SalamanderObfuscator(PSK, device)
    raw = _udp()
    raw.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    r_addr = raw.getsockname()
    try:
        # 1. accepted but not flushed: close() sends them
        ca = SalamanderPacketConn(_udp(), oa, batch=max_batch)
        ca.set_coalescing(max_batch, max_wait_us)
        a_addr = ca.local_addr()
        sent = [_payload(rng, 1 + (i * 37) % 1300) for i in range(n)]
        for p in sent:
            assert ca.write_to(p, r_addr) == len(p)
        ca.close()
        got = []
        raw.settimeout(10.0)
        for _ in sent:
            wire, addr = raw.recvfrom(4096)
            assert addr == a_addr
            got.append(ref.deobfuscate(PSK, wire))
        assert sorted(got) == sorted(sent)

        # 2. close() wakes blocked readers (and a writer blocked on a full queue)
        for coalescing in (True, False):
            cb = SalamanderPacketConn(_udp(), oa, batch=max_batch)
            if coalescing:
                cb.set_coalescing(max_batch, max_wait_us)
            errs = []

            def blocked_read():
                try:
                    cb.read_from()
                    errs.append("returned")
                except OSError as e:
                    errs.append(e.errno)
            ts = [threading.Thread(target=blocked_read) for _ in range(3 if coalescing else 1)]
            for t in ts:
                t.start()
            time.sleep(0.3)
            cb.close()
            for t in ts:
                t.join(20)
                assert not t.is_alive(), "reader still blocked after close()"
            assert errs == [errno.EBADF] * len(ts), (coalescing, errs)

        # 3. a failed send after write_to returned: reported by the next write_to.
        # A limited broadcast without SO_BROADCAST fails in sendmmsg with EACCES.
        cc = SalamanderPacketConn(_udp(), oa, batch=max_batch)
        cc.set_coalescing(max_batch, 50)
        assert cc.write_to(b"to nowhere", ("255.255.255.255", r_addr[1])) == 10
        cc.flush()
        assert cc.stats()["tx_errors"] == 1
        try:
            cc.write_to(b"next", r_addr)
            raise AssertionError("send error not reported")
        except OSError as e:
            assert e.errno == errno.EACCES, e
        assert cc.write_to(b"after", r_addr) == 5   # reported once, then cleared
        cc.flush()
        wire, _ = raw.recvfrom(4096)
        assert ref.deobfuscate(PSK, wire) == b"after"
        cc.close()

        # 4. free without close (a Go finalizer on a dropped connection): the
        # connection owns the descriptor it was given, so free closes it -- and a
        # coalescing one sends what write_to accepted before the socket goes
        _free_unclosed_closes_fd(oa, r_addr, raw, max_batch)
    finally:
        raw.close()
        oa.close()


def run_rx_gpu_failure_scenario(device: int = 0, max_batch: int = 16):
    """A receive batch whose GPU step fails (CPU tier only: tests/emu/hip_emu.h
    HYEMU_FAIL_EVENTS_FROM=5 fails every wait of the coalescing connection's receive
    queue).  The reference drops only datagrams Deobfuscate rejects (conn.go:81-86); a
    device failure is an error, not invalid packets: ReadFrom raises EIO (once per
    failed batch, after the datagrams queued before it) and rx_dropped stays 0."""
    import time
    rng = np.random.default_rng(31)
    osend, orecv = SalamanderObfuscator(PSK, device), SalamanderObfuscator(PSK, device)
    raw = _udp()
    cb = SalamanderPacketConn(_udp(), orecv, batch=max_batch)
    try:
        cb.set_coalescing(max_batch, 50)   # its send queue: events 1-4, receive queue: 5-8
        b_addr = cb.local_addr()
        for rnd in range(2):
            for _ in range(3):
                p = _payload(rng, 100)
                wire = bytearray(108)
                assert osend.obfuscate(p, wire, salt=rng.bytes(8)) == 108
                raw.sendto(bytes(wire), b_addr)
            time.sleep(0.2)   # one receive batch
            try:
                cb.read_from()
                raise AssertionError("a failed receive batch was not reported")
            except OSError as e:
                assert e.errno == errno.EIO, e
            assert cb.stats()["rx_dropped"] == 0, cb.stats()
    finally:
        cb.close()
        raw.close()
        osend.close()
        orecv.close()


def run_tx_gpu_failure_scenario(device: int = 0, max_batch: int = 16):
    """A send batch whose GPU step fails (CPU tier only: HYEMU_FAIL_EVENTS_FROM=1 fails
    every event of the connection's queues, the sleep-polling wait's hipEventQuery
    included).  WriteTo had already returned len(p): the datagram is counted as a tx
    error and is not sent (nothing unobfuscated reaches the socket), and the next
    WriteTo raises EIO once -- the reference returns the error of conn.go:93-98 to the
    caller whose datagram failed, which a queued send cannot do (include/hyobfs_conn.h)."""
    oa = SalamanderObfuscator(PSK, device)
    raw = _udp()
    raw.settimeout(0.5)
    r_addr = raw.getsockname()
    ca = SalamanderPacketConn(_udp(), oa, batch=max_batch)
    try:
        ca.set_coalescing(max_batch, 50)
        assert ca.write_to(b"x" * 100, r_addr) == 100
        ca.flush()
        assert ca.stats()["tx_errors"] == 1, ca.stats()
        try:
            ca.write_to(b"y", r_addr)
            raise AssertionError("a failed send batch was not reported")
        except OSError as e:
            assert e.errno == errno.EIO, e
        try:
            raw.recvfrom(4096)
            raise AssertionError("a datagram whose GPU step failed reached the socket")
        except socket.timeout:
            pass
    finally:
        ca.close()
        raw.close()
        oa.close()


def _free_unclosed_closes_fd(oa, r_addr, raw, max_batch):
    """hyobfs_conn_wrap on a dup'd descriptor, hyobfs_conn_free with no
    hyobfs_conn_close first (include/hyobfs_conn.h): the fd leaves the process's
    descriptor table (fstat fails with EBADF), the caller's own socket is untouched,
    and the coalescer's accepted datagrams are on the wire."""
    import ctypes
    import os
    lib = oa._lib
    for coalescing in (False, True):
        s = _udp()
        fd = os.dup(s.fileno())
        h = ctypes.c_void_p()
        assert lib.hyobfs_conn_wrap(fd, oa._h, max_batch, ctypes.byref(h)) == 0
        if coalescing:
            assert lib.hyobfs_conn_set_coalescing(h, max_batch, 100000) == 0
            sa = _sockaddr(r_addr, socket.AF_INET)
            assert lib.hyobfs_conn_write_to(h, b"freed but sent", 14, sa, len(sa)) == 14
        os.fstat(fd)                      # open while wrapped
        lib.hyobfs_conn_free(h)
        try:
            os.fstat(fd)
            raise AssertionError(f"fd {fd} still open after hyobfs_conn_free (coalescing={coalescing})")
        except OSError as e:
            assert e.errno == errno.EBADF, e
        os.fstat(s.fileno())              # the caller's socket is its own
        if coalescing:
            wire, _ = raw.recvfrom(4096)
            assert ref.deobfuscate(PSK, wire) == b"freed but sent"
        s.close()


def run_deadline_scenarios(device: int = 0, max_batch: int = 16):
    """SetReadDeadline / SetWriteDeadline (conn.go:109-119, net.Conn semantics) in
    plain and coalescing mode: an idle read times out at its deadline; moving the
    deadline into the past wakes a read that is blocked right now; clearing it
    (None) lets reads block again; a passed write deadline fails write_to; data
    that is there is read before the deadline matters."""
    import threading
    import time
    oa = SalamanderObfuscator(PSK, device)
    raw = _udp()
    try:
        for coalescing in (False, True):
            c = SalamanderPacketConn(_udp(), oa, batch=max_batch)
            if coalescing:
                c.set_coalescing(max_batch, 100)
            addr = c.local_addr()
            # 1. an idle read ends at its deadline
            t0 = time.time()
            c.set_read_deadline(t0 + 0.3)
            try:
                c.read_from()
                raise AssertionError("read did not time out")
            except TimeoutError:
                pass
            dt = time.time() - t0
            assert 0.25 <= dt < 5.0, (coalescing, dt)
            # 2. a datagram that is there is read while the deadline is in the future
            c.set_read_deadline(time.time() + 5.0)
            raw.sendto(ref.obfuscate(PSK, b"hello", b"\x01" * 8, 13), addr)
            assert c.read_from() == (b"hello", raw.getsockname())
            # 3. a read blocked with no deadline wakes when the deadline moves into the past
            c.set_read_deadline(None)
            got = []

            def blocked():
                try:
                    c.read_from()
                    got.append("returned")
                except TimeoutError:
                    got.append("timeout")
            th = threading.Thread(target=blocked)
            th.start()
            time.sleep(0.3)
            assert th.is_alive(), "read returned without data or deadline"
            c.set_read_deadline(time.time() - 1.0)
            th.join(10)
            assert not th.is_alive() and got == ["timeout"], (coalescing, got)
            # 4. a passed write deadline fails the write; clearing it lets writes through
            c.set_write_deadline(time.time() - 1.0)
            try:
                c.write_to(b"late", raw.getsockname())
                raise AssertionError("write after the deadline succeeded")
            except TimeoutError:
                pass
            c.set_deadline(None)
            assert c.write_to(b"on time", raw.getsockname()) == 7
            if coalescing:
                c.flush()
            wire, _ = raw.recvfrom(4096)
            assert ref.deobfuscate(PSK, wire) == b"on time"
            c.close()
    finally:
        raw.close()
        oa.close()


def run_close_race_scenarios(device: int = 0, threads: int = 8, per_writer: int = 1500, run_s: float = 0.4):
    """Close racing the per-datagram calls (include/hyobfs_conn.h, hyobfs_conn_close):
    `threads` threads (half writers, half readers) call write_to / read_from in a
    loop while the main thread closes the connection, in plain and coalescing
    mode.  Every thread must leave with EBADF (Go: net.ErrClosed) -- never a crash
    or a use of freed memory (the CPU tier runs this under AddressSanitizer) --
    every call after close must fail with EBADF, and every datagram a write_to
    accepted must reach the wire (close sends what the coalescer holds; a write
    that races close is refused or sent, never dropped)."""
    import threading
    import time
    sink, pump = _udp(), _udp()
    sink.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 32 << 20)
    s_addr = sink.getsockname()
    ob = SalamanderObfuscator(PSK, device)
    valid = [ref.obfuscate(PSK, bytes([i]) * (20 + i), bytes([i]) * 8, 28 + i) for i in range(8)]
    try:
        for coalescing in (False, True):
            c = SalamanderPacketConn(_udp(), ob, batch=64)
            if coalescing:
                c.set_coalescing(64, 200)
            c_addr = c.local_addr()
            stop_pump = threading.Event()
            accepted = [0] * threads
            errs = []

            def pumper():   # valid datagrams into the connection for the readers
                i = 0
                while not stop_pump.is_set():
                    try:
                        pump.sendto(valid[i % len(valid)], c_addr)
                    except OSError:
                        pass
                    i += 1
                    if i % 64 == 0:
                        time.sleep(0.001)

            def worker(t):
                write = t % 2 == 0
                try:
                    while True:
                        if write:
                            p = bytes([t]) + accepted[t].to_bytes(4, "little") + b"w" * 40
                            assert c.write_to(p, s_addr) == len(p)
                            accepted[t] += 1
                            if accepted[t] >= per_writer:
                                time.sleep(0.0005)
                        else:
                            m, _ = c.read_from()
                            assert m in [ref.deobfuscate(PSK, v) for v in valid], m
                except OSError as e:
                    if e.errno != errno.EBADF:
                        errs.append((t, repr(e)))
                        return
                except BaseException as e:   # noqa: BLE001 -- reported below
                    errs.append((t, repr(e)))
                    return
                # after close: every further call fails the same way
                for _ in range(3):
                    try:
                        c.write_to(b"late", s_addr) if write else c.read_from()
                        errs.append((t, "call after close succeeded"))
                    except OSError as e:
                        if e.errno != errno.EBADF:
                            errs.append((t, repr(e)))

            pt = threading.Thread(target=pumper)
            ws = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
            pt.start()
            for w in ws:
                w.start()
            time.sleep(run_s)
            c.close()
            for w in ws:
                w.join(30)
                assert not w.is_alive(), (coalescing, "a thread is still inside a call after close()")
            stop_pump.set()
            pt.join(10)
            assert not errs, (coalescing, errs[:5])
            # the main thread's calls after close
            for call in (lambda: c.write_to(b"x", s_addr), lambda: c.read_from(), lambda: c.flush(),
                         lambda: c.set_read_deadline(None), lambda: c.set_write_deadline(None),
                         lambda: c.set_coalescing(16, 10), lambda: c.close()):
                try:
                    call()
                    raise AssertionError((coalescing, "call after close succeeded"))
                except OSError as e:
                    assert e.errno == errno.EBADF, (coalescing, e)
            # every accepted datagram is on the wire
            want = sum(accepted)
            assert want > 0
            sink.settimeout(2.0)
            got = 0
            while got < want:
                try:
                    wire, addr = sink.recvfrom(4096)
                except TimeoutError:
                    break
                assert addr == c_addr
                assert len(ref.deobfuscate(PSK, wire)) == 45
                got += 1
            assert got == want, (coalescing, got, want)
            del c
    finally:
        sink.close()
        pump.close()
        ob.close()
