// hyobfs_conn.cpp -- obfsPacketConn (extras/obfs/conn.go) over a UDP socket,
// the Salamander work on the GPU through the C ABI of include/hyobfs.h.
// See include/hyobfs_conn.h for the reference mapping and kept behaviour.
#include "../../include/hyobfs_conn.h"

#include "conn_coalesce.h"

#include <errno.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <new>
#include <vector>

namespace {
constexpr uint32_t kBuf = HYOBFS_UDP_BUFFER_SIZE;   // udpBufferSize, conn.go:10

struct Ring {   // pinned, device-mapped slots of kBuf bytes
    uint8_t* in = nullptr;
    uint8_t* out = nullptr;
    uint32_t* len = nullptr;
    uint32_t* olen = nullptr;
    uint64_t* salts = nullptr;
    uint32_t n = 0;
    bool alloc(uint32_t cnt) {
        n = cnt;
        in = static_cast<uint8_t*>(hyobfs_host_alloc((size_t)cnt * kBuf));
        out = static_cast<uint8_t*>(hyobfs_host_alloc((size_t)cnt * kBuf));
        len = static_cast<uint32_t*>(hyobfs_host_alloc((size_t)cnt * 4));
        olen = static_cast<uint32_t*>(hyobfs_host_alloc((size_t)cnt * 4));
        salts = static_cast<uint64_t*>(hyobfs_host_alloc((size_t)cnt * 8));
        return in && out && len && olen && salts;
    }
    void release() {
        hyobfs_host_free(in);
        hyobfs_host_free(out);
        hyobfs_host_free(len);
        hyobfs_host_free(olen);
        hyobfs_host_free(salts);
        in = out = nullptr;
        len = olen = nullptr;
        salts = nullptr;
    }
};
}  // namespace

struct hyobfs_conn {
    int fd = -1;
    hyobfs_salamander* ctx = nullptr;      // retained (hyobfs::ctx_retain) until the connection is freed
    std::mutex read_mu, write_mu;          // readMutex / writeMutex, conn.go:25-28
    uint8_t read_buf[kBuf];                // readBuf
    uint8_t write_buf[kBuf];               // writeBuf
    Ring rx, tx;
    std::vector<mmsghdr> rmsg, wmsg;
    std::vector<iovec> riov, wiov;
    std::vector<sockaddr_storage> raddr;
    hyobfs::Coalescer* co = nullptr;       // set: per-datagram calls go through batches
    hyobfs::Deadlines dl;                  // SetReadDeadline / SetWriteDeadline (absolute, 0 = none)
    std::mutex life_mu;                    // close / free / set_coalescing against each other
    std::atomic<bool> closing{false};      // Close() (or free) has begun: calls return -1, EBADF
    std::atomic<int> inflight{0};          // threads inside a call on the connection
};

namespace {
// A call in progress on the connection.  Close publishes `closing` and then waits
// for `inflight` to drain; a caller publishes its increment and then reads
// `closing`.  Both pairs are sequentially consistent (a store followed by a load
// of another variable: release/acquire would let either side miss the other,
// x86's store buffer does exactly that), so a caller either sees `closing` and
// leaves without touching the connection's state, or the closer sees the caller
// and waits for it.  The memory itself is freed only by hyobfs_conn_free, which
// no call may race (include/hyobfs_conn.h).
struct InFlight {
    hyobfs_conn* c;
    explicit InFlight(hyobfs_conn* x) : c(x) { c->inflight.fetch_add(1, std::memory_order_seq_cst); }
    ~InFlight() { c->inflight.fetch_sub(1, std::memory_order_seq_cst); }
    bool closed() const {
        if (!c->closing.load(std::memory_order_seq_cst)) return false;
        errno = EBADF;
        return true;
    }
};

// Stops the coalescer (it sends what WriteTo accepted while the socket is still
// open), then waits for every caller still inside the connection.  Caller holds
// life_mu and has checked that the connection is not closing yet.
void quiesce(hyobfs_conn* c, bool wake_readers) {
    c->closing.store(true, std::memory_order_seq_cst);
    hyobfs::coalescer_stop(c->co);
    // a plain-mode ReadFrom blocked in poll: shutdown wakes it (a 0-byte read,
    // turned into EBADF below); Linux does this for unconnected UDP too
    if (wake_readers) (void)shutdown(c->fd, SHUT_RD);
    while (c->inflight.load(std::memory_order_seq_cst) > 0) std::this_thread::yield();
}
}  // namespace

extern "C" {

int hyobfs_conn_wrap(int fd, hyobfs_salamander* ctx, uint32_t batch, hyobfs_conn** out) {
    if (fd < 0 || !ctx || !out) return HYOBFS_ERR_INVALID;
    if (batch == 0) batch = 1024;
    auto* c = new (std::nothrow) hyobfs_conn();
    if (!c) return HYOBFS_ERR_NOMEM;
    c->fd = fd;
    c->ctx = ctx;
    if (!c->rx.alloc(batch) || !c->tx.alloc(batch)) {
        c->rx.release();
        c->tx.release();
        delete c;
        return HYOBFS_ERR_NOMEM;
    }
    c->rmsg.resize(batch);
    c->wmsg.resize(batch);
    c->riov.resize(batch);
    c->wiov.resize(batch);
    c->raddr.resize(batch);
    hyobfs::ctx_retain(ctx);   // the context outlives every connection on it (hyobfs_salamander_free)
    *out = c;
    return HYOBFS_OK;
}

// Close(), conn.go:101-103, which closes the inner conn: later calls fail with
// EBADF (Go: net.ErrClosed).  The coalescer first sends every datagram WriteTo
// accepted, then its threads stop; threads blocked in calls are woken; the fd
// closes once no thread of ours can touch it.  The memory stays until
// hyobfs_conn_free, so calls racing or following Close never see freed state.
int hyobfs_conn_close(hyobfs_conn* c) {
    if (!c) return HYOBFS_ERR_INVALID;
    std::lock_guard<std::mutex> lk(c->life_mu);
    if (c->closing.load(std::memory_order_seq_cst)) {
        errno = EBADF;
        return HYOBFS_ERR_CLOSED;   // Go: a second Close returns an error too
    }
    quiesce(c, true);
    const int rc = close(c->fd);
    return rc == 0 ? HYOBFS_OK : HYOBFS_ERR_IO;
}

// A connection freed without Close (a Go finalizer on a dropped gpuPacketConn)
// closes its descriptor too: the connection owns the fd from hyobfs_conn_wrap on,
// as Go's UDPConn closes its fd from its own finalizer.
void hyobfs_conn_free(hyobfs_conn* c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(c->life_mu);
        if (!c->closing.load(std::memory_order_seq_cst)) {
            quiesce(c, false);   // the coalescer sends what write_to accepted first
            (void)close(c->fd);
        }
    }
    hyobfs::coalescer_free(c->co);   // (already stopped)
    c->rx.release();
    c->tx.release();
    hyobfs::ctx_release(c->ctx);
    delete c;
}

// ReadFrom, conn.go:73-88
int64_t hyobfs_conn_read_from(hyobfs_conn* c, uint8_t* p, size_t cap, void* addr, uint32_t* addrlen) {
    if (!c) {
        errno = EINVAL;
        return -1;
    }
    InFlight g(c);
    if (g.closed()) return -1;
    if (c->co) return hyobfs::coalescer_read(c->co, p, cap, addr, addrlen);
    timeval tv{0, 0};
    socklen_t tl = sizeof tv;
    (void)getsockopt(c->fd, SOL_SOCKET, SO_RCVTIMEO, &tv, &tl);
    const int64_t rcv_ns = (int64_t)tv.tv_sec * 1000000000ll + (int64_t)tv.tv_usec * 1000ll;
    const int64_t rcv_limit = rcv_ns ? hyobfs::realtime_ns() + rcv_ns : 0;   // one limit for the whole call
    for (;;) {
        std::lock_guard<std::mutex> lk(c->read_mu);
        // wait in slices of at most 50 ms, re-reading the read deadline (it may be
        // set or moved while this call waits: net.Conn deadlines apply to blocked
        // calls too; without one, the socket's SO_RCVTIMEO read once bounds the
        // call), then receive without blocking
        for (;;) {
            int64_t d = c->dl.read.load(std::memory_order_acquire);
            if (!d) d = rcv_limit;
            const int64_t left = d ? d - hyobfs::realtime_ns() : 50000000;
            if (d && left <= 0) {
                errno = EAGAIN;
                return -1;
            }
            pollfd pf{c->fd, POLLIN, 0};
            const int pr = poll(&pf, 1, (int)std::min<int64_t>(50, (left + 999999) / 1000000));
            if (g.closed()) return -1;
            if (pr > 0) break;
            if (pr < 0 && errno != EINTR) return -1;
        }
        const int flags = MSG_DONTWAIT;
        socklen_t al = addrlen ? *addrlen : 0;
        const ssize_t n = recvfrom(c->fd, c->read_buf, kBuf, flags, static_cast<sockaddr*>(addr), addr ? &al : nullptr);
        if (addrlen) *addrlen = al;
        if (n <= 0 && g.closed()) return -1;   // woken by Close()
        if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) continue;   // readiness went stale: wait again
        if (n <= 0) return n;   // error or empty datagram: returned as is (:77-80)
        const size_t m = hyobfs_salamander_deobfuscate(c->ctx, c->read_buf, (size_t)n, p, cap);
        if (m > 0) return (int64_t)m;
        // invalid packet: drop it and read again (:86)
    }
}

// WriteTo, conn.go:90-99
int64_t hyobfs_conn_write_to(hyobfs_conn* c, const uint8_t* p, size_t len, const void* addr, uint32_t addrlen) {
    if (!c) {
        errno = EINVAL;
        return -1;
    }
    InFlight g(c);
    if (g.closed()) return -1;
    if (c->co) return hyobfs::coalescer_write(c->co, p, len, addr, addrlen);
    std::lock_guard<std::mutex> lk(c->write_mu);
    if (const int64_t d = c->dl.write.load(std::memory_order_acquire); d && hyobfs::realtime_ns() >= d) {
        errno = EAGAIN;   // SetWriteDeadline has passed
        return -1;
    }
    // Obfuscate into the 2048-byte writeBuf: 0 when len > 2040 (salamander.go:60-62)
    const size_t nn = hyobfs_salamander_obfuscate_auto(c->ctx, p, len, c->write_buf, kBuf);
    const ssize_t rc = sendto(c->fd, c->write_buf, nn, 0, static_cast<const sockaddr*>(addr), addrlen);
    if (rc < 0) return -1;
    return (int64_t)len;   // n = len(p) on success (:95-97), even for the empty-datagram case
}

int hyobfs_conn_read_batch(hyobfs_conn* c, hyobfs_dgram* msgs, uint32_t n) {
    if (!c || (!msgs && n)) {
        errno = EINVAL;
        return -1;
    }
    if (n == 0) return 0;
    InFlight g(c);
    if (g.closed()) return -1;
    if (c->co) {   // the coalescer's reader owns the socket's receive side
        errno = EBUSY;
        return -1;
    }
    std::lock_guard<std::mutex> lk(c->read_mu);
    n = std::min(n, c->rx.n);
    for (;;) {
        for (uint32_t i = 0; i < n; ++i) {
            c->riov[i].iov_base = c->rx.in + (size_t)i * kBuf;
            c->riov[i].iov_len = kBuf;
            memset(&c->rmsg[i], 0, sizeof(mmsghdr));
            c->rmsg[i].msg_hdr.msg_iov = &c->riov[i];
            c->rmsg[i].msg_hdr.msg_iovlen = 1;
            c->rmsg[i].msg_hdr.msg_name = &c->raddr[i];
            c->rmsg[i].msg_hdr.msg_namelen = sizeof(sockaddr_storage);
        }
        const int k = recvmmsg(c->fd, c->rmsg.data(), n, MSG_WAITFORONE, nullptr);
        if (k <= 0 && g.closed()) return -1;   // woken by Close()
        if (k <= 0) return k;
        for (int i = 0; i < k; ++i) c->rx.len[i] = c->rmsg[i].msg_len;
        hyobfs_batch b{};
        b.n = (uint64_t)k;
        b.in = c->rx.in;
        b.in_stride = kBuf;
        b.in_len = c->rx.len;
        b.out = c->rx.out;
        b.out_stride = kBuf;
        b.out_cap = (uint64_t)k * kBuf;
        b.out_len = c->rx.olen;
        if (hyobfs_salamander_deobfuscate_host(c->ctx, &b, 0) != HYOBFS_OK) {
            errno = EIO;
            return -1;
        }
        int got = 0;
        for (int i = 0; i < k; ++i) {
            // an empty datagram is a 0-byte read, as ReadFrom returns it (conn.go:77-80)
            const bool empty = c->rx.len[i] == 0;
            const uint32_t m = empty ? 0u : c->rx.olen[i];
            if (!empty && (m == 0 || m > msgs[got].cap)) continue;   // Deobfuscate returned 0: dropped
            if (m) memcpy(msgs[got].buf, c->rx.out + (size_t)i * kBuf, m);
            msgs[got].len = m;
            const uint32_t al = std::min<uint32_t>(c->rmsg[i].msg_hdr.msg_namelen, sizeof msgs[got].addr);
            memcpy(msgs[got].addr, &c->raddr[i], al);
            msgs[got].addrlen = al;
            ++got;
        }
        if (got) return got;
        // every datagram was invalid: read again, like ReadFrom
    }
}

int hyobfs_conn_write_batch(hyobfs_conn* c, const hyobfs_dgram* msgs, uint32_t n) {
    if (!c || (!msgs && n)) {
        errno = EINVAL;
        return -1;
    }
    InFlight g(c);
    if (g.closed()) return -1;
    if (c->co) {
        errno = EBUSY;
        return -1;
    }
    std::lock_guard<std::mutex> lk(c->write_mu);
    uint32_t sent = 0;
    while (sent < n) {
        const uint32_t k = std::min(n - sent, c->tx.n);
        for (uint32_t i = 0; i < k; ++i) {
            const hyobfs_dgram& d = msgs[sent + i];
            const uint32_t L = std::min<uint32_t>(d.len, kBuf);   // longer ones are dropped below anyway
            memcpy(c->tx.in + (size_t)i * kBuf, d.buf, L);
            c->tx.len[i] = d.len > kBuf ? kBuf : d.len;   // > 2040 -> out_len 0 -> empty datagram
        }
        hyobfs_salamander_next_salts(c->ctx, reinterpret_cast<uint8_t*>(c->tx.salts), k);   // RandSrc
        hyobfs_batch b{};
        b.n = k;
        b.in = c->tx.in;
        b.in_stride = kBuf;
        b.in_len = c->tx.len;
        b.salts = c->tx.salts;
        b.out = c->tx.out;
        b.out_stride = kBuf;   // len(writeBuf): Obfuscate needs len+8 <= 2048
        b.out_cap = (uint64_t)k * kBuf;
        b.out_len = c->tx.olen;
        if (hyobfs_salamander_obfuscate_host(c->ctx, &b, 0) != HYOBFS_OK) {
            errno = EIO;
            return -1;
        }
        for (uint32_t i = 0; i < k; ++i) {
            const hyobfs_dgram& d = msgs[sent + i];
            c->wiov[i].iov_base = c->tx.out + (size_t)i * kBuf;
            c->wiov[i].iov_len = c->tx.olen[i];
            memset(&c->wmsg[i], 0, sizeof(mmsghdr));
            c->wmsg[i].msg_hdr.msg_iov = &c->wiov[i];
            c->wmsg[i].msg_hdr.msg_iovlen = 1;
            c->wmsg[i].msg_hdr.msg_name = const_cast<uint8_t*>(d.addr);
            c->wmsg[i].msg_hdr.msg_namelen = d.addrlen;
        }
        uint32_t done = 0;
        while (done < k) {
            const int r = sendmmsg(c->fd, c->wmsg.data() + done, k - done, 0);
            if (r < 0) return sent + done ? (int)(sent + done) : -1;
            done += (uint32_t)r;
        }
        sent += k;
    }
    return (int)sent;
}

int hyobfs_conn_set_coalescing(hyobfs_conn* c, uint32_t max_batch, uint32_t max_wait_us) {
    if (!c) return HYOBFS_ERR_INVALID;
    std::lock_guard<std::mutex> lk(c->life_mu);
    if (c->closing.load(std::memory_order_seq_cst)) return HYOBFS_ERR_CLOSED;
    if (c->co || max_batch == 0 || max_batch > (1u << 16)) return HYOBFS_ERR_INVALID;
    c->co = hyobfs::coalescer_new(c->fd, c->ctx, max_batch, max_wait_us, &c->dl);
    return c->co ? HYOBFS_OK : HYOBFS_ERR_NOMEM;
}

int hyobfs_conn_set_read_deadline(hyobfs_conn* c, int64_t unix_ns) {
    if (!c || unix_ns < 0) return HYOBFS_ERR_INVALID;
    InFlight g(c);
    if (g.closed()) return HYOBFS_ERR_CLOSED;
    c->dl.read.store(unix_ns, std::memory_order_release);
    hyobfs::coalescer_poke(c->co);   // blocked reads re-read it (net.Conn: also currently-blocked calls)
    return HYOBFS_OK;
}

int hyobfs_conn_set_write_deadline(hyobfs_conn* c, int64_t unix_ns) {
    if (!c || unix_ns < 0) return HYOBFS_ERR_INVALID;
    InFlight g(c);
    if (g.closed()) return HYOBFS_ERR_CLOSED;
    c->dl.write.store(unix_ns, std::memory_order_release);
    hyobfs::coalescer_poke(c->co);
    return HYOBFS_OK;
}

int hyobfs_conn_flush(hyobfs_conn* c) {
    if (!c) return HYOBFS_ERR_INVALID;
    InFlight g(c);
    if (g.closed()) return HYOBFS_ERR_CLOSED;   // (Close already sent everything accepted)
    return c->co ? hyobfs::coalescer_flush(c->co) : HYOBFS_OK;
}

int hyobfs_conn_stats(hyobfs_conn* c, uint64_t out[6]) {   // also after Close: the counters stay
    if (!c || !out) return HYOBFS_ERR_INVALID;
    if (!c->co) {
        for (int i = 0; i < 6; ++i) out[i] = 0;
        return HYOBFS_OK;
    }
    hyobfs::coalescer_stats(c->co, out);
    return HYOBFS_OK;
}

}  // extern "C"
