// conn_coalesce.cpp -- batching behind the per-datagram WriteTo / ReadFrom of a
// coalescing hyobfs_conn (include/hyobfs_conn.h, hyobfs_conn_set_coalescing).
//
// The reference calls Obfuscate / Deobfuscate once per datagram inside
// obfsPacketConn.WriteTo / ReadFrom (extras/obfs/conn.go:73-99); a GPU call per
// datagram is a PCIe round trip.  Here many callers' datagrams share one GPU
// batch:
//   * send: WriteTo reserves a slot in the filling batch (a short spin lock),
//     copies the datagram and returns len(p).  A flusher thread seals the batch
//     when it is full, max_wait_us after its first datagram, or once no WriteTo
//     has added to it for idle_us (the writers paused: a light load does not wait
//     for max_wait; HYOBFS_COALESCE_IDLE_US, default min(100, max_wait_us)), and launches its
//     obfuscation on the GPU, which reads and writes the batch in place (mapped
//     pinned memory, gpu_queue_submit); while that kernel runs the thread sends
//     the PREVIOUS batch with sendmmsg, and the next batch fills.  Three send
//     batches rotate: filling, on the GPU, on the wire.  Like a UDP sendto, the call
//     returns once the datagram is queued.  A later send failure is counted and
//     its errno is returned by the NEXT WriteTo on the connection (-1, that
//     datagram not accepted): the reference returns it to the caller whose
//     datagram failed (conn.go:93-98), which a queued send cannot do.
//   * receive: a reader thread receives up to max_batch datagrams with
//     recvmmsg and launches their deobfuscation as one GPU batch; while it runs
//     the thread hands the previous batch to the queue and receives the next one
//     (when the socket has nothing more, it finishes the batch on the GPU first);
//     ReadFrom takes the next datagram from the queue.  Datagrams that do not
//     deobfuscate are dropped and an empty datagram is a 0-byte read, as in
//     ReadFrom (conn.go:77-86).  The socket's SO_RCVTIMEO bounds the wait (one
//     absolute deadline per call, like SetReadDeadline).
//   * shutdown: stop() sends what was accepted, wakes every caller blocked in
//     ReadFrom / WriteTo (they return -1, EBADF) and joins the threads.  A
//     writer takes its slot under the spin lock and checks `stop` there: the
//     flusher's last look for pending datagrams happens under the same lock
//     after it saw `stop`, so a datagram is either refused (EBADF) or sent --
//     never accepted and dropped.  The memory is freed only once no caller is
//     left inside.
#include "conn_coalesce.h"

#include <errno.h>
#include <poll.h>
#include <sys/prctl.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/time.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/hyobfs_conn.h"

namespace hyobfs {
namespace {

constexpr uint32_t kBuf = HYOBFS_UDP_BUFFER_SIZE;   // udpBufferSize, conn.go:10
using Clock = std::chrono::steady_clock;

struct Pinned {   // device-mapped pinned slots of kBuf bytes
    uint8_t* in = nullptr;
    uint8_t* out = nullptr;
    uint32_t* len = nullptr;
    uint32_t* olen = nullptr;
    uint64_t* salts = nullptr;
    bool alloc(uint32_t n) {
        in = static_cast<uint8_t*>(hyobfs_host_alloc((size_t)n * kBuf));
        out = static_cast<uint8_t*>(hyobfs_host_alloc((size_t)n * kBuf));
        len = static_cast<uint32_t*>(hyobfs_host_alloc((size_t)n * 4));
        olen = static_cast<uint32_t*>(hyobfs_host_alloc((size_t)n * 4));
        salts = static_cast<uint64_t*>(hyobfs_host_alloc((size_t)n * 8));
        return in && out && len && olen && salts;
    }
    void release() {
        hyobfs_host_free(in);
        hyobfs_host_free(out);
        hyobfs_host_free(len);
        hyobfs_host_free(olen);
        hyobfs_host_free(salts);
    }
};

// HYOBFS_COALESCE_OVERLAP=0: no overlap (seal, GPU, send one batch at a time);
// HYOBFS_COALESCE_ZEROCOPY=0: the GPU step through hyobfs_salamander_*_host (staged
// copies, synchronous) instead of in place.  Both 1 by default; A/B knobs, read once.
static bool env_flag(const char* name, bool dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoi(e) != 0 : dflt;
}
static bool overlap_on() {
    static const bool v = env_flag("HYOBFS_COALESCE_OVERLAP", true);
    return v;
}
static bool zerocopy_on() {
    static const bool v = env_flag("HYOBFS_COALESCE_ZEROCOPY", true);
    return v;
}
// Idle seal (HYOBFS_COALESCE_IDLE_US, default 100): a filling batch no WriteTo has added
// to for this long is sealed without waiting for max_wait_us.  Under load the writers
// arrive far more often and batches still fill; at a light load a datagram waits about
// this long instead of max_wait_us.  Shorter is not better on a shared host: every
// batch costs ~25 us of CPU (launch, event, thread wake-ups), and 16 connections
// sealing every 20 us used the box's whole 16-core CPU share and were throttled
// (millisecond tails, profiles/r06_host/).
static uint32_t coalesce_idle_us() {
    static const uint32_t v = [] {
        const char* e = std::getenv("HYOBFS_COALESCE_IDLE_US");
        const long x = e ? std::atol(e) : 100;
        return (uint32_t)(x < 0 ? 0 : x);
    }();
    return v;
}

struct Batch {
    Pinned b;
    std::vector<sockaddr_storage> addr;
    std::vector<uint32_t> alen;
    std::vector<mmsghdr> msg;
    std::vector<iovec> iov;
    // send side (count / sealed / first under the spin lock)
    uint32_t count = 0;
    bool sealed = false;
    Clock::time_point first{}, last{};   // the first and the latest datagram's arrival
    std::atomic<uint32_t> committed{0};
    bool gpu_ok = false;   // its GPU step was launched (or done) without error
    // receive side (k / next under rx_mu)
    uint32_t k = 0, next = 0;
    std::atomic<uint32_t> done{0};
    bool alloc(uint32_t n) {
        addr.resize(n);
        alen.resize(n);
        msg.resize(n);
        iov.resize(n);
        return b.alloc(n);
    }
};

class Spin {
    std::atomic_flag f = ATOMIC_FLAG_INIT;

   public:
    void lock() {
        while (f.test_and_set(std::memory_order_acquire)) std::this_thread::yield();
    }
    void unlock() { f.clear(std::memory_order_release); }
};

}  // namespace

int64_t realtime_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
        .count();
}

// Waits on cv until pred() or the absolute deadline dl (0: none) passes; false on the deadline.
template <class Pred>
static bool wait_deadline(std::condition_variable& cv, std::unique_lock<std::mutex>& lk, const std::atomic<int64_t>& dl,
                          Pred pred) {
    for (;;) {
        if (pred()) return true;
        const int64_t d = dl.load(std::memory_order_acquire);
        if (d == 0) {
            cv.wait(lk);   // a deadline set later pokes the condition variable
            continue;
        }
        const int64_t now = realtime_ns();
        if (now >= d) return pred();
        cv.wait_for(lk, std::chrono::nanoseconds(d - now));
    }
}

struct Coalescer {
    int fd = -1;
    const Deadlines* dl = nullptr;
    hyobfs_salamander* ctx = nullptr;
    uint32_t max_batch = 0;
    std::chrono::microseconds max_wait{0};
    std::chrono::microseconds idle{0};   // seal a batch no WriteTo added to for this long
    std::atomic<bool> stop{false};
    GpuQueue* gq_tx = nullptr;           // the send side's stream (gpu_queue_*)
    GpuQueue* gq_rx = nullptr;
    // send: batches rotate filling -> on the GPU -> on the wire
    static constexpr int kTx = 3;
    Batch tx[kTx];
    int cur = 0;                         // filling batch, under spin
    Spin spin;
    std::mutex tx_mu;                    // waits: flusher for datagrams, writers for space
    std::condition_variable cv_flush, cv_space;
    std::atomic<uint64_t> accepted{0}, sent{0}, tx_batches{0}, tx_errors{0};
    std::atomic<int> tx_err_pending{0};  // errno of the first failed send not yet reported
    std::thread flusher;
    // receive
    static constexpr int kRx = 4;
    Batch rx[kRx];
    std::mutex rx_mu;
    std::condition_variable cv_ready, cv_free;
    std::deque<int> ready, freelist;
    int rx_err = 0;                      // transient receive error, reported once
    int rx_fatal = 0;                    // the socket is unusable (EBADF, ENOTSOCK, ...): every later read
    std::atomic<uint64_t> received{0}, rx_batches{0}, rx_dropped{0}, rx_gpu_errors{0};
    std::thread reader;
    std::atomic<int> callers{0};         // threads inside coalescer_read / coalescer_write
    bool stopped = false;

    bool has_space() const { return !tx[cur].sealed && tx[cur].count < max_batch; }
    void flush_loop();
    void submit_tx(int i);
    void finish_tx(int i);
    void read_loop();
    void submit_rx(int i, uint32_t k);
    void finish_rx(int i);
};

// The sealed batch i onto the GPU: salts, then one obfuscate launch in place (or,
// HYOBFS_COALESCE_ZEROCOPY=0, the synchronous staged call).
void Coalescer::submit_tx(int i) {
    Batch& b = tx[i];
    const uint32_t n = b.count;   // no writer changes a sealed batch's count
    while (b.committed.load(std::memory_order_acquire) < n) std::this_thread::yield();
    hyobfs_salamander_next_salts(ctx, reinterpret_cast<uint8_t*>(b.b.salts), n);   // RandSrc, salamander.go:65
    hyobfs_batch d{};
    d.n = n;
    d.in = b.b.in;
    d.in_stride = kBuf;
    d.in_len = b.b.len;
    d.salts = b.b.salts;
    d.out = b.b.out;
    d.out_stride = kBuf;   // len(writeBuf): Obfuscate needs len + 8 <= 2048, else an empty datagram
    d.out_cap = (uint64_t)n * kBuf;
    d.out_len = b.b.olen;
    b.gpu_ok = (zerocopy_on() ? gpu_queue_submit(gq_tx, &d, true, i) : hyobfs_salamander_obfuscate_host(ctx, &d, 0)) ==
               HYOBFS_OK;
}

// Waits for batch i's kernel, sends it with sendmmsg and frees the batch for writers.
void Coalescer::finish_tx(int i) {
    Batch& b = tx[i];
    const uint32_t n = b.count;
    if (b.gpu_ok && zerocopy_on()) b.gpu_ok = gpu_queue_wait(gq_tx, i) == HYOBFS_OK;
    if (!b.gpu_ok) {
        tx_errors += n;
        int z = 0;
        tx_err_pending.compare_exchange_strong(z, EIO);
    } else {
        for (uint32_t j = 0; j < n; ++j) {
            b.iov[j].iov_base = b.b.out + (size_t)j * kBuf;
            b.iov[j].iov_len = b.b.olen[j];
            memset(&b.msg[j], 0, sizeof(mmsghdr));
            b.msg[j].msg_hdr.msg_iov = &b.iov[j];
            b.msg[j].msg_hdr.msg_iovlen = 1;
            b.msg[j].msg_hdr.msg_name = &b.addr[j];
            b.msg[j].msg_hdr.msg_namelen = b.alen[j];
        }
        uint32_t done = 0;
        while (done < n) {
            const int r = sendmmsg(fd, b.msg.data() + done, n - done, 0);
            if (r > 0) {
                done += (uint32_t)r;
                continue;
            }
            if (r < 0 && errno == EINTR) continue;
            if (r < 0 && (errno == EAGAIN || errno == ENOBUFS)) {   // socket buffer full: wait for room
                pollfd pf{fd, POLLOUT, 0};
                (void)poll(&pf, 1, 10);
                continue;
            }
            ++tx_errors;   // this datagram cannot be sent (e.g. no route): skip it, report it to the next WriteTo
            int z = 0;
            tx_err_pending.compare_exchange_strong(z, errno ? errno : EIO);
            ++done;
        }
        ++tx_batches;
    }
    sent += n;   // handled (sent or lost): flush() must not wait for them
    spin.lock();
    b.count = 0;
    b.committed.store(0, std::memory_order_relaxed);
    b.sealed = false;
    spin.unlock();
    {
        std::lock_guard<std::mutex> lk(tx_mu);   // writers waiting for space re-check under tx_mu
    }
    cv_space.notify_all();
}

void Coalescer::flush_loop() {
    int prev = -1;   // a batch whose kernel was launched and which is not sent yet
    for (;;) {
        int sealed = -1;
        {
            std::unique_lock<std::mutex> lk(tx_mu);
            auto pending = [&] {
                spin.lock();
                const bool p = tx[cur].count > 0;
                spin.unlock();
                return p;
            };
            auto due = [&] {
                spin.lock();
                const bool full = tx[cur].count >= max_batch;
                spin.unlock();
                return full || stop.load();
            };
            if (prev < 0) {
                cv_flush.wait(lk, [&] { return stop.load() || pending(); });
                if (!pending()) return;   // stopping, nothing left to send
            }
            if (pending()) {
                // due: full, stopping, max_wait after the first datagram, or idle since the
                // last one.  Nothing on the GPU: sleep until one of those; a batch on the
                // GPU: seal this one only if it is due now, else send that one first
                auto wake = [&] {   // the earlier of the deadline and the idle point
                    spin.lock();
                    const Clock::time_point d = std::min(tx[cur].first + max_wait, tx[cur].last + idle);
                    spin.unlock();
                    return d;
                };
                bool go;
                if (prev < 0) {
                    for (;;) {
                        const Clock::time_point w = wake();
                        if (due() || Clock::now() >= w) break;
                        cv_flush.wait_until(lk, w, due);
                    }
                    go = true;
                } else {
                    go = due() || Clock::now() >= wake();
                }
                if (go) {   // seal the filling batch; writers move on to the next (already sent)
                    spin.lock();
                    tx[cur].sealed = true;
                    sealed = cur;
                    cur = (cur + 1) % kTx;
                    spin.unlock();
                }
            }
        }
        if (sealed >= 0) {
            cv_space.notify_all();
            submit_tx(sealed);
        }
        if (prev >= 0) finish_tx(prev);
        prev = sealed;
        if (prev >= 0 && !overlap_on()) {
            finish_tx(prev);
            prev = -1;
        }
    }
}

void Coalescer::submit_rx(int i, uint32_t k) {
    Batch& b = rx[i];
    for (uint32_t j = 0; j < k; ++j) {
        b.b.len[j] = b.msg[j].msg_len;
        b.alen[j] = b.msg[j].msg_hdr.msg_namelen;
    }
    hyobfs_batch d{};
    d.n = (uint64_t)k;
    d.in = b.b.in;
    d.in_stride = kBuf;
    d.in_len = b.b.len;
    d.out = b.b.out;
    d.out_stride = kBuf;
    d.out_cap = (uint64_t)k * kBuf;
    d.out_len = b.b.olen;
    b.k = k;
    b.gpu_ok = (zerocopy_on() ? gpu_queue_submit(gq_rx, &d, false, i) : hyobfs_salamander_deobfuscate_host(ctx, &d, 0)) ==
               HYOBFS_OK;
    received += (uint64_t)k;
}

// Waits for batch i's kernel and queues it for ReadFrom.  A batch whose GPU step
// failed is not "invalid packets" (the reference drops only datagrams Deobfuscate
// rejects, conn.go:81-86): its datagrams are lost, the batch goes back to the free
// list, and ReadFrom reports EIO once (rx_err), as WriteTo does for the send side.
void Coalescer::finish_rx(int i) {
    Batch& b = rx[i];
    if (b.gpu_ok && zerocopy_on()) b.gpu_ok = gpu_queue_wait(gq_rx, i) == HYOBFS_OK;
    {
        std::lock_guard<std::mutex> lk(rx_mu);
        if (!b.gpu_ok) {
            rx_gpu_errors += b.k;
            rx_err = EIO;
            freelist.push_back(i);
        } else {
            ++rx_batches;
            b.next = 0;
            b.done.store(0, std::memory_order_relaxed);
            ready.push_back(i);
        }
    }
    cv_ready.notify_all();
}

void Coalescer::read_loop() {
    int prev = -1;   // a batch whose kernel was launched and which is not queued yet
    for (;;) {
        int bi;
        {
            std::unique_lock<std::mutex> lk(rx_mu);
            if (prev >= 0 && freelist.empty()) {   // no free batch: the launched one goes to readers
                lk.unlock();                       // first, never waiting on their progress
                finish_rx(prev);
                prev = -1;
                lk.lock();
            }
            cv_free.wait(lk, [&] { return stop.load() || !freelist.empty(); });
            if (stop) break;
            bi = freelist.front();
            freelist.pop_front();
        }
        Batch& b = rx[bi];
        int k = -1;
        while (!stop) {
            // with a batch on the GPU only look: nothing waiting means queue that one first
            pollfd pf{fd, POLLIN, 0};
            const int pr = poll(&pf, 1, prev >= 0 ? 0 : 50);
            if (pr <= 0) {   // timeout or EINTR: check stop, poll again
                if (prev >= 0) {
                    finish_rx(prev);
                    prev = -1;
                }
                continue;
            }
            for (uint32_t i = 0; i < max_batch; ++i) {
                b.iov[i].iov_base = b.b.in + (size_t)i * kBuf;
                b.iov[i].iov_len = kBuf;
                memset(&b.msg[i], 0, sizeof(mmsghdr));
                b.msg[i].msg_hdr.msg_iov = &b.iov[i];
                b.msg[i].msg_hdr.msg_iovlen = 1;
                b.msg[i].msg_hdr.msg_name = &b.addr[i];
                b.msg[i].msg_hdr.msg_namelen = sizeof(sockaddr_storage);
            }
            k = recvmmsg(fd, b.msg.data(), max_batch, MSG_DONTWAIT, nullptr);
            if (k > 0) break;
            if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
                const int e = errno;
                if (prev >= 0) {   // what was received before the error is delivered first
                    finish_rx(prev);
                    prev = -1;
                }
                std::unique_lock<std::mutex> lk(rx_mu);
                // the socket is gone (closed under us): every later ReadFrom fails with
                // it (Go: net.ErrClosed each time), the thread parks until stop instead
                // of spinning on POLLNVAL; other errors are reported once, then retried
                const bool fatal = e == EBADF || e == ENOTSOCK || e == EINVAL || e == EFAULT;
                if (fatal)
                    rx_fatal = e;
                else
                    rx_err = e;   // reported by ReadFrom once the queue is empty
                cv_ready.notify_all();
                cv_free.wait_for(lk, fatal ? std::chrono::hours(24) : std::chrono::milliseconds(1),
                                 [&] { return stop.load(); });
                break;
            }
        }
        if (stop || k <= 0) {
            std::lock_guard<std::mutex> lk(rx_mu);
            freelist.push_back(bi);
            cv_ready.notify_all();
            if (stop) break;
            continue;
        }
        submit_rx(bi, (uint32_t)k);
        if (prev >= 0) finish_rx(prev);
        prev = bi;
        if (!overlap_on()) {
            finish_rx(prev);
            prev = -1;
        }
    }
    // stopping: a kernel may still be writing the batch on the GPU, whose buffers
    // are freed after this thread is joined
    if (prev >= 0 && rx[prev].gpu_ok && zerocopy_on()) (void)gpu_queue_wait(gq_rx, prev);
}

Coalescer* coalescer_new(int fd, hyobfs_salamander* ctx, uint32_t max_batch, uint32_t max_wait_us,
                         const Deadlines* dl) {
    auto* q = new (std::nothrow) Coalescer();
    if (!q) return nullptr;
    q->fd = fd;
    q->dl = dl;
    q->ctx = ctx;
    q->max_batch = max_batch;
    q->max_wait = std::chrono::microseconds(max_wait_us);
    q->idle = std::chrono::microseconds(std::min<uint32_t>(max_wait_us, coalesce_idle_us()));
    bool ok = true;
    for (auto& b : q->tx) ok = ok && b.alloc(max_batch);
    for (auto& b : q->rx) ok = ok && b.alloc(max_batch);
    if (ok && zerocopy_on()) {
        q->gq_tx = gpu_queue_new(ctx);
        q->gq_rx = gpu_queue_new(ctx);
        ok = q->gq_tx && q->gq_rx;
    }
    if (!ok) {
        gpu_queue_free(q->gq_tx);
        gpu_queue_free(q->gq_rx);
        for (auto& b : q->tx) b.b.release();
        for (auto& b : q->rx) b.b.release();
        delete q;
        return nullptr;
    }
    for (int i = 0; i < Coalescer::kRx; ++i) q->freelist.push_back(i);
    // named threads: per-thread CPU use is attributable (tools/udp_bench, top -H)
    q->flusher = std::thread([q] {
        (void)prctl(PR_SET_NAME, "hyobfs-tx", 0, 0, 0);
        (void)prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);   // wake at the idle point (and from gpu_queue_wait's sleeps) on time
        q->flush_loop();
    });
    q->reader = std::thread([q] {
        (void)prctl(PR_SET_NAME, "hyobfs-rx", 0, 0, 0);
        (void)prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);   // gpu_queue_wait's short sleeps end on time
        q->read_loop();
    });
    return q;
}

void coalescer_stop(Coalescer* q) {
    if (!q || q->stopped) return;
    {
        std::lock_guard<std::mutex> a(q->tx_mu);
        std::lock_guard<std::mutex> b(q->rx_mu);
        q->stop = true;
    }
    q->cv_flush.notify_all();
    q->cv_space.notify_all();
    q->cv_free.notify_all();
    q->cv_ready.notify_all();
    q->flusher.join();   // sends what was accepted first
    q->reader.join();
    q->stopped = true;
}

void coalescer_free(Coalescer* q) {
    if (!q) return;
    coalescer_stop(q);
    // callers woken by stop leave through the mutexes and condition variables
    // of q: free it only once the last one is out
    while (q->callers.load(std::memory_order_seq_cst) > 0) {
        q->cv_space.notify_all();
        q->cv_ready.notify_all();
        std::this_thread::yield();
    }
    gpu_queue_free(q->gq_tx);   // (waits for its stream: nothing is left on it)
    gpu_queue_free(q->gq_rx);
    for (auto& b : q->tx) b.b.release();
    for (auto& b : q->rx) b.b.release();
    delete q;
}

namespace {
struct CallerGuard {   // counts a caller inside the coalescer (see coalescer_free)
    Coalescer* q;
    explicit CallerGuard(Coalescer* c) : q(c) { q->callers.fetch_add(1, std::memory_order_seq_cst); }
    ~CallerGuard() { q->callers.fetch_sub(1, std::memory_order_seq_cst); }
};
}  // namespace

int64_t coalescer_write(Coalescer* q, const uint8_t* p, size_t len, const void* addr, uint32_t addrlen) {
    CallerGuard g(q);
    if (addrlen > sizeof(sockaddr_storage)) {
        errno = EINVAL;
        return -1;
    }
    if (q->stop.load()) {   // early out; the check that counts is the one under the spin lock
        errno = EBADF;
        return -1;
    }
    if (const int64_t d = q->dl->write.load(std::memory_order_acquire); d && realtime_ns() >= d) {
        errno = EAGAIN;   // the write deadline has passed
        return -1;
    }
    if (q->tx_err_pending.load(std::memory_order_relaxed)) {   // an earlier datagram's send failed
        const int e = q->tx_err_pending.exchange(0);
        if (e) {
            errno = e;
            return -1;
        }
    }
    Batch* b;
    uint32_t idx;
    for (;;) {
        q->spin.lock();
        if (q->stop.load()) {   // the flusher may have looked for the last time: refuse
            q->spin.unlock();
            errno = EBADF;
            return -1;
        }
        b = &q->tx[q->cur];
        if (q->has_space()) {
            idx = b->count++;
            const Clock::time_point now = Clock::now();
            if (idx == 0) b->first = now;
            b->last = now;
            q->spin.unlock();
            break;
        }
        q->spin.unlock();
        std::unique_lock<std::mutex> lk(q->tx_mu);
        q->cv_flush.notify_one();   // the filling batch is full
        const bool ok = wait_deadline(q->cv_space, lk, q->dl->write, [&] {
            q->spin.lock();
            const bool s = q->has_space();
            q->spin.unlock();
            return s || q->stop.load();
        });
        if (q->stop) {
            errno = EBADF;
            return -1;
        }
        if (!ok) {   // SetWriteDeadline passed while both batches were busy
            errno = EAGAIN;
            return -1;
        }
    }
    // Obfuscate into a 2048-byte slot: > 2040 bytes gives out_len 0, an empty
    // datagram, and WriteTo still reports len(p) (conn.go:92-98)
    const uint32_t L = len > kBuf ? kBuf : (uint32_t)len;
    if (len <= kBuf && len) memcpy(b->b.in + (size_t)idx * kBuf, p, len);
    b->b.len[idx] = L;
    if (addrlen) memcpy(&b->addr[idx], addr, addrlen);
    b->alen[idx] = addrlen;
    b->committed.fetch_add(1, std::memory_order_release);
    ++q->accepted;
    if (idx == 0 || idx + 1 == q->max_batch) {   // first datagram starts the wait; a full batch ends it
        std::lock_guard<std::mutex> lk(q->tx_mu);
        q->cv_flush.notify_one();
    }
    return (int64_t)len;
}

int64_t coalescer_read(Coalescer* q, uint8_t* p, size_t cap, void* addr, uint32_t* addrlen) {
    CallerGuard g(q);
    // SetReadDeadline: the connection's absolute read deadline if one is set
    // (re-read whenever it changes), else SO_RCVTIMEO, read when the call first has
    // to wait (a datagram already queued costs no system call): one absolute deadline
    // for the whole call
    const Clock::time_point start = Clock::now();
    bool have_to = false, timed = false;
    Clock::time_point deadline{};
    for (;;) {
        int bi;
        uint32_t idx;
        {
            std::unique_lock<std::mutex> lk(q->rx_mu);
            while (q->ready.empty()) {
                if (q->rx_fatal) {
                    errno = q->rx_fatal;
                    return -1;
                }
                if (q->rx_err) {
                    errno = q->rx_err;
                    q->rx_err = 0;
                    return -1;
                }
                if (q->stop) {
                    errno = EBADF;
                    return -1;
                }
                auto woken = [&] { return !q->ready.empty() || q->rx_err || q->rx_fatal || q->stop; };
                if (!have_to) {
                    timeval tv{0, 0};
                    socklen_t tl = sizeof tv;
                    (void)getsockopt(q->fd, SOL_SOCKET, SO_RCVTIMEO, &tv, &tl);
                    const auto t = std::chrono::seconds(tv.tv_sec) + std::chrono::microseconds(tv.tv_usec);
                    timed = t.count() != 0;
                    deadline = start + t;
                    have_to = true;
                }
                if (q->dl->read.load(std::memory_order_acquire)) {
                    if (!wait_deadline(q->cv_ready, lk, q->dl->read, woken)) {
                        errno = EAGAIN;
                        return -1;
                    }
                } else if (!timed) {
                    q->cv_ready.wait(lk);
                } else if (!q->cv_ready.wait_until(lk, deadline, woken)) {
                    errno = EAGAIN;
                    return -1;
                }
            }
            bi = q->ready.front();
            Batch& b = q->rx[bi];
            idx = b.next++;
            if (b.next == b.k) q->ready.pop_front();
        }
        Batch& b = q->rx[bi];
        const uint32_t L = b.b.len[idx], m = b.b.olen[idx];
        const bool deliver = L == 0 || (m != 0 && m <= cap);   // empty: a 0-byte read (conn.go:77-80)
        int64_t n = 0;
        if (deliver) {
            if (m && L) memcpy(p, b.b.out + (size_t)idx * kBuf, m);
            n = L ? m : 0;
            if (addr && addrlen) {
                const uint32_t al = b.alen[idx] < *addrlen ? b.alen[idx] : *addrlen;
                memcpy(addr, &b.addr[idx], al);
                *addrlen = b.alen[idx];
            }
        } else {
            ++q->rx_dropped;   // Deobfuscate returned 0: dropped, read on (conn.go:86)
        }
        if (b.done.fetch_add(1, std::memory_order_acq_rel) + 1 == b.k) {
            std::lock_guard<std::mutex> lk(q->rx_mu);
            q->freelist.push_back(bi);
            q->cv_free.notify_one();
        }
        if (deliver) return n;
    }
}

void coalescer_poke(Coalescer* q) {
    if (!q) return;
    {
        std::lock_guard<std::mutex> a(q->tx_mu);
        std::lock_guard<std::mutex> b(q->rx_mu);
    }
    q->cv_space.notify_all();
    q->cv_ready.notify_all();
}

int coalescer_flush(Coalescer* q) {
    // every accepted datagram is sent: by the flusher, or by stop() before it exits
    const uint64_t target = q->accepted.load();
    {
        std::lock_guard<std::mutex> lk(q->tx_mu);
        q->cv_flush.notify_one();
    }
    while (q->sent.load() < target) std::this_thread::sleep_for(std::chrono::microseconds(20));
    return HYOBFS_OK;
}

void coalescer_stats(const Coalescer* q, uint64_t out[6]) {
    out[0] = q->accepted.load();
    out[1] = q->tx_batches.load();
    out[2] = q->tx_errors.load();
    out[3] = q->received.load();
    out[4] = q->rx_batches.load();
    out[5] = q->rx_dropped.load();
}

}  // namespace hyobfs
