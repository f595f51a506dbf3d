// udp_bench -- host-to-host rate of the Salamander PacketConn wrapper
// (BASELINE config 5): loopback UDP, sender conns obfuscate with
// hyobfs_conn_write_batch (sendmmsg + one GPU batch), receiver conns
// deobfuscate with hyobfs_conn_read_batch (recvmmsg + one GPU batch).
// Every received payload is checked (sequence number + content tag).
//
//   udp_bench [mode=batch|single|raw|coalesce] [pairs=4] [seconds=5] [len=1200] [batch=1024]
//             [threads=2] [wait_us=50] [rate=0]
//
// "raw" sends and receives the same datagrams with plain sendmmsg/recvmmsg and no
// obfuscation: the loopback socket ceiling.  "single" uses WriteTo/ReadFrom, one
// GPU round trip per datagram, the shape of the reference's obfsPacketConn.
// "coalesce" keeps that per-datagram shape (WriteTo / ReadFrom, `threads`
// writer and `threads` reader threads per pair) on coalescing connections
// (hyobfs_conn_set_coalescing: GPU batches of up to `batch` behind the calls).
// rate > 0 offers that many datagrams per second in total (every writer paced to its
// share: whatever is due is sent, then the writer sleeps, at least 20 us): latency at a given load,
// raw against coalesce; 0 = as fast as the writers go (the saturated rate).
// Latency = receive time - send-call time of every 64th datagram (p50, p99).
// Prints one JSON line.
//   g++ -O2 -std=c++17 tools/udp_bench.cpp -Iinclude -Lhysteria_amd -lhyobfs
//       -Wl,-rpath,'$ORIGIN/../hysteria_amd' -lpthread -o tools/udp_bench
#include <arpa/inet.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <netinet/in.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <dirent.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <set>
#include <mutex>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../include/hyobfs_conn.h"

// cgroup v2 CPU throttling so far (nr_throttled, throttled_usec), 0 when unreadable
static void cg_throttle(uint64_t& n, uint64_t& us) {
    n = us = 0;
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.stat", "r")) {
        char k[64];
        unsigned long long v;
        while (fscanf(f, "%63s %llu", k, &v) == 2) {
            if (!strcmp(k, "nr_throttled")) n = v;
            if (!strcmp(k, "throttled_usec")) us = v;
        }
        fclose(f);
    }
}

// CPU time (utime + stime, clock ticks) and name of every thread of this process
struct TaskCpu {
    std::string comm;
    uint64_t ticks;
};
static std::map<int, TaskCpu> task_cpu() {
    std::map<int, TaskCpu> m;
    DIR* d = opendir("/proc/self/task");
    if (!d) return m;
    while (dirent* e = readdir(d)) {
        const int tid = atoi(e->d_name);
        if (tid <= 0) continue;
        char path[64], line[1024];
        snprintf(path, sizeof path, "/proc/self/task/%d/stat", tid);
        FILE* f = fopen(path, "r");
        if (!f) continue;
        const size_t n = fread(line, 1, sizeof line - 1, f);
        fclose(f);
        line[n] = 0;
        char* l = strchr(line, '(');
        char* r = strrchr(line, ')');
        if (!l || !r) continue;
        TaskCpu t{std::string(l + 1, r), 0};
        // fields after the comm: state(3) ... utime(14) stime(15)
        unsigned long long ut = 0, st = 0;
        int field = 3;
        for (char* q = strtok(r + 2, " "); q; q = strtok(nullptr, " "), ++field) {
            if (field == 14) ut = strtoull(q, nullptr, 10);
            if (field == 15) { st = strtoull(q, nullptr, 10); break; }
        }
        t.ticks = ut + st;
        m[tid] = t;
    }
    closedir(d);
    return m;
}

constexpr double kMinSleepNs = 20000.0;   // a paced writer's shortest sleep

static uint64_t tag(uint64_t seq) { return seq * 0x9E3779B97F4A7C15ull ^ 0xD1B54A32D192ED03ull; }

static uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// payload: sequence number, send time (steady clock, ns), then the sequence's tag
static void fill(uint8_t* p, uint32_t len, uint64_t seq) {
    memcpy(p, &seq, 8);
    const uint64_t t = tag(seq);
    for (uint32_t o = 16; o + 8 <= len; o += 8) memcpy(p + o, &t, 8);
}
static void stamp(uint8_t* p) {
    const uint64_t ts = now_ns();
    memcpy(p + 8, &ts, 8);
}

static bool check(const uint8_t* p, uint32_t len, uint32_t want_len) {
    if (len != want_len) return false;
    uint64_t seq;
    memcpy(&seq, p, 8);
    const uint64_t t = tag(seq);
    for (uint32_t o = 16; o + 8 <= len; o += 8)
        if (memcmp(p + o, &t, 8) != 0) return false;
    return true;
}

static int udp_socket(sockaddr_in* bound) {
    int fd = socket(AF_INET, SOCK_DGRAM, 0);
    int big = 64 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
        perror("bind");
        exit(1);
    }
    socklen_t al = sizeof *bound;
    getsockname(fd, reinterpret_cast<sockaddr*>(bound), &al);
    timeval tv{0, 200000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    return fd;
}

struct Pair {
    int sfd = -1, rfd = -1;
    sockaddr_in saddr{}, raddr{};
    hyobfs_salamander* sctx = nullptr;
    hyobfs_salamander* rctx = nullptr;
    hyobfs_conn* sc = nullptr;
    hyobfs_conn* rc = nullptr;
    std::atomic<uint64_t> sent{0}, recvd{0}, bad{0}, calls{0};
    std::mutex lat_mu;
    std::vector<uint64_t> lat;   // sampled send -> receive latencies (ns)
};

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "batch";
    const int pairs = argc > 2 ? atoi(argv[2]) : 4;
    const double seconds = argc > 3 ? atof(argv[3]) : 5.0;
    const uint32_t len = argc > 4 ? (uint32_t)atoi(argv[4]) : 1200;
    const uint32_t batch = argc > 5 ? (uint32_t)atoi(argv[5]) : 1024;
    const uint8_t psk[] = "udp_bench_password";
    const int threads = argc > 6 ? atoi(argv[6]) : 2;
    const uint32_t wait_us = argc > 7 ? (uint32_t)atoi(argv[7]) : 50;
    const double rate = argc > 8 ? atof(argv[8]) : 0.0;   // offered datagrams/s in total, 0 = unpaced
    const bool raw = mode == "raw", coalesce = mode == "coalesce", single = mode == "single" || coalesce;
    if (len < 16 || len > 2040) {
        fprintf(stderr, "len must be in [16, 2040]\n");
        return 2;
    }

    std::vector<Pair> P(pairs);
    for (auto& p : P) {
        p.sfd = udp_socket(&p.saddr);
        p.rfd = udp_socket(&p.raddr);
        if (!raw) {
            int st = hyobfs_salamander_new(psk, sizeof psk - 1, 0, &p.sctx);
            if (st == HYOBFS_OK) st = hyobfs_salamander_new(psk, sizeof psk - 1, 0, &p.rctx);
            if (st == HYOBFS_OK) st = hyobfs_conn_wrap(p.sfd, p.sctx, batch, &p.sc);
            if (st == HYOBFS_OK) st = hyobfs_conn_wrap(p.rfd, p.rctx, batch, &p.rc);
            if (st == HYOBFS_OK && coalesce) st = hyobfs_conn_set_coalescing(p.sc, batch, wait_us);
            if (st == HYOBFS_OK && coalesce) st = hyobfs_conn_set_coalescing(p.rc, batch, wait_us);
            if (st != HYOBFS_OK) {
                fprintf(stderr, "setup: %s\n", hyobfs_status_string(st));
                return 1;
            }
        }
    }

    std::atomic<bool> stop{false}, rstop{false};
    std::vector<std::thread> th;
    std::mutex tid_mu;
    std::set<int> writer_tids, reader_tids;   // the bench's own threads (CPU breakdown)
    auto note_tid = [&](std::set<int>& s) {
        std::lock_guard<std::mutex> lk(tid_mu);
        s.insert((int)syscall(SYS_gettid));
    };
    const int per_side = coalesce ? threads : 1;
    for (int pi = 0; pi < pairs; ++pi)
      for (int ti = 0; ti < per_side; ++ti) {
        Pair& p = P[pi];
        th.emplace_back([&, pi, ti] {   // sender
            (void)prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);   // paced writers wake on time
            note_tid(writer_tids);
            std::vector<uint8_t> buf((size_t)batch * len);
            std::vector<hyobfs_dgram> d(batch);
            std::vector<mmsghdr> mh(batch);
            std::vector<iovec> iov(batch);
            for (uint32_t i = 0; i < batch; ++i) {
                d[i].buf = buf.data() + (size_t)i * len;
                d[i].len = len;
                memcpy(d[i].addr, &p.raddr, sizeof p.raddr);
                d[i].addrlen = sizeof p.raddr;
                iov[i] = {d[i].buf, len};
                memset(&mh[i], 0, sizeof mh[i]);
                mh[i].msg_hdr.msg_iov = &iov[i];
                mh[i].msg_hdr.msg_iovlen = 1;
                mh[i].msg_hdr.msg_name = &p.raddr;
                mh[i].msg_hdr.msg_namelen = sizeof p.raddr;
            }
            uint64_t seq = (uint64_t)pi << 48 | (uint64_t)ti << 40;
            const double share = rate / (double)(pairs * per_side);   // this writer's datagrams/s
            const uint64_t t_start = now_ns();
            uint64_t issued = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                uint32_t nb = batch;
                if (share > 0) {   // send what is due by now, up to a batch
                    const uint64_t now = now_ns();
                    const uint64_t want = (uint64_t)((double)(now - t_start) * share * 1e-9);
                    if (want <= issued) {   // sleep until the next datagram is due, at least
                        // kMinSleepNs: a wakeup per datagram would cost the writer a core at
                        // 250 k datagrams/s and eat the box's CPU quota (what is due after a
                        // longer sleep goes out together, stamped when each is sent)
                        const double next_ns = (double)(issued + 1) / share * 1e9 + (double)t_start;
                        const double gap = next_ns - (double)now;
                        std::this_thread::sleep_for(std::chrono::nanoseconds((int64_t)std::max(gap, kMinSleepNs)));
                        continue;
                    }
                    nb = (uint32_t)std::min<uint64_t>(want - issued, batch);
                    issued += nb;
                }
                for (uint32_t i = 0; i < nb; ++i) fill(d[i].buf, len, seq++);
                if (single) {
                    for (uint32_t i = 0; i < nb && !stop.load(std::memory_order_relaxed); ++i) {
                        stamp(d[i].buf);
                        if (hyobfs_conn_write_to(p.sc, d[i].buf, len, &p.raddr, sizeof p.raddr) > 0) p.sent++;
                    }
                } else if (raw) {
                    for (uint32_t i = 0; i < nb; ++i) stamp(d[i].buf);
                    uint32_t done = 0;
                    while (done < nb) {
                        int r = sendmmsg(p.sfd, mh.data() + done, nb - done, 0);
                        if (r <= 0) break;
                        done += r;
                    }
                    p.sent += done;
                } else {
                    for (uint32_t i = 0; i < nb; ++i) stamp(d[i].buf);
                    int r = hyobfs_conn_write_batch(p.sc, d.data(), nb);
                    if (r > 0) p.sent += r;
                }
            }
        });
        th.emplace_back([&] {   // receiver
            note_tid(reader_tids);
            std::vector<uint8_t> buf((size_t)batch * 2048);
            std::vector<hyobfs_dgram> d(batch);
            std::vector<mmsghdr> mh(batch);
            std::vector<iovec> iov(batch);
            for (uint32_t i = 0; i < batch; ++i) {
                d[i].buf = buf.data() + (size_t)i * 2048;
                d[i].cap = 2048;
                iov[i] = {d[i].buf, 2048};
            }
            while (!rstop.load(std::memory_order_relaxed)) {
                int k;
                if (single) {
                    int64_t n = hyobfs_conn_read_from(p.rc, d[0].buf, 2048, nullptr, nullptr);
                    k = n > 0 ? 1 : 0;
                    d[0].len = n > 0 ? (uint32_t)n : 0;
                } else if (raw) {
                    for (uint32_t i = 0; i < batch; ++i) {
                        memset(&mh[i], 0, sizeof mh[i]);
                        mh[i].msg_hdr.msg_iov = &iov[i];
                        mh[i].msg_hdr.msg_iovlen = 1;
                    }
                    k = recvmmsg(p.rfd, mh.data(), batch, MSG_WAITFORONE, nullptr);
                    for (int i = 0; i < k; ++i) d[i].len = mh[i].msg_len;
                } else {
                    k = hyobfs_conn_read_batch(p.rc, d.data(), batch);
                }
                if (k <= 0) continue;
                p.calls++;
                uint64_t bad = 0;
                const uint64_t t_rx = now_ns();
                for (int i = 0; i < k; ++i) {
                    bad += !check(d[i].buf, d[i].len, len);
                    uint64_t seq, ts;
                    memcpy(&seq, d[i].buf, 8);
                    memcpy(&ts, d[i].buf + 8, 8);
                    if ((seq & 63) == 0 && t_rx > ts) {   // every 64th datagram
                        std::lock_guard<std::mutex> lk(p.lat_mu);
                        p.lat.push_back(t_rx - ts);
                    }
                }
                p.recvd += k;
                p.bad += bad;
            }
        });
    }

    // warm up 0.5 s, then count over the timed window
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    uint64_t thr_n0, thr_us0, thr_n1, thr_us1;
    cg_throttle(thr_n0, thr_us0);
    rusage ru0{}, ru1{};
    getrusage(RUSAGE_SELF, &ru0);
    const auto tc0 = task_cpu();
    uint64_t r0 = 0, s0 = 0;
    for (auto& p : P) r0 += p.recvd, s0 += p.sent;
    // coalescing counters (hyobfs_conn_stats: [1] tx batches, [4] rx batches) over the window
    auto batches = [&](uint64_t& txb, uint64_t& rxb) {
        txb = rxb = 0;
        for (auto& p : P) {
            uint64_t st[6] = {};
            if (coalesce && hyobfs_conn_stats(p.sc, st) == HYOBFS_OK) txb += st[1];
            if (coalesce && hyobfs_conn_stats(p.rc, st) == HYOBFS_OK) rxb += st[4];
        }
    };
    uint64_t txb0, rxb0, txb1, rxb1;
    batches(txb0, rxb0);
    const auto t0 = std::chrono::steady_clock::now();
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    uint64_t r1 = 0, s1 = 0;
    for (auto& p : P) r1 += p.recvd, s1 += p.sent;
    batches(txb1, rxb1);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    getrusage(RUSAGE_SELF, &ru1);
    const auto tc1 = task_cpu();
    cg_throttle(thr_n1, thr_us1);
    // cores used per thread class over the window: the bench's writers and readers, and
    // every other thread (the library's coalescer threads, the HIP runtime's) by name
    const double hz = (double)sysconf(_SC_CLK_TCK);
    std::map<std::string, double> by_class;
    for (const auto& [tid, t1] : tc1) {
        auto it = tc0.find(tid);
        const uint64_t d = t1.ticks - (it != tc0.end() ? it->second.ticks : 0);
        const std::string cls = writer_tids.count(tid) ? "bench_writers" : reader_tids.count(tid) ? "bench_readers"
                                                                                                    : "other:" + t1.comm;
        by_class[cls] += (double)d / hz;
    }
    auto tv_s = [](const timeval& t) { return (double)t.tv_sec + 1e-6 * (double)t.tv_usec; };
    const double cpu_s = tv_s(ru1.ru_utime) - tv_s(ru0.ru_utime) + tv_s(ru1.ru_stime) - tv_s(ru0.ru_stime);
    stop = true;
    std::this_thread::sleep_for(std::chrono::milliseconds(400));
    rstop = true;
    for (auto& t : th) t.join();
    uint64_t bad = 0, calls = 0, sent = 0, recvd = 0;
    std::vector<uint64_t> lat;
    for (auto& p : P) lat.insert(lat.end(), p.lat.begin(), p.lat.end());
    std::sort(lat.begin(), lat.end());
    auto pct = [&](double q) { return lat.empty() ? 0.0 : lat[(size_t)(q * (lat.size() - 1))] / 1e3; };
    for (auto& p : P) {
        bad += p.bad, calls += p.calls, sent += p.sent, recvd += p.recvd;
        if (p.sc) hyobfs_conn_free(p.sc);   // a connection owns its fd: free closes it
        if (p.rc) hyobfs_conn_free(p.rc);
        if (!p.sc) close(p.sfd);
        if (!p.rc) close(p.rfd);
        hyobfs_salamander_free(p.sctx);
        hyobfs_salamander_free(p.rctx);
    }
    const double rx = (double)(r1 - r0), tx = (double)(s1 - s0);
    std::string cls_json;
    for (const auto& [k, v] : by_class) {
        char b[160];
        snprintf(b, sizeof b, "%s\"%s\": %.2f", cls_json.empty() ? "" : ", ", k.c_str(), v / dt);
        cls_json += b;
    }
    printf("{\"mode\": \"%s\", \"offered_rate\": %.0f, \"pairs\": %d, \"threads_per_side\": %d, \"wait_us\": %u, \"len\": %u, \"batch\": %u, \"seconds\": %.3f, "
           "\"rx_datagrams_per_s\": %.0f, \"tx_datagrams_per_s\": %.0f, \"rx_payload_GiB_s\": %.4f, "
           "\"tx_payload_GiB_s\": %.4f, \"loss_frac\": %.4f, \"bad\": %llu, \"avg_per_read\": %.1f, "
           "\"latency_us_p50\": %.1f, \"latency_us_p99\": %.1f, \"latency_samples\": %zu, "
           "\"cpu_cores_used\": %.2f, \"cgroup_throttled_periods\": %llu, \"cgroup_throttled_ms\": %.1f, \"cpu_cores_by_thread\": {%s}, "
           "\"tx_batches_per_s\": %.0f, \"rx_batches_per_s\": %.0f}\n",
           mode.c_str(), rate, pairs, per_side, coalesce ? wait_us : 0u, len, batch, dt, rx / dt, tx / dt, rx * len / dt / (1u << 30), tx * len / dt / (1u << 30),
           sent ? 1.0 - (double)recvd / (double)sent : 0.0, (unsigned long long)bad,
           calls ? (double)recvd / (double)calls : 0.0, pct(0.5), pct(0.99), lat.size(), cpu_s / dt,
           (unsigned long long)(thr_n1 - thr_n0), (double)(thr_us1 - thr_us0) / 1e3, cls_json.c_str(),
           (double)(txb1 - txb0) / dt, (double)(rxb1 - rxb0) / dt);
    return bad ? 1 : 0;
}
