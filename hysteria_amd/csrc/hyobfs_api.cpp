// hyobfs_api.cpp -- the C ABI of include/hyobfs.h.
//
// A context mirrors salamanderObfuscator (extras/obfs/salamander.go:26-32):
// the PSK (here also its BLAKE2b prefix state, KeyParams), the salt source
// (RandSrc), and a lock for the per-packet path (lk).  It is bound to one
// HIP device.  Every compute call runs the gfx950 kernels of salamander.hip;
// there is no CPU path.
#ifdef HYOBFS_EMULATE
#include "hip_emu.h"   // tests/emu: CPU emulation for the CPU test tier, never shipped
#else
#include <hip/hip_runtime.h>
#endif

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/hyobfs.h"
#include "conn_coalesce.h"
#include "kernels.h"

using hyobfs::BatchParams;
using hyobfs::KeyParams;

struct hyobfs_salamander {
    std::atomic<int> refs{1};   // the caller's reference + one per connection (hyobfs::ctx_retain)
    std::vector<uint8_t> psk;
    int device = 0;
    KeyParams kp{};
    hipStream_t stream = nullptr;
    std::mutex mu;              // per-packet path, salt source, owned buffers (lk)
    uint64_t rng = 0;           // SplitMix64 state (RandSrc)
    std::atomic<int> kernel{0}; // HYOBFS_KERNEL_* for batch launches (set_kernel may race batch calls)
    // per-packet staging in mapped pinned host memory: [in | out | salt | len | total]
    uint8_t* stage = nullptr;
    uint8_t* stage_dev = nullptr;
    size_t stage_cap = 0;       // bytes for each of in and out
    // packed batches without a caller workspace: tile-sum scratch allocated
    // stream-ordered from this context-owned pool and freed behind the launch
    // on the same stream, so any number of caller streams (and threads) share
    // it and device memory stays bounded (release threshold below)
    hipMemPool_t pool = nullptr;
    std::mutex pool_mu;          // creation only
    // host-batch pipeline: three slots, one stream each (see *_host)
    struct Slot {
        hipStream_t s = nullptr;
        uint8_t* in = nullptr;      // chunk x in_stride
        uint8_t* out = nullptr;     // chunk x out_stride
        uint32_t* len = nullptr;    // chunk
        uint64_t* salts = nullptr;  // chunk
        uint32_t* olen = nullptr;   // chunk
        void* ws = nullptr;
        uint64_t in_cap = 0, out_cap = 0, n_cap = 0, ws_cap = 0;
    } slot[3];
    std::mutex pipe_mu;
};

namespace {

struct DeviceGuard {   // keep the caller's current device unchanged
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// ---- BLAKE2b compression on the host, used only for the PSK-only prefix
// blocks (blocks that hold no salt byte) when len(PSK) > 120.
const uint64_t kIV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                         0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                         0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
const uint8_t kSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

void host_compress(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
    uint64_t v[16];
    for (int i = 0; i < 8; ++i) {
        v[i] = h[i];
        v[i + 8] = kIV[i];
    }
    v[12] ^= t;
    if (last) v[14] = ~v[14];
    auto G = [&](int a, int b, int c, int d, uint64_t x, uint64_t y) {
        v[a] = v[a] + v[b] + x;
        v[d] = rotr(v[d] ^ v[a], 32);
        v[c] = v[c] + v[d];
        v[b] = rotr(v[b] ^ v[c], 24);
        v[a] = v[a] + v[b] + y;
        v[d] = rotr(v[d] ^ v[a], 16);
        v[c] = v[c] + v[d];
        v[b] = rotr(v[b] ^ v[c], 63);
    };
    for (int r = 0; r < 12; ++r) {
        const uint8_t* s = kSigma[r];
        G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

void block_words(const uint8_t* msg, size_t msg_len, size_t blk, uint64_t m[16]) {
    for (int j = 0; j < 16; ++j) {
        uint64_t w = 0;
        for (int b = 7; b >= 0; --b) {
            const size_t pos = 128 * blk + 8 * j + b;
            w = (w << 8) | (pos < msg_len ? msg[pos] : 0u);
        }
        m[j] = w;
    }
}

// keyLocked's hash, BLAKE2b-256(PSK || salt), split at the first block that
// holds a salt byte: host compresses the blocks before it, the GPU the rest.
KeyParams make_key_params(const uint8_t* psk, size_t psk_len) {
    KeyParams k{};
    const size_t T = psk_len + HYOBFS_SALT_LEN;
    const size_t nb = (T + 127) / 128;                  // T >= 12, so nb >= 1
    const size_t fb = psk_len / 128;                   // block with salt[0]
    std::vector<uint8_t> msg(T, 0);                     // salt bytes stay 0
    if (psk_len) std::memcpy(msg.data(), psk, psk_len);
    for (int i = 0; i < 8; ++i) k.h[i] = kIV[i];
    k.h[0] ^= 0x01010000ull ^ (uint64_t)HYOBFS_KEY_LEN;  // digest 32, unkeyed
    for (size_t b = 0; b < fb; ++b) {                   // PSK-only blocks
        uint64_t m[16];
        block_words(msg.data(), T, b, m);
        host_compress(k.h, m, 128ull * (b + 1), false);
    }
    k.nblk = (uint32_t)(nb - fb);                       // 1 or 2
    for (uint32_t b = 0; b < k.nblk; ++b) {
        block_words(msg.data(), T, fb + b, k.m + 16 * b);
        k.t[b] = (fb + b + 1 == nb) ? (uint64_t)T : 128ull * (fb + b + 1);
    }
    k.salt_pos = (uint32_t)(psk_len - 128 * fb);
    return k;
}

inline uint64_t splitmix_next(uint64_t& s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// Ensure the mapped staging buffer holds `bytes` of input and of output.
int ensure_stage(hyobfs_salamander* c, size_t bytes) {
    if (bytes <= c->stage_cap && c->stage) return HYOBFS_OK;
    size_t cap = c->stage_cap ? c->stage_cap : 4096;
    while (cap < bytes) cap *= 2;
    if (c->stage) (void)hipHostFree(c->stage);
    c->stage = nullptr;
    c->stage_cap = 0;
    void* p = nullptr;
    if (hipHostMalloc(&p, 2 * cap + 64, hipHostMallocMapped) != hipSuccess) return HYOBFS_ERR_NOMEM;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
        (void)hipHostFree(p);
        return HYOBFS_ERR_HIP;
    }
    c->stage = static_cast<uint8_t*>(p);
    c->stage_dev = static_cast<uint8_t*>(d);
    c->stage_cap = cap;
    return HYOBFS_OK;
}

// One datagram through the batch kernel, staged in mapped pinned memory.
// Caller holds c->mu and has checked the reference's length rules.
size_t run_one(hyobfs_salamander* c, bool obf, const uint8_t* in, size_t in_len,
               const uint8_t* salt, uint8_t* out, size_t W) {
    DeviceGuard g(c->device);
    if (!g.ok) return 0;
    const size_t need = in_len > W ? in_len : W;
    if (ensure_stage(c, need + 16) != HYOBFS_OK) return 0;
    // layout: in at 0, out at cap (16-aligned), salt + len words at 2*cap
    uint8_t* h_in = c->stage;
    uint8_t* h_out = c->stage + c->stage_cap;
    uint8_t* h_misc = c->stage + 2 * c->stage_cap;
    if (in_len) std::memcpy(h_in, in, in_len);
    if (obf) std::memcpy(h_misc, salt, HYOBFS_SALT_LEN);
    uint32_t* h_len = reinterpret_cast<uint32_t*>(h_misc + 8);
    *h_len = 0xFFFFFFFFu;
    BatchParams b{};
    b.kernel = c->kernel.load(std::memory_order_relaxed);
    b.n = 1;
    b.in = c->stage_dev;
    b.len_uniform = (uint32_t)in_len;
    b.salts = reinterpret_cast<const uint64_t*>(c->stage_dev + 2 * c->stage_cap);
    b.out = c->stage_dev + c->stage_cap;
    b.out_cap = W;
    b.out_stride = W;   // one slot of exactly len(out) = W bytes
    b.pkt_cap = (uint32_t)W;
    b.out_len = reinterpret_cast<uint32_t*>(c->stage_dev + 2 * c->stage_cap + 8);
    if (hyobfs::launch_salamander(obf, b, c->kp, c->stream) != hipSuccess) return 0;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return 0;
    if (*h_len != W) return 0;
    std::memcpy(out, h_out, W);
    return W;
}

// The context's scratch pool (created on first use).
constexpr uint64_t kPoolKeepBytes = 32ull << 20;   // cached across calls; more is returned at sync points
hipMemPool_t scratch_pool(hyobfs_salamander* c) {
    std::lock_guard<std::mutex> lk(c->pool_mu);
    if (c->pool) return c->pool;
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = c->device;
    hipMemPool_t p = nullptr;
    if (hipMemPoolCreate(&p, &props) != hipSuccess) return nullptr;
    uint64_t keep = kPoolKeepBytes;
    (void)hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep);
    c->pool = p;
    return p;
}

// The launch parameters of a batch (no device call).
int fill_params(hyobfs_salamander* c, const hyobfs_batch* b, bool obf, BatchParams& bp) {
    if (!c || !b) return HYOBFS_ERR_INVALID;
    if (b->n && (!b->in || !b->out)) return HYOBFS_ERR_INVALID;
    if (obf && b->n && !b->salts) return HYOBFS_ERR_INVALID;
    if (reinterpret_cast<uintptr_t>(b->out) & 15) return HYOBFS_ERR_INVALID;
    if (b->out_stride > hyobfs::kMaxDatagram) return HYOBFS_ERR_INVALID;
    bp = BatchParams{};
    bp.n = b->n;
    bp.in = b->in;
    bp.in_off = b->in_off;
    bp.in_stride = b->in_stride;
    bp.in_len = b->in_len;
    bp.len_uniform = b->len_uniform;
    uint64_t cap = b->pkt_cap ? b->pkt_cap : 0;
    if (b->out_stride && (cap == 0 || b->out_stride < cap)) cap = b->out_stride;
    bp.pkt_cap = (uint32_t)cap;
    bp.salts = b->salts;
    bp.out = b->out;
    bp.out_cap = b->out_cap;
    bp.out_stride = b->out_stride;
    bp.out_off = b->out_off;
    bp.out_len = b->out_len;
    bp.out_total = reinterpret_cast<unsigned long long*>(b->out_total);
    bp.kernel = c->kernel.load(std::memory_order_relaxed);
    // device scratch: the caller's workspace, or (run_batch) the context's pool
    const uint64_t need = hyobfs::batch_workspace_bytes(obf, bp);
    if (need && b->workspace) {
        if (b->workspace_bytes < need) return HYOBFS_ERR_INVALID;
        bp.scratch = b->workspace;
        bp.tile_sums = static_cast<uint64_t*>(b->workspace);   // (packed, explicit offsets: the tile sums)
    }
    return HYOBFS_OK;
}

int validate_and_fill(hyobfs_salamander* c, const hyobfs_batch* b, bool obf, BatchParams& bp,
                      hipStream_t s) {
    const int rc = fill_params(c, b, obf, bp);
    if (rc != HYOBFS_OK) return rc;
    if (b->out_total && hipMemsetAsync(b->out_total, 0, sizeof(uint64_t), s) != hipSuccess)
        return HYOBFS_ERR_HIP;
    return HYOBFS_OK;
}

int run_batch(hyobfs_salamander* c, const hyobfs_batch* b, void* stream, bool obf) {
    if (!c || !b) return HYOBFS_ERR_INVALID;
    DeviceGuard g(c->device);
    if (!g.ok) return HYOBFS_ERR_HIP;
    hipStream_t s = static_cast<hipStream_t>(stream);   // NULL = the HIP null stream
    BatchParams bp;
    const int rc = validate_and_fill(c, b, obf, bp, s);
    if (rc != HYOBFS_OK) return rc;
    void* scratch = nullptr;
    const uint64_t need = hyobfs::batch_workspace_bytes(obf, bp);
    if (need && !b->workspace) {   // no caller workspace: the context's pool
        hipMemPool_t pool = scratch_pool(c);
        if (!pool) return HYOBFS_ERR_HIP;
        if (hipMallocFromPoolAsync(&scratch, need, pool, s) != hipSuccess) return HYOBFS_ERR_NOMEM;
        bp.scratch = scratch;
        bp.tile_sums = static_cast<uint64_t*>(scratch);
    }
    const hipError_t e = hyobfs::launch_salamander(obf, bp, c->kp, s);
    if (scratch && hipFreeAsync(scratch, s) != hipSuccess) return HYOBFS_ERR_HIP;   // after the launch, in stream order
    return e == hipSuccess ? HYOBFS_OK : HYOBFS_ERR_HIP;
}

// One batch per shard, each on its own context's stream (and device): launch all, then wait for all.
int run_sharded(hyobfs_salamander* const* ctxs, const hyobfs_batch* batches, int nshards, bool obf) {
    if (nshards < 0 || (nshards && (!ctxs || !batches))) return HYOBFS_ERR_INVALID;
    for (int i = 0; i < nshards; ++i) {
        if (!ctxs[i]) return HYOBFS_ERR_INVALID;
        for (int j = 0; j < i; ++j)
            if (ctxs[j] == ctxs[i]) return HYOBFS_ERR_INVALID;   // one context (stream) per shard
    }
    int rc = HYOBFS_OK;
    int launched = 0;
    for (; launched < nshards; ++launched) {
        rc = run_batch(ctxs[launched], &batches[launched], ctxs[launched]->stream, obf);
        if (rc != HYOBFS_OK) break;
    }
    for (int i = 0; i < launched; ++i) {   // drain what was launched, even after a failure
        DeviceGuard g(ctxs[i]->device);
        if ((!g.ok || hipStreamSynchronize(ctxs[i]->stream) != hipSuccess) && rc == HYOBFS_OK) rc = HYOBFS_ERR_HIP;
    }
    return rc;
}

// Grow a device buffer (caller holds the pipeline lock; the slot's stream is idle).
template <class T>
int grow(T*& p, uint64_t& cap, uint64_t need_bytes) {
    if (cap >= need_bytes && p) return HYOBFS_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    void* q = nullptr;
    if (hipMalloc(&q, need_bytes ? need_bytes : 16) != hipSuccess) return HYOBFS_ERR_NOMEM;
    p = static_cast<T*>(q);
    cap = need_bytes;
    return HYOBFS_OK;
}

// Whether the kernels may read and write host pointer p where it is: pinned host
// memory mapped into the device's address space under the same address
// (hipHostMalloc, hyobfs_host_alloc).  Pageable memory is not (it is staged).
bool device_mapped_host(const void* p) {
    if (!p) return true;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable: not an error of the call
        return false;
    }
    return a.type == hipMemoryTypeHost && a.devicePointer == p;
}

// HYOBFS_HOST_ZEROCOPY=0 stages even mapped host buffers (A/B knob, read once)
bool host_zerocopy_on() {
    static const bool v = [] {
        const char* e = std::getenv("HYOBFS_HOST_ZEROCOPY");
        return !e || std::atoi(e) != 0;
    }();
    return v;
}

// Host batch.  When every buffer the kernels touch is mapped pinned memory, one
// batch call runs in place on it (the kernels read and write across PCIe, no
// staging copies: 38.2 against 32.9 GiB/s for 1M x 1200 B).
// Otherwise through the three-slot pipeline: H2D(k) | kernels(k) | D2H(k) on
// slot k % 3's stream; streams overlap each other, so the copy engines and
// the compute queue work on different chunks at once.
int run_host(hyobfs_salamander* c, const hyobfs_batch* b, uint64_t chunk, bool obf) {
    if (!c || !b) return HYOBFS_ERR_INVALID;
    if (b->n == 0) return HYOBFS_OK;
    if (!b->in || !b->out || b->in_off || b->in_stride == 0 || b->out_stride == 0) return HYOBFS_ERR_INVALID;
    if (obf && !b->salts) return HYOBFS_ERR_INVALID;
    if (b->out_stride > hyobfs::kMaxDatagram) return HYOBFS_ERR_INVALID;
    if (b->out_cap < b->n * b->out_stride) return HYOBFS_ERR_INVALID;
    DeviceGuard g(c->device);
    if (!g.ok) return HYOBFS_ERR_HIP;
    std::lock_guard<std::mutex> lk(c->pipe_mu);
    if (!c->slot[0].s && hipStreamCreateWithFlags(&c->slot[0].s, hipStreamNonBlocking) != hipSuccess)
        return HYOBFS_ERR_HIP;
    if (host_zerocopy_on() && device_mapped_host(b->in) && device_mapped_host(b->out) &&
        device_mapped_host(b->in_len) && device_mapped_host(obf ? b->salts : nullptr) &&
        device_mapped_host(b->out_len)) {
        hyobfs_batch d = *b;
        d.out_off = nullptr;
        d.out_total = nullptr;
        d.workspace = nullptr;
        d.workspace_bytes = 0;
        int rc = run_batch(c, &d, c->slot[0].s, obf);
        if (hipStreamSynchronize(c->slot[0].s) != hipSuccess && rc == HYOBFS_OK) rc = HYOBFS_ERR_HIP;
        return rc;
    }
    if (chunk == 0) chunk = std::max<uint64_t>(4096, (64ull << 20) / std::max<uint64_t>(b->in_stride, 1));
    chunk = std::min<uint64_t>(chunk, b->n);
    const uint64_t in_bytes = chunk * b->in_stride, out_bytes = chunk * b->out_stride;
    for (auto& sl : c->slot) {
        if (!sl.s && hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking) != hipSuccess) return HYOBFS_ERR_HIP;
        uint64_t dummy = 0;
        int rc = HYOBFS_OK;
        if (sl.in_cap < in_bytes) rc |= grow(sl.in, sl.in_cap, in_bytes);
        if (sl.out_cap < out_bytes) rc |= grow(sl.out, sl.out_cap, out_bytes);
        if (sl.n_cap < chunk) {
            uint64_t c1 = 0, c2 = 0, c3 = 0;
            rc |= grow(sl.len, c1, chunk * 4);
            rc |= grow(sl.salts, c2, chunk * 8);
            rc |= grow(sl.olen, c3, chunk * 4);
            sl.n_cap = chunk;
        }
        const uint64_t ws_need = hyobfs_batch_workspace_size(chunk);
        if (sl.ws_cap < ws_need) rc |= grow(sl.ws, sl.ws_cap, ws_need);
        (void)dummy;
        if (rc != HYOBFS_OK) return HYOBFS_ERR_NOMEM;
    }
    const uint64_t nchunks = (b->n + chunk - 1) / chunk;
    // enqueue every chunk; on a failure stop enqueueing, but always drain the
    // three streams before returning: copies already queued still reference
    // the caller's host buffers
    auto enqueue = [&]() -> int {
      for (uint64_t k = 0; k < nchunks; ++k) {
        auto& sl = c->slot[k % 3];
        const uint64_t first = k * chunk, m = std::min<uint64_t>(chunk, b->n - first);
        hipStream_t s = sl.s;
        // slot reuse: the previous chunk on this stream is ordered before us
        if (hipMemcpyAsync(sl.in, b->in + first * b->in_stride, m * b->in_stride, hipMemcpyHostToDevice, s) !=
            hipSuccess)
            return HYOBFS_ERR_HIP;
        if (b->in_len &&
            hipMemcpyAsync(sl.len, b->in_len + first, m * 4, hipMemcpyHostToDevice, s) != hipSuccess)
            return HYOBFS_ERR_HIP;
        if (obf && hipMemcpyAsync(sl.salts, b->salts + first, m * 8, hipMemcpyHostToDevice, s) != hipSuccess)
            return HYOBFS_ERR_HIP;
        hyobfs_batch d{};
        d.n = m;
        d.in = sl.in;
        d.in_stride = b->in_stride;
        d.in_len = b->in_len ? sl.len : nullptr;
        d.len_uniform = b->len_uniform;
        d.pkt_cap = b->pkt_cap;
        d.salts = obf ? sl.salts : nullptr;
        d.out = sl.out;
        d.out_cap = m * b->out_stride;
        d.out_stride = b->out_stride;
        d.out_len = b->out_len ? sl.olen : nullptr;
        d.workspace = sl.ws;
        d.workspace_bytes = sl.ws_cap;
        const int rc = run_batch(c, &d, s, obf);
        if (rc != HYOBFS_OK) return rc;
        if (hipMemcpyAsync(b->out + first * b->out_stride, sl.out, m * b->out_stride, hipMemcpyDeviceToHost, s) !=
            hipSuccess)
            return HYOBFS_ERR_HIP;
        if (b->out_len &&
            hipMemcpyAsync(b->out_len + first, sl.olen, m * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
            return HYOBFS_ERR_HIP;
      }
      return HYOBFS_OK;
    };
    int rc = enqueue();
    for (auto& sl : c->slot)
        if (hipStreamSynchronize(sl.s) != hipSuccess && rc == HYOBFS_OK) rc = HYOBFS_ERR_HIP;
    return rc;
}

}  // namespace

extern "C" {

int hyobfs_abi_version(void) { return HYOBFS_ABI_VERSION; }

#if __has_include("build_id.h")
#include "build_id.h"   // generated by the Makefile: the kernel-source hash
#endif
#ifndef HYOBFS_BUILD_ID
#define HYOBFS_BUILD_ID "unknown"
#endif
const char* hyobfs_build_id(void) { return HYOBFS_BUILD_ID; }

const char* hyobfs_status_string(int st) {
    switch (st) {
        case HYOBFS_OK: return "ok";
        case HYOBFS_ERR_PSK_TOO_SHORT: return "PSK must be at least 4 bytes";
        case HYOBFS_ERR_INVALID: return "invalid argument";
        case HYOBFS_ERR_HIP: return "HIP runtime error";
        case HYOBFS_ERR_NOMEM: return "out of memory";
        case HYOBFS_ERR_NO_DEVICE: return "no usable gfx950 device";
        case HYOBFS_ERR_IO: return "socket I/O error";
        case HYOBFS_ERR_CLOSED: return "use of closed connection";
        default: return "unknown status";
    }
}

int hyobfs_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int hyobfs_device_pci_bus_id(int device, char* buf, int len) {
    if (!buf || len < 13 || device < 0 || device >= hyobfs_device_count()) return HYOBFS_ERR_INVALID;
    return hipDeviceGetPCIBusId(buf, len, device) == hipSuccess ? HYOBFS_OK : HYOBFS_ERR_HIP;
}

int hyobfs_salamander_new(const uint8_t* psk, size_t psk_len, int device, hyobfs_salamander** out) {
    if (!out) return HYOBFS_ERR_INVALID;
    if (psk_len < HYOBFS_PSK_MIN_LEN) return HYOBFS_ERR_PSK_TOO_SHORT;   // salamander.go:35-37
    if (!psk) return HYOBFS_ERR_INVALID;
    if (device < 0 || device >= hyobfs_device_count() || !is_gfx950(device)) return HYOBFS_ERR_NO_DEVICE;
    auto* c = new (std::nothrow) hyobfs_salamander();
    if (!c) return HYOBFS_ERR_NOMEM;
    c->psk.assign(psk, psk + psk_len);                                  // pskCopy, :38
    c->device = device;
    c->kp = make_key_params(psk, psk_len);
    c->rng = (uint64_t)std::chrono::high_resolution_clock::now().time_since_epoch().count();  // :43
    {
        DeviceGuard g(device);
        if (!g.ok || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            delete c;
            return HYOBFS_ERR_HIP;
        }
    }
    *out = c;
    return HYOBFS_OK;
}

}  // extern "C"

namespace hyobfs {
void ctx_retain(hyobfs_salamander* c) { c->refs.fetch_add(1, std::memory_order_relaxed); }
void ctx_release(hyobfs_salamander* c) {
    if (!c || c->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
    {
        DeviceGuard g(c->device);
        if (c->stream) {
            (void)hipStreamSynchronize(c->stream);
            (void)hipStreamDestroy(c->stream);
        }
        if (c->pool) {
            // scratch frees are queued on the callers' streams, which may be gone
            // by now: wait for the whole device before the pool goes
            (void)hipDeviceSynchronize();
            (void)hipMemPoolDestroy(c->pool);
        }
        if (c->stage) (void)hipHostFree(c->stage);
        for (auto& sl : c->slot) {
            if (sl.s) {
                (void)hipStreamSynchronize(sl.s);
                (void)hipStreamDestroy(sl.s);
            }
            (void)hipFree(sl.in);
            (void)hipFree(sl.out);
            (void)hipFree(sl.len);
            (void)hipFree(sl.salts);
            (void)hipFree(sl.olen);
            (void)hipFree(sl.ws);
        }
    }
    delete c;
}
// ---- the coalescer's asynchronous batches (conn_coalesce.h)
struct GpuQueue {
    hyobfs_salamander* ctx = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t ev[4] = {};
};

static bool coalesce_spin() {
    static const bool v = [] {
        const char* e = std::getenv("HYOBFS_COALESCE_SPIN");
        return e && std::atoi(e) != 0;
    }();
    return v;
}

GpuQueue* gpu_queue_new(hyobfs_salamander* c) {
    DeviceGuard g(c->device);
    if (!g.ok) return nullptr;
    auto* q = new (std::nothrow) GpuQueue();
    if (!q) return nullptr;
    q->ctx = c;
    bool ok = hipStreamCreateWithFlags(&q->s, hipStreamNonBlocking) == hipSuccess;
    for (auto& e : q->ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        gpu_queue_free(q);
        return nullptr;
    }
    return q;
}

void gpu_queue_free(GpuQueue* q) {
    if (!q) return;
    DeviceGuard g(q->ctx->device);
    if (q->s) (void)hipStreamSynchronize(q->s);
    for (auto& e : q->ev)
        if (e) (void)hipEventDestroy(e);
    if (q->s) (void)hipStreamDestroy(q->s);
    delete q;
}

int gpu_queue_submit(GpuQueue* q, const hyobfs_batch* b, bool obf, int slot) {
    const int rc = run_batch(q->ctx, b, q->s, obf);
    if (rc != HYOBFS_OK) return rc;
    DeviceGuard g(q->ctx->device);
    return hipEventRecord(q->ev[slot & 3], q->s) == hipSuccess ? HYOBFS_OK : HYOBFS_ERR_HIP;
}

// Waits for the slot's batch by sleeping between event queries.  hipEventSynchronize
// busy-waits here even on a blocking-sync event: with 16 connections' streams sharing the
// GPU's hardware queues a batch takes ~100 us, and the coalescer threads spent that much
// CPU per batch spinning -- 12 of the box's 16 cores at half load (a phase probe,
// tools/ab_patches/coalesce_cpu_probe.patch).  A GPU step takes >= ~18 us,
// so the first query comes after 8 us and the later ones every 8-16 us: a few us of CPU
// per batch and at most ~16 us of added latency.  HYOBFS_COALESCE_SPIN=1 spins instead.
int gpu_queue_wait(GpuQueue* q, int slot) {
    hipEvent_t e = q->ev[slot & 3];
    if (coalesce_spin()) return hipEventSynchronize(e) == hipSuccess ? HYOBFS_OK : HYOBFS_ERR_HIP;
    for (uint32_t us = 8;; us = us < 16 ? us * 2 : 16) {
        const hipError_t r = hipEventQuery(e);
        if (r == hipSuccess) return HYOBFS_OK;
        if (r != hipErrorNotReady) return HYOBFS_ERR_HIP;
        std::this_thread::sleep_for(std::chrono::microseconds(us));
    }
}

}  // namespace hyobfs

extern "C" {

// The caller's reference; a connection still using the context keeps it alive
// until that connection is freed (hyobfs_conn_free).
void hyobfs_salamander_free(hyobfs_salamander* c) { hyobfs::ctx_release(c); }

int hyobfs_salamander_device(const hyobfs_salamander* c) { return c ? c->device : -1; }

int hyobfs_salamander_set_kernel(hyobfs_salamander* c, int kernel) {
    if (!c || kernel < HYOBFS_KERNEL_AUTO || kernel > HYOBFS_KERNEL_FLAT) return HYOBFS_ERR_INVALID;
    c->kernel.store(kernel, std::memory_order_relaxed);
    return HYOBFS_OK;
}

void hyobfs_salamander_seed(hyobfs_salamander* c, uint64_t seed) {
    if (!c) return;
    std::lock_guard<std::mutex> lk(c->mu);
    c->rng = seed;
}

void hyobfs_salamander_next_salts(hyobfs_salamander* c, uint8_t* salts, size_t n) {
    if (!c || !salts) return;
    std::lock_guard<std::mutex> lk(c->mu);
    for (size_t i = 0; i < n; ++i) {
        const uint64_t x = splitmix_next(c->rng);
        std::memcpy(salts + 8 * i, &x, 8);   // little-endian host
    }
}

int hyobfs_salamander_key(hyobfs_salamander* c, const uint8_t salt[8], uint8_t key[32]) {
    if (!c || !salt || !key) return HYOBFS_ERR_INVALID;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (!g.ok) return HYOBFS_ERR_HIP;
    if (ensure_stage(c, 64) != HYOBFS_OK) return HYOBFS_ERR_NOMEM;
    std::memcpy(c->stage, salt, 8);
    if (hyobfs::launch_keys(c->kp, reinterpret_cast<const uint64_t*>(c->stage_dev),
                            c->stage_dev + c->stage_cap, 1, c->stream) != hipSuccess)
        return HYOBFS_ERR_HIP;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return HYOBFS_ERR_HIP;
    std::memcpy(key, c->stage + c->stage_cap, 32);
    return HYOBFS_OK;
}

int hyobfs_salamander_keys_batch(hyobfs_salamander* c, const uint64_t* salts, uint8_t* keys,
                                 uint64_t n, void* stream) {
    if (!c || (n && (!salts || !keys))) return HYOBFS_ERR_INVALID;
    DeviceGuard g(c->device);
    if (!g.ok) return HYOBFS_ERR_HIP;
    hipStream_t s = static_cast<hipStream_t>(stream);   // NULL = the HIP null stream
    return hyobfs::launch_keys(c->kp, salts, keys, n, s) == hipSuccess ? HYOBFS_OK : HYOBFS_ERR_HIP;
}

size_t hyobfs_salamander_obfuscate(hyobfs_salamander* c, const uint8_t* in, size_t in_len,
                                   const uint8_t salt[8], uint8_t* out, size_t out_len) {
    if (!c || !salt || (!in && in_len)) return 0;
    const size_t W = in_len + HYOBFS_SALT_LEN;
    if (out_len < W || !out) return 0;                         // salamander.go:60-62
    if (in_len > hyobfs::kMaxDatagram) return 0;
    std::lock_guard<std::mutex> lk(c->mu);
    return run_one(c, true, in, in_len, salt, out, W);
}

size_t hyobfs_salamander_obfuscate_auto(hyobfs_salamander* c, const uint8_t* in, size_t in_len,
                                        uint8_t* out, size_t out_len) {
    if (!c || (!in && in_len)) return 0;
    const size_t W = in_len + HYOBFS_SALT_LEN;
    if (out_len < W || !out) return 0;                         // salamander.go:60-62
    if (in_len > hyobfs::kMaxDatagram) return 0;
    std::lock_guard<std::mutex> lk(c->mu);
    uint8_t salt[8];
    const uint64_t x = splitmix_next(c->rng);                   // RandSrc.Read, :65
    std::memcpy(salt, &x, 8);
    return run_one(c, true, in, in_len, salt, out, W);
}

size_t hyobfs_salamander_deobfuscate(hyobfs_salamander* c, const uint8_t* in, size_t in_len,
                                     uint8_t* out, size_t out_len) {
    if (!c || (!in && in_len)) return 0;
    if (in_len <= HYOBFS_SALT_LEN) return 0;                   // salamander.go:75-76
    const size_t W = in_len - HYOBFS_SALT_LEN;
    if (out_len < W || !out) return 0;                         // :76-77
    if (in_len > hyobfs::kMaxDatagram) return 0;
    std::lock_guard<std::mutex> lk(c->mu);
    return run_one(c, false, in, in_len, nullptr, out, W);
}

uint64_t hyobfs_batch_workspace_bytes(const hyobfs_batch* b) {
    if (!b) return 0;
    hyobfs::BatchParams bp{};
    bp.n = b->n;
    bp.in = b->in;
    bp.in_off = b->in_off;
    bp.in_stride = b->in_stride;
    bp.in_len = b->in_len;
    bp.out_cap = b->out_cap;
    bp.out_stride = b->out_stride;
    // the largest need over the kernel choices: independent of the context's
    uint64_t m = 0;
    for (int k : {hyobfs::kKernelAuto, hyobfs::kKernelWave, hyobfs::kKernelFlat}) {
        bp.kernel = k;
        const uint64_t v = hyobfs::batch_workspace_bytes(true, bp);
        m = v > m ? v : m;
    }
    return m;
}

uint64_t hyobfs_batch_workspace_size(uint64_t n) {
    const uint64_t ntiles = (n + hyobfs::kTile - 1) / hyobfs::kTile;
    return (ntiles + 1) * sizeof(uint64_t);
}

int hyobfs_salamander_batch_kernel(hyobfs_salamander* c, const hyobfs_batch* b, int obfuscate) {
    BatchParams bp;
    const int rc = fill_params(c, b, obfuscate != 0, bp);
    return rc != HYOBFS_OK ? rc : hyobfs::batch_kernel(obfuscate != 0, bp);
}

int hyobfs_salamander_obfuscate_batch(hyobfs_salamander* c, const hyobfs_batch* b, void* stream) {
    return run_batch(c, b, stream, true);
}

int hyobfs_salamander_deobfuscate_batch(hyobfs_salamander* c, const hyobfs_batch* b, void* stream) {
    return run_batch(c, b, stream, false);
}

int hyobfs_salamander_obfuscate_batch_sharded(hyobfs_salamander* const* ctxs, const hyobfs_batch* batches,
                                              int nshards) {
    return run_sharded(ctxs, batches, nshards, true);
}

int hyobfs_salamander_deobfuscate_batch_sharded(hyobfs_salamander* const* ctxs, const hyobfs_batch* batches,
                                                int nshards) {
    return run_sharded(ctxs, batches, nshards, false);
}

int hyobfs_shard_bounds(const uint32_t* in_len, uint64_t n, int nshards, uint64_t* bounds) {
    if (nshards <= 0 || !bounds) return HYOBFS_ERR_INVALID;
    bounds[0] = 0;
    if (!in_len) {   // equal counts, the remainder spread over the first shards
        for (int i = 1; i <= nshards; ++i) bounds[i] = n / nshards * i + std::min<uint64_t>(n % nshards, i);
        return HYOBFS_OK;
    }
    uint64_t total = 0;
    for (uint64_t k = 0; k < n; ++k) total += (uint64_t)in_len[k] + 8;
    // shard i starts at the first datagram whose preceding weight reaches total * i / nshards
    uint64_t acc = 0, k = 0;
    for (int i = 1; i < nshards; ++i) {
        const unsigned __int128 target = (unsigned __int128)total * (unsigned)i / (unsigned)nshards;
        while (k < n && acc < target) acc += (uint64_t)in_len[k++] + 8;
        bounds[i] = k;
    }
    bounds[nshards] = n;
    return HYOBFS_OK;
}

// the encode kernel derives keys in registers: no workspace
uint64_t hyobfs_gecko_workspace_size(uint64_t) { return 0; }

int hyobfs_gecko_encode_batch(hyobfs_salamander* c, const hyobfs_gecko_batch* b, void* stream) {
    if (!c || !b) return HYOBFS_ERR_INVALID;
    if (b->n == 0) return HYOBFS_OK;
    if (!b->msg || !b->frames || !b->salts || !b->out || !b->out_off)
        return HYOBFS_ERR_INVALID;
    // an all-zero pad key: a caller that zero-initialised the struct and set no key
    // would get identical, predictable padding in every batch (the reference's pad
    // bytes come from crypto/rand, gecko_frame.go:55)
    bool zero_key = true;
    for (int i = 0; i < 32; ++i) zero_key = zero_key && b->pad_key[i] == 0;
    if (zero_key) return HYOBFS_ERR_INVALID;
    DeviceGuard g(c->device);
    if (!g.ok) return HYOBFS_ERR_HIP;
    const hipError_t e = hyobfs::launch_gecko_encode(c->kp, *b, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? HYOBFS_OK : HYOBFS_ERR_HIP;
}

int hyobfs_gecko_parse_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint64_t n,
                             hyobfs_gecko_parsed* out, void* stream) {
    if (n == 0) return HYOBFS_OK;
    if (!in || !in_off || !in_len || !out) return HYOBFS_ERR_INVALID;
    return hyobfs::launch_gecko_parse(in, in_off, in_len, n, out, static_cast<hipStream_t>(stream)) == hipSuccess
               ? HYOBFS_OK
               : HYOBFS_ERR_HIP;
}

int hyobfs_salamander_obfuscate_host(hyobfs_salamander* c, const hyobfs_batch* b, uint64_t chunk) {
    return run_host(c, b, chunk, true);
}

int hyobfs_salamander_deobfuscate_host(hyobfs_salamander* c, const hyobfs_batch* b, uint64_t chunk) {
    return run_host(c, b, chunk, false);
}

void* hyobfs_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocMapped) != hipSuccess) return nullptr;
    return p;
}

void hyobfs_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int hyobfs_synth_stream(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t start, void* stream) {
    if (!dst || (reinterpret_cast<uintptr_t>(dst) & 15)) return HYOBFS_ERR_INVALID;
    return hyobfs::launch_synth_stream(dst, nbytes, seed, start, static_cast<hipStream_t>(stream)) ==
                   hipSuccess
               ? HYOBFS_OK
               : HYOBFS_ERR_HIP;
}

int hyobfs_synth_u64(uint64_t* dst, uint64_t n, uint64_t seed, uint64_t first, void* stream) {
    if (!dst) return HYOBFS_ERR_INVALID;
    return hyobfs::launch_synth_u64(dst, n, seed, first, static_cast<hipStream_t>(stream)) == hipSuccess
               ? HYOBFS_OK
               : HYOBFS_ERR_HIP;
}

int hyobfs_synth_bimodal_lengths(uint32_t* dst, uint64_t n, uint64_t seed, uint64_t first,
                                 void* stream) {
    if (!dst) return HYOBFS_ERR_INVALID;
    return hyobfs::launch_synth_bimodal(dst, n, seed, first, static_cast<hipStream_t>(stream)) ==
                   hipSuccess
               ? HYOBFS_OK
               : HYOBFS_ERR_HIP;
}

}  // extern "C"
