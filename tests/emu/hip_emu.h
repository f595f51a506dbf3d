// hip_emu.h -- CPU emulation of the HIP subset used by hysteria_amd/csrc.
//
// TEST INFRASTRUCTURE ONLY.  tests/emu/build.sh compiles the unmodified kernel
// and ABI sources with clang for x86-64 against this header (-DHYOBFS_EMULATE),
// into tests/emu/libhyobfs_emu.so, under AddressSanitizer.  That library is
// never shipped or loaded by the product package: it lets the CPU test tier
// run the kernels' logic (indexing, ownership, scans, pipelining) against the
// oracle and catch out-of-bounds accesses before a kernel ever reaches a GPU.
//
// Model: a launch runs its workgroups one after another; a workgroup runs as
// blockDim.x std::threads.  __syncthreads is a barrier of the workgroup,
// wavefront operations (__shfl_*, readfirstlane) exchange values through a
// per-wave slot array between two barriers of the 64 lanes.  __shared__
// variables are function-local statics (one workgroup at a time).  All lanes
// are assumed active at every wavefront operation, which the kernels satisfy
// (they only shuffle in wave-uniform code).  Launches from several host
// threads are serialised.
#pragma once
#include <algorithm>
#include <atomic>
#include <barrier>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <sanitizer/asan_interface.h>

#define __global__
#define __device__
#define __host__
#define __constant__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static

struct dim3 {
    uint32_t x = 1, y = 1, z = 1;
    dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {}
};
struct uint4 {
    uint32_t x, y, z, w;
};
struct uint2 {
    uint32_t x, y;
};
inline uint2 make_uint2(uint32_t a, uint32_t b) { return uint2{a, b}; }
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }

typedef int hipError_t;
typedef void* hipStream_t;
typedef void* hipEvent_t;
enum { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorOutOfMemory = 2, hipErrorNotReady = 600 };
enum { hipHostMallocMapped = 2, hipStreamNonBlocking = 1 };
enum hipDeviceAttribute_t { hipDeviceAttributeMultiprocessorCount = 0 };
struct hipDeviceProp_t {
    char gcnArchName[256];
};

namespace hyemu {
struct Ctx {
    std::unique_ptr<uint8_t[]> dyn;   // the block's dynamic LDS (exactly the launch's shmem bytes: ASan-checked)
    std::barrier<>* block = nullptr;
    std::barrier<>* wave[16] = {};
    uint64_t slots[1024];
};
inline Ctx g_ctx;
inline thread_local dim3 t_thread, t_block;
inline dim3 g_grid, g_blockdim;
inline int env_int(const char* k, int d) {
    const char* v = std::getenv(k);
    return v ? std::atoi(v) : d;
}
inline int g_cus = env_int("HYEMU_CUS", 4), g_per_cu = env_int("HYEMU_PER_CU", 1);

template <class T>
inline T xchg(T v, int src_lane) {
    const int t = (int)t_thread.x, lane = t & 63, w = t >> 6;
    uint64_t bits = 0;
    static_assert(sizeof(T) <= 8, "shuffle of a value wider than 64 bits");
    std::memcpy(&bits, &v, sizeof(T));
    g_ctx.slots[t] = bits;
    g_ctx.wave[w]->arrive_and_wait();
    T out = v;
    if (src_lane >= 0 && src_lane < 64) std::memcpy(&out, &g_ctx.slots[w * 64 + src_lane], sizeof(T));
    g_ctx.wave[w]->arrive_and_wait();
    return out;
}

inline void wave_sync() { g_ctx.wave[(int)t_thread.x >> 6]->arrive_and_wait(); }

inline std::mutex g_launch_mu;   // the state above is global: one launch at a time

template <class F>
inline void launch(dim3 grid, dim3 block, size_t shmem, F&& body) {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    g_grid = grid;
    g_blockdim = block;
    const uint32_t nt = block.x;
    for (uint32_t b = 0; b < grid.x; ++b) {
        g_ctx.dyn.reset(new uint8_t[shmem ? shmem : 1]);
        std::memset(g_ctx.dyn.get(), 0xCD, shmem ? shmem : 1);
        std::barrier<> bar((std::ptrdiff_t)nt);
        std::vector<std::unique_ptr<std::barrier<>>> waves;
        for (uint32_t w = 0; w < (nt + 63) / 64; ++w) {
            waves.emplace_back(new std::barrier<>((std::ptrdiff_t)std::min<uint32_t>(64, nt - 64 * w)));
            g_ctx.wave[w] = waves.back().get();
        }
        g_ctx.block = &bar;
        std::vector<std::thread> th;
        th.reserve(nt);
        for (uint32_t t = 0; t < nt; ++t)
            th.emplace_back([&, t, b] {
                t_thread = dim3(t);
                t_block = dim3(b);
                body();
            });
        for (auto& x : th) x.join();
    }
}
}  // namespace hyemu

#define threadIdx (hyemu::t_thread)
#define blockIdx (hyemu::t_block)
#define gridDim (hyemu::g_grid)
#define blockDim (hyemu::g_blockdim)

inline void hyemu_wave_sync() { hyemu::wave_sync(); }
inline void __syncthreads() { hyemu::g_ctx.block->arrive_and_wait(); }

template <class T>
inline T __shfl_up(T v, unsigned d, int width = 64) {
    (void)width;
    const int lane = (int)(threadIdx.x & 63);
    T r = hyemu::xchg(v, lane - (int)d);
    return lane >= (int)d ? r : v;
}
template <class T>
inline T __shfl_xor(T v, int m, int width = 64) {
    (void)width;
    return hyemu::xchg(v, (int)(threadIdx.x & 63) ^ m);
}
template <class T>
inline T __shfl(T v, int src, int width = 64) {
    (void)width;
    return hyemu::xchg(v, src);
}
inline unsigned long long __ballot(int pred) {
    const int t = (int)threadIdx.x, w = t >> 6;
    const int lanes = (int)std::min<uint32_t>(64, hyemu::g_blockdim.x - 64 * w);
    hyemu::g_ctx.slots[t] = pred != 0;
    hyemu::g_ctx.wave[w]->arrive_and_wait();
    unsigned long long m = 0;
    for (int l = 0; l < lanes; ++l) m |= (unsigned long long)(hyemu::g_ctx.slots[w * 64 + l] & 1) << l;
    hyemu::g_ctx.wave[w]->arrive_and_wait();
    return m;
}
// like the builtin: int in, int out (a caller that widens the result must
// convert it to unsigned first, exactly as on the GPU)
inline int hyemu_readfirstlane(int v) { return hyemu::xchg(v, 0); }
#define __builtin_amdgcn_readfirstlane(x) hyemu_readfirstlane((int)(x))
inline int hyemu_readlane(int v, int l) { return hyemu::xchg(v, l); }
#define __builtin_amdgcn_readlane(x, l) hyemu_readlane((int)(x), (int)(l))
// DPP quad_perm only (dpp_ctrl 0x00-0xFF): lane i of each quad reads lane ctrl[i]
inline int hyemu_mov_dpp(int v, int ctrl) {
    if (ctrl < 0 || ctrl > 0xFF) std::abort();
    const int lane = (int)(threadIdx.x & 63);
    return hyemu::xchg(v, (lane & ~3) | ((ctrl >> (2 * (lane & 3))) & 3));
}
#define __builtin_amdgcn_mov_dpp(v, ctrl, rm, bm, bc) hyemu_mov_dpp((int)(v), (ctrl))
// full row/bank masks and quad_perm (no lane out of bounds): `old` is never taken
#define __builtin_amdgcn_update_dpp(old, v, ctrl, rm, bm, bc) ((void)(old), hyemu_mov_dpp((int)(v), (ctrl)))
inline uint32_t hyemu_alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
}
#define __builtin_amdgcn_alignbit(a, b, c) hyemu_alignbit((a), (b), (c))

inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

template <class T>
inline T min(T a, T b) { return a < b ? a : b; }
template <class T>
inline T max(T a, T b) { return a < b ? b : a; }

inline unsigned long long atomicCAS(unsigned long long* p, unsigned long long cmp, unsigned long long v) {
    __atomic_compare_exchange_n(p, &cmp, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
    return cmp;
}
enum { hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2 };
inline int hipMemcpy(void* d, const void* s, size_t n, int) { std::memcpy(d, s, n); return 0; }
inline int hipMemcpyAsync(void* d, const void* s, size_t n, int, hipStream_t) { std::memcpy(d, s, n); return 0; }
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
    return __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
}
inline unsigned long long atomicMax(unsigned long long* p, unsigned long long v) {
    unsigned long long cur = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (cur < v && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
    return cur;
}

#define hipLaunchKernelGGL(kernel, grid, block, shmem, stream, ...) \
    hyemu::launch(dim3(grid), dim3(block), (size_t)(shmem), [&] { kernel(__VA_ARGS__); })
inline bool hyemu_readable(const void* p) { return !__asan_address_is_poisoned(p); }
inline uint8_t* hyemu_dyn_lds() { return hyemu::g_ctx.dyn.get(); }
// keeps a load whose value the kernel discards (a prefetch) from being optimised away
inline void hyemu_sink(uint32_t v) {
    static volatile uint32_t s;
    s = v;
}

// ---- runtime API subset
inline hipError_t hipGetLastError() { return hipSuccess; }
inline const char* hipGetErrorString(hipError_t) { return "emulated"; }
inline hipError_t hipGetDeviceCount(int* n) { *n = 1; return hipSuccess; }
inline hipError_t hipDeviceGetPCIBusId(char* buf, int len, int dev) {
    if (dev != 0 || len < 13) return hipErrorInvalidValue;
    std::snprintf(buf, (size_t)len, "0000:00:00.0");   // the one emulated device
    return hipSuccess;
}
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
inline hipError_t hipSetDevice(int d) { return d == 0 ? hipSuccess : hipErrorInvalidValue; }
inline hipError_t hipGetDeviceProperties(hipDeviceProp_t* p, int) {
    std::strcpy(p->gcnArchName, "gfx950:emulated");
    return hipSuccess;
}
inline hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) { *v = hyemu::g_cus; return hipSuccess; }
template <class K>
inline hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int* nb, K, int, size_t) {
    *nb = hyemu::g_per_cu;
    return hipSuccess;
}
inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) { *s = (hipStream_t)1; return hipSuccess; }
inline hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
enum { hipEventDisableTiming = 2, hipEventBlockingSync = 1 };
// Events are numbered in creation order (1, 2, ...).  Fault injection for the CPU tier:
// HYEMU_FAIL_EVENTS_FROM=k makes hipEventSynchronize / hipEventQuery fail for every event numbered k or
// later (a coalescing connection's send queue creates events 1-4 and its receive queue
// 5-8 in a fresh process: k = 5 fails exactly the receive side's GPU steps).
namespace hyemu {
inline std::atomic<uintptr_t> g_events{0};
}
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
    *e = (hipEvent_t)(hyemu::g_events.fetch_add(1) + 1);
    return hipSuccess;
}
inline hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }   // launches run synchronously
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
inline hipError_t hipEventSynchronize(hipEvent_t e) {
    static const uintptr_t from = (uintptr_t)hyemu::env_int("HYEMU_FAIL_EVENTS_FROM", 0);
    return from && (uintptr_t)e >= from ? hipErrorInvalidValue : hipSuccess;
}
// launches run synchronously: an event is complete when queried (or failed, as above)
inline hipError_t hipEventQuery(hipEvent_t e) { return hipEventSynchronize(e); }
enum hipMemoryType { hipMemoryTypeUnregistered = 0, hipMemoryTypeHost = 1, hipMemoryTypeDevice = 2 };
struct hipPointerAttribute_t {
    hipMemoryType type;
    int device;
    void* devicePointer;
    void* hostPointer;
    int isManaged;
    unsigned allocationFlags;
};
inline hipError_t hipDeviceSynchronize() { return hipSuccess; }
inline hipError_t hipMalloc(void** p, size_t n) {
    *p = std::malloc(n ? n : 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
inline hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }
// hipHostMalloc'd ranges are "mapped" (device pointer = host pointer), as on the GPU:
// host batches whose arrays all come from hyobfs_host_alloc take the zero-copy path;
// any other pointer is pageable (hipPointerGetAttributes fails)
namespace hyemu {
inline std::mutex& host_mu() { static std::mutex m; return m; }
inline std::vector<std::pair<uintptr_t, size_t>>& host_ranges() { static std::vector<std::pair<uintptr_t, size_t>> v; return v; }
}  // namespace hyemu
inline hipError_t hipHostMalloc(void** p, size_t n, unsigned) {
    const hipError_t e = hipMalloc(p, n);
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lk(hyemu::host_mu());
        hyemu::host_ranges().push_back({reinterpret_cast<uintptr_t>(*p), n ? n : 1});
    }
    return e;
}
inline hipError_t hipHostFree(void* p) {
    {
        std::lock_guard<std::mutex> lk(hyemu::host_mu());
        auto& v = hyemu::host_ranges();
        for (size_t i = 0; i < v.size(); ++i)
            if (v[i].first == reinterpret_cast<uintptr_t>(p)) {
                v.erase(v.begin() + (long)i);
                break;
            }
    }
    return hipFree(p);
}
inline hipError_t hipPointerGetAttributes(hipPointerAttribute_t* a, const void* p) {
    const uintptr_t x = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(hyemu::host_mu());
    for (const auto& r : hyemu::host_ranges())
        if (x >= r.first && x < r.first + r.second) {
            *a = hipPointerAttribute_t{hipMemoryTypeHost, 0, const_cast<void*>(p), const_cast<void*>(p), 0, 0};
            return hipSuccess;
        }
    return hipErrorInvalidValue;
}
inline hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) { *d = h; return hipSuccess; }
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) { std::memset(p, v, n); return hipSuccess; }
// stream-ordered pool allocation (launches run synchronously here)
typedef void* hipMemPool_t;
enum hipMemAllocationType { hipMemAllocationTypePinned = 1 };
enum hipMemLocationType { hipMemLocationTypeDevice = 1 };
enum hipMemPoolAttr { hipMemPoolAttrReleaseThreshold = 4 };
struct hipMemLocation {
    hipMemLocationType type;
    int id;
};
struct hipMemPoolProps {
    hipMemAllocationType allocType;
    int handleTypes;
    hipMemLocation location;
};
inline hipError_t hipMemPoolCreate(hipMemPool_t* p, const hipMemPoolProps*) { *p = (hipMemPool_t)1; return hipSuccess; }
inline hipError_t hipMemPoolSetAttribute(hipMemPool_t, hipMemPoolAttr, void*) { return hipSuccess; }
inline hipError_t hipMemPoolDestroy(hipMemPool_t) { return hipSuccess; }
inline hipError_t hipMallocFromPoolAsync(void** p, size_t n, hipMemPool_t, hipStream_t) { return hipMalloc(p, n); }
inline hipError_t hipFreeAsync(void* p, hipStream_t) { return hipFree(p); }
