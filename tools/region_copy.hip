// region_copy.hip -- HBM calibration: how the concurrent footprint of a copy
// changes its bandwidth.  Each wave copies one contiguous region of R bytes
// (1 KiB per wave instruction, U in flight per lane), non-persistent grid,
// non-temporal loads and stores -- the access shape of a wave-group kernel
// whose group output is R bytes -- against the grid-stride copy whose
// concurrent footprint is a few MB.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

template <int U>
__global__ __launch_bounds__(256) void region_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                   size_t nchunks, size_t region_chunks) {
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const size_t c0 = w * region_chunks, c1 = std::min(nchunks, c0 + region_chunks);
    for (size_t c = c0; c < c1; c += 64 * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = c + u * 64 + lane;
            if (i < c1) v[u] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = c + u * 64 + lane;
            if (i < c1) __builtin_nontemporal_store(v[u], dst + i);
        }
    }
}

// slab-interleaved: wave w copies slabs w, w + W, ... of S chunks each (W = all waves of the grid)
template <int U>
__global__ __launch_bounds__(256) void slab_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                 size_t nchunks, size_t slab_chunks) {
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t W = (size_t)gridDim.x * 4;
    const int lane = threadIdx.x & 63;
    for (size_t s = w; s * slab_chunks < nchunks; s += W) {
        const size_t c0 = s * slab_chunks, c1 = std::min(nchunks, c0 + slab_chunks);
        for (size_t c = c0; c < c1; c += 64 * U) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t i = c + u * 64 + lane;
                if (i < c1) v[u] = __builtin_nontemporal_load(src + i);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t i = c + u * 64 + lane;
                if (i < c1) __builtin_nontemporal_store(v[u], dst + i);
            }
        }
    }
}

template <class F>
static double timeit(F launch, size_t bytes) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < 15; ++i) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return 2.0 * bytes / (ts[ts.size() / 2] * 1e-3) / 1e9;
}

int main() {
    const size_t bytes = 1266679808ull;   // 1M x 1208 B
    const size_t nch = bytes / 16;
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    u32x4 *src, *dst;
    CK(hipMalloc(&src, bytes + 4096)); CK(hipMalloc(&dst, bytes + 4096));
    CK(hipMemset(src, 0x5a, bytes)); CK(hipMemset(dst, 0, bytes));
    printf("{\"bytes\": %zu, \"results\": [\n", bytes);
    bool first = true;
    for (size_t R : {4096ul, 16384ul, 77312ul, 309248ul, 1236992ul}) {
        const size_t rc = R / 16, waves = (nch + rc - 1) / rc;
        const unsigned blocks = (unsigned)((waves + 3) / 4);
        const double g4 = timeit([&] { hipLaunchKernelGGL(region_copy<4>, dim3(blocks), dim3(256), 0, 0, src, dst, nch, rc); }, bytes);
        const double g8 = timeit([&] { hipLaunchKernelGGL(region_copy<8>, dim3(blocks), dim3(256), 0, 0, src, dst, nch, rc); }, bytes);
        printf("%s {\"kind\": \"region\", \"region_bytes\": %zu, \"u4_GBs\": %.1f, \"u8_GBs\": %.1f}", first ? "" : ",\n", R, g4, g8);
        first = false;
    }
    for (size_t S : {4096ul, 16384ul, 65536ul}) {
        for (int per_cu : {8, 16}) {
            const unsigned blocks = (unsigned)(cus * per_cu);
            const size_t sc = S / 16;
            const double g4 = timeit([&] { hipLaunchKernelGGL(slab_copy<4>, dim3(blocks), dim3(256), 0, 0, src, dst, nch, sc); }, bytes);
            printf(",\n {\"kind\": \"slab\", \"slab_bytes\": %zu, \"wg_per_cu\": %d, \"u4_GBs\": %.1f}", S, per_cu, g4);
        }
    }
    printf("\n]}\n");
    return 0;
}
