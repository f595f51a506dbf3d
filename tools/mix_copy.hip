// mix_copy.hip -- on-box ceiling for a write-heavy stream (the Gecko encode's mix:
// 1.12 GB of wire written, 0.31 GB of message read, the rest of the wire generated).
// Each 16-byte output chunk is either loaded from the source (RD of every 32
// chunks) or generated from its index; every output line is written whole with a
// non-temporal 16-byte store.  Reports algorithmic GB/s (read + written bytes) for
// RD = 0 (write only), 9 (Gecko's mix: reads ~0.28 x writes) and 32 (a copy).
//   hipcc -O3 --offload-arch=gfx950 tools/mix_copy.hip -o tools/mix_copy && tools/mix_copy
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

// one-shot workgroups, each owns a 16 KiB output region in address order; chunks
// whose index mod 32 is below RD come from the source (packed: source offset =
// the number of loaded chunks before it), the others are generated
template <int RD>
__global__ __launch_bounds__(256) void mix16(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst,
                                             size_t nchunks) {
    const size_t c0 = (size_t)blockIdx.x * 1024;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const size_t c = c0 + threadIdx.x + 256 * u;
        const unsigned m = (unsigned)(c & 31);
        if (m < RD) {   // loads issued unconditionally when RD = 32 (a plain copy)
            const size_t s = (c >> 5) * RD + m;
            v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + 16 * s));
        } else {
            v[u] = u32x4{(unsigned)c, (unsigned)(c >> 32), (unsigned)c * 0x9E3779B9u, 0x5bd1e995u};
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const size_t c = c0 + threadIdx.x + 256 * u;
        if (c < nchunks) __builtin_nontemporal_store(v[u], reinterpret_cast<u32x4*>(dst + 16 * c));
    }
}

template <int RD>
static void run(const unsigned char* src, unsigned char* dst, size_t wbytes, int iters) {
    const size_t nchunks = wbytes / 16;
    const int blocks = (int)((nchunks + 1023) / 1024);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    hipLaunchKernelGGL((mix16<RD>), dim3(blocks), dim3(256), 0, 0, src, dst, nchunks);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < iters; ++i) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((mix16<RD>), dim3(blocks), dim3(256), 0, 0, src, dst, nchunks);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[ts.size() / 2];
    const double rbytes = (double)wbytes * RD / 32;
    printf("{\"read_per_32\": %d, \"write_GB\": %.3f, \"read_GB\": %.3f, \"ms\": %.4f, \"GBs\": %.1f, \"frac_of_8TBs\": %.4f}\n",
           RD, wbytes / 1e9, rbytes / 1e9, ms, (wbytes + rbytes) / (ms * 1e-3) / 1e9, (wbytes + rbytes) / (ms * 1e-3) / 8e12);
}

int main(int argc, char** argv) {
    const size_t wbytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 1124518218ull) & ~(size_t)16383;
    unsigned char *src, *dst;
    CK(hipMalloc(&src, wbytes));
    CK(hipMalloc(&dst, wbytes));
    CK(hipMemset(src, 0x5a, wbytes));
    for (int rep = 0; rep < 2; ++rep) {
        run<0>(src, dst, wbytes, 20);
        run<9>(src, dst, wbytes, 20);
        run<32>(src, dst, wbytes, 20);
    }
    CK(hipFree(src));
    CK(hipFree(dst));
    return 0;
}
