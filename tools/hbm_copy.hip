// hbm_copy.hip -- on-box HBM calibration for the roofline denominator.
// Measures a plain 16-byte-per-lane device copy (the "copy kernel" BASELINE.md
// asks to report against) and the same copy with a byte-misaligned source, at
// the byte counts of the 1M x 1200 B obfuscate batch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy16(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst,
                                              size_t nchunks) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < nchunks; base += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t c = base + u * 256;
            if (c < nchunks) {
                if (NT) v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + 16 * c));
                else __builtin_memcpy(&v[u], src + 16 * c, 16);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t c = base + u * 256;
            if (c < nchunks) {
                if (NT) __builtin_nontemporal_store(v[u], reinterpret_cast<u32x4*>(dst + 16 * c));
                else *reinterpret_cast<u32x4*>(dst + 16 * c) = v[u];
            }
        }
    }
}

template <int U, bool NT>
static double run(const unsigned char* src, unsigned char* dst, size_t bytes, int blocks, int iters) {
    const size_t nchunks = bytes / 16;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    hipLaunchKernelGGL((copy16<U, NT>), dim3(blocks), dim3(256), 0, 0, src, dst, nchunks);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < iters; ++i) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((copy16<U, NT>), dim3(blocks), dim3(256), 0, 0, src, dst, nchunks);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return 2.0 * bytes / (ts[ts.size() / 2] * 1e-3) / 1e9;   // read + write, median
}

int main(int argc, char** argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : 1258291200ull;   // 1M x 1200 B
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned char *src, *dst;
    CK(hipMalloc(&src, bytes + 4096)); CK(hipMalloc(&dst, bytes + 4096));
    CK(hipMemset(src, 0x5a, bytes + 4096)); CK(hipMemset(dst, 0, bytes + 4096));
    printf("{\"bytes\": %zu, \"cus\": %d, \"results\": [\n", bytes, cus);
    bool first = true;
    for (int per_cu : {1, 2, 4, 8, 16}) {
        const int blocks = per_cu * cus;
        for (int mis : {0, 8, 3}) {
            double g4 = run<4, false>(src + mis, dst, bytes, blocks, 20);
            double g8 = run<8, false>(src + mis, dst, bytes, blocks, 20);
            double n4 = mis == 0 ? run<4, true>(src, dst, bytes, blocks, 20) : 0.0;
            printf("%s {\"wg_per_cu\": %d, \"src_misalign\": %d, \"u4_GBs\": %.1f, \"u8_GBs\": %.1f, \"u4_nt_GBs\": %.1f}",
                   first ? "" : ",\n", per_cu, mis, g4, g8, n4);
            first = false;
        }
    }
    // grid-sized "one pass" copy: one chunk per lane, no grid-stride loop
    {
        const size_t nch = bytes / 16;
        const int blocks = (int)((nch + 256 * 4 - 1) / (256 * 4));
        double g = run<4, false>(src, dst, bytes, blocks, 20);
        printf(",\n {\"wg_per_cu\": \"one-pass grid %d\", \"src_misalign\": 0, \"u4_GBs\": %.1f}", blocks, g);
    }
    printf("\n]}\n");
    return 0;
}
