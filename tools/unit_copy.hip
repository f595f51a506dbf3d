// unit_copy.hip -- HBM calibration for the shape of a one-shot "unit" kernel:
// a workgroup of NW waves owns one unit of 64 datagrams (1M x 1200 B in,
// 1M x 1208 B out: 76,800 B read, 77,312 B written per unit); wave 0 first
// spends H rounds of dependent 64-bit VALU work (the 64 BLAKE2b keys of the
// unit cost ~2,000 VALU instructions), then a barrier, then every wave copies
// its contiguous 1/NW of the unit (U chunks of 16 B per lane in flight).
// PRE=1: every wave issues its first U loads before the barrier.
// Compared with one-shot 4 KiB regions per wave (region_copy.hip).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr size_t kInUnit = 64 * 1200 / 16, kOutUnit = 64 * 1208 / 16;   // chunks per unit

template <int NW, int U, int PRE>
__global__ __launch_bounds__(64 * NW) void unit_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                     size_t units, int H, unsigned long long* sink) {
    __shared__ unsigned long long s_key[64];
    const size_t unit = blockIdx.x;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // this wave's share: output chunks [o0, o1), input chunks [i0, i1)
    const size_t o0 = kOutUnit * wv / NW, o1 = kOutUnit * (wv + 1) / NW;
    const u32x4* s = src + unit * kInUnit;
    u32x4* d = dst + unit * kOutUnit;
    u32x4 v[U];
    if (PRE) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t c = o0 + u * 64 + lane;
            if (c < o1 && c < kInUnit) v[u] = __builtin_nontemporal_load(s + c);
        }
    }
    if (wv == 0) {   // the "hash": H rounds of dependent 64-bit work per lane
        unsigned long long a = unit * 64 + lane, b = 0x9e3779b97f4a7c15ull;
        for (int r = 0; r < H; ++r) {
            a += b;
            b = (b ^ a) >> 24 | (b ^ a) << 40;
            a += b;
            b = (b ^ a) >> 63 | (b ^ a) << 1;
        }
        s_key[lane] = a ^ b;
    }
    __syncthreads();
    const unsigned long long key = s_key[lane & 63];
    for (size_t c0 = o0; c0 < o1; c0 += 64 * U) {
        if (!PRE || c0 != o0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t c = c0 + u * 64 + lane;
                if (c < o1 && c < kInUnit) v[u] = __builtin_nontemporal_load(s + c);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t c = c0 + u * 64 + lane;
            u32x4 x = v[u];
            x.x ^= (unsigned)key;
            if (c < o1) __builtin_nontemporal_store(x, d + c);
        }
    }
    if (key == 42 && lane == 0) *sink = key;   // keep the hash alive
}

template <class F>
static double timeit(F launch, double bytes) {
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
    return bytes / (ts[ts.size() / 2] * 1e-3) / 1e9;
}

int main() {
    const size_t units = (1u << 20) / 64;
    const size_t in_bytes = units * kInUnit * 16, out_bytes = units * kOutUnit * 16;
    u32x4 *src, *dst;
    unsigned long long* sink;
    CK(hipMalloc(&src, in_bytes + 4096)); CK(hipMalloc(&dst, out_bytes + 4096)); CK(hipMalloc(&sink, 8));
    CK(hipMemset(src, 0x5a, in_bytes)); CK(hipMemset(dst, 0, out_bytes));
    const double bytes = (double)in_bytes + out_bytes;
    printf("{\"in_bytes\": %zu, \"out_bytes\": %zu, \"results\": [\n", in_bytes, out_bytes);
    bool first = true;
    auto row = [&](const char* name, int H, double gbs) {
        printf("%s {\"shape\": \"%s\", \"hash_rounds\": %d, \"GBs\": %.1f}", first ? "" : ",\n", name, H, gbs);
        first = false;
    };
    for (int H : {0, 250, 500}) {
#define RUN(NW, U, PRE)                                                                                 \
    row("waves" #NW "_u" #U "_pre" #PRE, H, timeit([&] {                                               \
            hipLaunchKernelGGL((unit_copy<NW, U, PRE>), dim3((unsigned)units), dim3(64 * NW), 0, 0, src, \
                               dst, units, H, sink);                                                    \
        }, bytes))
        RUN(16, 4, 0);
        RUN(16, 4, 1);
        RUN(16, 6, 1);
        RUN(8, 4, 1);
        RUN(8, 8, 1);
        RUN(4, 8, 1);
#undef RUN
    }
    printf("\n]}\n");
    return 0;
}
