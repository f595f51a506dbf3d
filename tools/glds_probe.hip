// glds_probe.hip -- does global_load_lds_dwordx4 return the right bytes from
// device memory and from mapped pinned host memory?  (probe for the staged tile
// kernel, salamander_tile.h HY_TILE_STAGE)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void probe(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst, unsigned n16) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[4096];
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (unsigned i = w; i * 64 < n16; i += 4) {
        const unsigned ch = i * 64 + lane;
        if (ch < n16)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 16 * ch),
                                             (__attribute__((address_space(3))) void*)(lds + 1024 * i), 16, 0, 0);
    }
    __syncthreads();
    for (unsigned b = threadIdx.x; b < 16 * n16; b += blockDim.x) dst[b] = lds[b];
}

// unaligned 16-byte LDS reads (ds_read_b128 at any byte address), as the packed
// tile kernel composes output chunks from staged input at arbitrary byte phases
__global__ void probe_unaligned(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[4096 + 32];
    for (unsigned b = threadIdx.x; b < 4096 + 32; b += blockDim.x) lds[b] = src[b % 4096];
    __syncthreads();
    const unsigned off = (threadIdx.x * 37u) % 4000u;   // every byte phase
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    v4u v;
    __builtin_memcpy(&v, lds + off, 16);
    __builtin_memcpy(dst + 16 * threadIdx.x, &v, 16);
}

int main() {
    const unsigned n16 = 256;   // 4 KiB
    std::vector<unsigned char> ref(16 * n16);
    for (size_t i = 0; i < ref.size(); ++i) ref[i] = (unsigned char)(i * 131 + 7);
    unsigned char *dsrc, *ddst, *hsrc, *hsrc_dev;
    hipMalloc(&dsrc, ref.size());
    hipMalloc(&ddst, ref.size());
    hipMemcpy(dsrc, ref.data(), ref.size(), hipMemcpyHostToDevice);
    hipHostMalloc(&hsrc, ref.size(), hipHostMallocMapped);
    std::memcpy(hsrc, ref.data(), ref.size());
    hipHostGetDevicePointer((void**)&hsrc_dev, hsrc, 0);
    std::vector<unsigned char> got(ref.size());
    for (int pass = 0; pass < 2; ++pass) {
        hipMemset(ddst, 0, ref.size());
        hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, pass ? hsrc_dev : dsrc, ddst, n16);
        hipDeviceSynchronize();
        hipMemcpy(got.data(), ddst, got.size(), hipMemcpyDeviceToHost);
        size_t bad = 0, first = ~0ul;
        for (size_t i = 0; i < got.size(); ++i)
            if (got[i] != ref[i]) {
                ++bad;
                if (first == ~0ul) first = i;
            }
        std::printf("{\"source\": \"%s\", \"bytes\": %zu, \"bad\": %zu, \"first_bad\": %ld}\n",
                    pass ? "mapped pinned host" : "device", got.size(), bad, bad ? (long)first : -1L);
    }
    {
        hipMemset(ddst, 0, ref.size());
        hipLaunchKernelGGL(probe_unaligned, dim3(1), dim3(256), 0, 0, dsrc, ddst);
        hipDeviceSynchronize();
        hipMemcpy(got.data(), ddst, got.size(), hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (unsigned t = 0; t < 256; ++t) {
            const unsigned off = (t * 37u) % 4000u;
            for (unsigned j = 0; j < 16; ++j) bad += got[16 * t + j] != ref[(off + j) % 4096];
        }
        std::printf("{\"source\": \"unaligned ds_read_b128\", \"reads\": 256, \"bad_bytes\": %zu}\n", bad);
    }
    return 0;
}
