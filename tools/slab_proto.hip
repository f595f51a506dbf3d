// slab_proto.hip -- experiment: a copy-shaped obfuscate kernel for slotted
// uniform batches.  Keys come from the library's keys kernel; each wave owns
// one aligned output slab (64 lanes x U chunks x 16 B) and exits, so the waves
// in flight sweep the output in address order like the region-copy
// calibration.  Checks its output against the library's batch kernel and
// prints the timings of both.  Not part of the product.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/hyobfs.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)
typedef unsigned __int128 u128;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u128 ld16(const uint8_t* p) { u128 v; __builtin_memcpy(&v, p, 16); return v; }
__device__ __forceinline__ u128 ld16nt(const uint8_t* p) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    u128 r; __builtin_memcpy(&r, &v, 16); return r;
}
__device__ __forceinline__ void st16nt(uint8_t* p, u128 r) {
    v4u v; __builtin_memcpy(&v, &r, 16); __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
}
__device__ __forceinline__ u128 bmask(uint32_t lo, uint32_t hi) {
    const uint32_t nb = hi - lo;
    const u128 m = nb >= 16 ? ~(u128)0 : (((u128)1 << (8 * nb)) - 1);
    return m << (8 * lo);
}

constexpr int kMaxQ = 16;
struct SlabBuf { uint4 key[2 * kMaxQ]; uint64_t salt[kMaxQ]; };

// 256-bit rotate left by 8r bits: byte j of the result is byte (j - r) mod 32
__device__ __forceinline__ void rot_key(const uint64_t k[4], uint32_t r, uint4& lo, uint4& hi) {
    const uint32_t wr = r >> 3, s = (r & 7) * 8;
    uint64_t w[4], o[4];
    for (int i = 0; i < 4; ++i) {
        const uint64_t a0 = k[i], a1 = k[(i + 3) & 3], a2 = k[(i + 2) & 3], a3 = k[(i + 1) & 3];
        w[i] = wr == 0 ? a0 : wr == 1 ? a1 : wr == 2 ? a2 : a3;
    }
    for (int i = 0; i < 4; ++i) o[i] = s ? ((w[i] << s) | (w[(i + 3) & 3] >> (64 - s))) : w[i];
    lo = make_uint4((uint32_t)o[0], (uint32_t)(o[0] >> 32), (uint32_t)o[1], (uint32_t)(o[1] >> 32));
    hi = make_uint4((uint32_t)o[2], (uint32_t)(o[2] >> 32), (uint32_t)o[3], (uint32_t)(o[3] >> 32));
}

template <int U>
__global__ __launch_bounds__(256, 8) void slab_obf(const uint8_t* __restrict__ in, uint32_t L,
                                                   const uint64_t* __restrict__ salts,
                                                   const uint8_t* __restrict__ keys, uint8_t* __restrict__ out,
                                                   uint64_t n) {
    __shared__ SlabBuf sb[4];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    SlabBuf& T = sb[wid];
    const uint64_t stride = L + 8;
    const uint64_t total = n * stride;
    constexpr uint64_t S = 64ull * U * 16;
    const uint64_t s0 = ((uint64_t)blockIdx.x * 4 + wid) * S;
    if (s0 >= total) return;
    const uint64_t s1 = min(total, s0 + S);
    const uint64_t q0 = s0 / stride, q1 = (s1 - 1) / stride;
    const uint32_t cnt = (uint32_t)(q1 - q0 + 1);
    if (lane < (int)cnt) {
        const uint64_t q = q0 + lane;
        uint4 lo, hi;
        uint64_t k4[4];
        __builtin_memcpy(k4, keys + 32 * q, 32);
        rot_key(k4, (uint32_t)((q * stride + 8) & 31), lo, hi);
        T.key[2 * lane] = lo;
        T.key[2 * lane + 1] = hi;
        T.salt[lane] = salts[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    u128 v[U];
    bool fast[U];
    uint32_t qi[U];
    const uint64_t o0 = q0 * stride;
    const uint32_t d0 = (uint32_t)(s0 - o0);   // slab start relative to datagram q0's region
    const float inv = 1.0f / (float)stride;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t a = s0 + (uint64_t)(u * 64 + lane) * 16;
        const uint32_t x = d0 + (uint32_t)(u * 64 + lane) * 16;
        uint32_t r = (uint32_t)((float)x * inv);
        if ((r + 1) * (uint32_t)stride <= x) ++r;
        if (r * (uint32_t)stride > x) --r;
        const uint64_t q = q0 + r;
        const uint64_t o = o0 + (uint64_t)r * stride;
        qi[u] = r;
        fast[u] = a < s1 && o + 8 <= a && a + 16 <= o + stride;
        v[u] = 0;
        if (fast[u]) v[u] = ld16nt(in + q * L + (a - o - 8));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t a = s0 + (uint64_t)(u * 64 + lane) * 16;
        if (fast[u]) {
            const uint4 kk = T.key[2 * qi[u] + ((a >> 4) & 1)];
            u128 k; __builtin_memcpy(&k, &kk, 16);
            st16nt(out + a, v[u] ^ k);
        }
    }
    // boundary chunks of this slab (salt, datagram edges), same wave, right after
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t a = s0 + (uint64_t)(u * 64 + lane) * 16;
        if (fast[u] || a >= s1) continue;
        u128 r = 0;
        const uint64_t qa = q0 + qi[u], qb = min(n - 1, (a + 15) / stride);
        for (uint64_t k = qa; k <= qb; ++k) {
            const uint64_t o = k * stride;
            const uint32_t ki = (uint32_t)(k - q0);
            // salt [o, o+8)
            const uint64_t sb = max(o, a), se = min(o + 8, a + 16);
            if (sb < se) {
                u128 Sv = (u128)T.salt[ki];
                Sv = o >= a ? (Sv << (8 * (o - a))) : (Sv >> (8 * (a - o)));
                r |= Sv & bmask((uint32_t)(sb - a), (uint32_t)(se - a));
            }
            const uint64_t ps = max(o + 8, a), pe = min(o + stride, a + 16);
            if (ps < pe) {
                const int base = (int)((int64_t)a - (int64_t)(o + 8));
                const int ws = min(max(base, 0), (int)L - 16);
                const u128 V = ld16(in + k * L + ws);
                const int d = ws - base;
                const u128 X = d >= 0 ? (V << (8 * d)) : (V >> (8 * -d));
                const uint4 kk = T.key[2 * ki + ((a >> 4) & 1)];
                u128 kx; __builtin_memcpy(&kx, &kk, 16);
                r |= (X ^ kx) & bmask((uint32_t)(ps - a), (uint32_t)(pe - a));
            }
        }
        st16nt(out + a, r);   // uniform slotted: every chunk byte belongs to a region
    }
}

int main(int argc, char** argv) {
    const uint64_t n = 1 << 20;
    const uint32_t L = 1200;
    hyobfs_salamander* ctx = nullptr;
    if (hyobfs_salamander_new((const uint8_t*)"average_password", 16, 0, &ctx) != HYOBFS_OK) return 1;
    uint8_t *in, *out, *ref, *keys;
    uint64_t* salts;
    CK(hipMalloc(&in, n * L + 64)); CK(hipMalloc(&out, n * (L + 8) + 64)); CK(hipMalloc(&ref, n * (L + 8) + 64));
    CK(hipMalloc(&keys, 32 * n)); CK(hipMalloc(&salts, 8 * n));
    hyobfs_synth_stream(in, n * L, 1, 0, nullptr);
    hyobfs_synth_u64(salts, n, 2, 0, nullptr);
    hyobfs_batch b{};
    b.n = n; b.in = in; b.in_stride = L; b.len_uniform = L; b.salts = salts; b.out = ref;
    b.out_cap = n * (L + 8); b.out_stride = L + 8;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto tm = [&](auto f) {
        f(); CK(hipDeviceSynchronize());
        std::vector<float> t;
        for (int r = 0; r < 7; ++r) {
            CK(hipEventRecord(e0)); for (int i = 0; i < 10; ++i) f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms / 10);
        }
        std::sort(t.begin(), t.end()); return t[t.size() / 2];
    };
    const double alg = (double)n * (2 * L + 16);
    const float t_lib = tm([&] { hyobfs_salamander_obfuscate_batch(ctx, &b, nullptr); });
    const float t_keys = tm([&] { hyobfs_salamander_keys_batch(ctx, salts, keys, n, nullptr); });
    const uint64_t total = n * (L + 8);
    auto run = [&](auto kern, uint64_t S) {
        const uint64_t waves = (total + S - 1) / S;
        hipLaunchKernelGGL(kern, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, 0, in, L, salts, keys, out, n);
    };
    const float t_s2 = tm([&] { run(slab_obf<2>, 2048); });
    bool ok2 = true;
    {
        std::vector<uint8_t> a(total), c(total);
        CK(hipMemcpy(a.data(), ref, total, hipMemcpyDeviceToHost)); CK(hipMemcpy(c.data(), out, total, hipMemcpyDeviceToHost));
        ok2 = memcmp(a.data(), c.data(), total) == 0;
    }
    CK(hipMemset(out, 0, total));
    const float t_s4 = tm([&] { run(slab_obf<4>, 4096); });
    const float t_s8 = tm([&] { run(slab_obf<8>, 8192); });
    const float t_s16 = tm([&] { run(slab_obf<16>, 16384); });
    bool ok = true;
    {
        std::vector<uint8_t> a(total), c(total);
        CK(hipMemcpy(a.data(), ref, total, hipMemcpyDeviceToHost)); CK(hipMemcpy(c.data(), out, total, hipMemcpyDeviceToHost));
        ok = memcmp(a.data(), c.data(), total) == 0;
    }
    printf("{\"lib_ms\": %.4f, \"lib_GBs\": %.1f, \"keys_ms\": %.4f, \"slab2k_ms\": %.4f, \"slab4k_ms\": %.4f, \"slab8k_ms\": %.4f, \"slab16k_ms\": %.4f, "
           "\"slab4k_GBs\": %.1f, \"slab8k_GBs\": %.1f, \"slab4k_plus_keys_GBs\": %.1f, \"match2k\": %s, \"match16k\": %s}\n",
           t_lib, alg / t_lib / 1e6, t_keys, t_s2, t_s4, t_s8, t_s16, alg / t_s4 / 1e6, alg / t_s8 / 1e6,
           alg / (t_s4 + t_keys) / 1e6, ok2 ? "true" : "false", ok ? "true" : "false");
    return 0;
}
