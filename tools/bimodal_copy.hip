// bimodal_copy.hip -- the ceiling of BASELINE configs[2]'s access pattern on this box.
//
// configs[2]: 4M datagrams, 40 % 64 B / 60 % 1350 B (SplitMix64 seed 3, as
// hyobfs_synth_bimodal_lengths), CONTIGUOUS input, PACKED output with an 8-byte
// salt in front of every payload.  Each kernel below moves exactly those bytes --
// every input byte read once, every output byte written once, salt bytes written
// as zeros -- with no hash and no XOR, so its rate is what the access pattern
// alone allows (algorithmic bytes = 2 x input + 8 per datagram, as bench.py's
// bimodal roofline minus the 8-byte salt reads).
//
//   wave<DPW>  the wave-group kernel's shape (salamander_wave.h): one wavefront per
//              DPW consecutive datagrams, their output range swept in 16-byte
//              chunks, 6 per lane in flight; the group's two edge chunks are shared
//              with the neighbouring groups and stored byte-masked.
//   flat<R>    a flat grid: one wavefront per R bytes of OUTPUT (R = 1, 2 or 4 KiB),
//              one-shot, the datagrams that reach into its range looked up from a
//              per-range index (first datagram) + their offsets; every output line
//              is written whole by one wave.
//   copy       a plain streaming copy of the same number of bytes (4 KiB per wave).
// A chunk touches at most two datagrams (the shortest output is 72 B): with
// contiguous input the payload byte at output position p of datagram k sits at
// input p - 8 (k + 1), so a chunk is two unaligned 16-byte loads and byte selects.
//
//   hipcc -O3 --offload-arch=gfx950 tools/bimodal_copy.hip -o tools/bimodal_copy && tools/bimodal_copy
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned __int128 u128;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
typedef __attribute__((address_space(1))) u32x4 gu32x4w;

static uint64_t sm64_at(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ u128 ld16(const uint8_t* p) {   // any alignment, non-temporal
    const u32x4 v = __builtin_nontemporal_load((gu32x4*)p);
    u128 r;
    __builtin_memcpy(&r, &v, 16);
    return r;
}
__device__ __forceinline__ void st16(uint8_t* p, u128 v) {   // 16-aligned, non-temporal
    u32x4 x;
    __builtin_memcpy(&x, &v, 16);
    __builtin_nontemporal_store(x, (gu32x4w*)p);
}
__device__ __forceinline__ u128 mask_from(int32_t lo) {   // bytes [max(lo,0), 16)
    return lo <= 0 ? ~(u128)0 : lo >= 16 ? (u128)0 : (~(u128)0) << (8 * lo);
}

// The 16 output bytes at x: datagram d holds x (its region [od, od1)), datagram d+1
// starts at od1.  in0 is the input base (16 guard bytes before it).
__device__ __forceinline__ u128 chunk(const uint8_t* in0, uint64_t x, uint64_t d, uint64_t od, uint64_t od1) {
    const u128 A = ld16(in0 + (int64_t)x - 8 * (int64_t)(d + 1));
    const u128 B = od1 + 8 < x + 16 ? ld16(in0 + (int64_t)x - 8 * (int64_t)(d + 2)) : (u128)0;   // d+1's payload
    const int32_t pa = (int32_t)((int64_t)od + 8 - (int64_t)x);    // first payload byte of d
    const int32_t sb = (int32_t)((int64_t)od1 - (int64_t)x);       // d+1's salt
    const int32_t pb = sb + 8;                                     // d+1's payload
    const u128 mA = mask_from(pa) & ~mask_from(sb), mB = mask_from(pb);
    return (A & mA) | (B & mB);
}

// ---- wave-group shape: wave w owns datagrams [w DPW, (w+1) DPW)
template <int DPW, int U>
__global__ __launch_bounds__(256) void wave_copy(const uint8_t* __restrict__ in0, uint8_t* __restrict__ out,
                                                 const uint64_t* __restrict__ out_off, uint64_t n) {
    __shared__ uint64_t s_o[4][DPW + 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t d0 = ((uint64_t)blockIdx.x * 4 + wid) * DPW;
    if (d0 >= n) return;
    const uint32_t cnt = (uint32_t)std::min<uint64_t>(DPW, n - d0);
    uint64_t* o = s_o[wid];
    if (lane <= (int)cnt) o[lane] = out_off[d0 + lane];   // out_off[n] = total
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t o0 = o[0], o1 = o[cnt];
    const uint64_t c0 = o0 >> 4, c1 = (o1 + 15) >> 4;
    for (uint64_t cb = c0; cb < c1; cb += 64 * U) {
        u128 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c = cb + u * 64 + lane;
            v[u] = 0;
            if (c < c1) {
                const uint64_t x = c << 4;
                uint32_t k = 0;
#pragma unroll
                for (uint32_t s = (DPW >= 64 ? 32 : DPW / 2); s; s >>= 1)
                    if (k + s < cnt && o[k + s] <= x) k += s;
                v[u] = chunk(in0, x, d0 + k, o[k], k + 1 <= cnt ? o[k + 1] : o1);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c = cb + u * 64 + lane;
            if (c >= c1) continue;
            const uint64_t x = c << 4;
            if (x >= o0 && x + 16 <= o1) {
                st16(out + x, v[u]);
            } else {   // shared with the neighbouring group: bytes [o0, o1) only
                for (int j = 0; j < 16; ++j)
                    if (x + j >= o0 && x + j < o1) out[x + j] = (uint8_t)(v[u] >> (8 * j));
            }
        }
    }
}

// ---- flat shape: wave w owns output bytes [w R, (w+1) R); first[w] = the datagram holding byte w R
template <int R>
__global__ __launch_bounds__(256) void flat_copy(const uint8_t* __restrict__ in0, uint8_t* __restrict__ out,
                                                 const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ first,
                                                 uint64_t n, uint64_t total) {
    constexpr int U = R / 1024;   // chunks per lane
    __shared__ uint64_t s_o[4][65];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + wid;
    const uint64_t x0 = w * R;
    if (x0 >= total) return;
    const uint64_t d0 = first[w];
    uint64_t* o = s_o[wid];
    const uint64_t dl = d0 + lane;
    o[lane] = dl <= n ? out_off[dl] : ~0ull;   // at most 57 datagrams start in 4 KiB
    if (lane == 0) o[64] = ~0ull;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    u128 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t x = x0 + 16 * (uint64_t)(u * 64 + lane);
        uint32_t k = 0;
#pragma unroll
        for (uint32_t s = 32; s; s >>= 1)
            if (o[k + s] <= x) k += s;
        v[u] = x < total ? chunk(in0, x, d0 + k, o[k], o[k + 1]) : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t x = x0 + 16 * (uint64_t)(u * 64 + lane);
        if (x < total) st16(out + x, v[u]);   // (the output buffer is padded to 16)
    }
}

// ---- flat shape staged through LDS: workgroup g owns output bytes [g T, (g+1) T).  With
// contiguous input the bytes behind them are one contiguous window, known from the
// tile's first datagram alone: the four waves copy it into LDS by LDS-DMA
// (global_load_lds_dwordx4, non-temporal, 1 KiB per instruction) while they load the
// offsets of the datagrams that reach into the tile; one barrier; every output chunk
// from two 8-byte-aligned LDS windows and byte selects, one 16-byte store each.
__device__ __forceinline__ u128 lds16(const uint8_t* l) {   // 8-aligned LDS
    const uint64_t* q = reinterpret_cast<const uint64_t*>(l);
    return (u128)q[1] << 64 | q[0];
}
template <int T>
__global__ __launch_bounds__(256) void flat_lds_copy(const uint8_t* __restrict__ in0, uint8_t* __restrict__ out,
                                                     const uint64_t* __restrict__ out_off,
                                                     const uint32_t* __restrict__ first, uint64_t n, uint64_t total) {
    constexpr int ND = T / 72 + 3;   // datagrams that can reach into T bytes (72 B the shortest output)
    constexpr int NDP = ND <= 64 ? 64 : ND <= 128 ? 128 : 256;
    extern __shared__ __attribute__((aligned(16))) uint8_t stage[];
    __shared__ uint64_t s_o[NDP + 1];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t x0 = (uint64_t)blockIdx.x * T;
    const uint64_t d0 = first[blockIdx.x];
    // the window: input positions x - 8 (d + 1) for d >= d0 and x in the tile, and the
    // next datagram's (x - 8 (d + 2)); 16-aligned, 16 guard bytes below in0
    const int64_t ws = ((int64_t)x0 - 8 * (int64_t)(d0 + 2)) & ~15ll;
    const int64_t we = (int64_t)x0 + T - 8 * (int64_t)(d0 + 1) + 16;
    const uint32_t nch = (uint32_t)((we - ws + 15) >> 4);
    for (uint32_t i = wid; i * 64u < nch; i += 4) {
        const uint32_t c = i * 64u + lane;
        if (c < nch)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(in0 + ws + 16 * (int64_t)c),
                                             (__attribute__((address_space(3))) void*)(stage + 1024u * i), 16, 0, 2);
    }
    for (int k = tid; k <= NDP; k += 256) s_o[k] = d0 + k <= n ? out_off[d0 + k] : ~0ull;
    __syncthreads();
    constexpr int U = T / 4096;
    u128 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t x = x0 + 16 * (uint64_t)(u * 256 + tid);
        uint32_t k = 0;
#pragma unroll
        for (uint32_t st = NDP / 2; st; st >>= 1)
            if (s_o[k + st] <= x) k += st;
        const uint64_t od = s_o[k], od1 = s_o[k + 1], d = d0 + k;
        const int64_t pa = (int64_t)x - 8 * (int64_t)(d + 1) - ws;
        const u128 A = lds16(stage + pa);
        const u128 B = od1 + 8 < x + 16 ? lds16(stage + pa - 8) : (u128)0;
        const int32_t ia = (int32_t)((int64_t)od + 8 - (int64_t)x), sb = (int32_t)((int64_t)od1 - (int64_t)x);
        v[u] = x < total ? (A & mask_from(ia) & ~mask_from(sb)) | (B & mask_from(sb + 8)) : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t x = x0 + 16 * (uint64_t)(u * 256 + tid);
        if (x < total) st16(out + x, v[u]);
    }
}

// ---- plain copy, 4 KiB per wave
__global__ __launch_bounds__(256) void plain_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  uint64_t nchunks) {
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    u128 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t c = w * 256 + u * 64 + lane;
        v[u] = c < nchunks ? ld16(src + 16 * c) : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t c = w * 256 + u * 64 + lane;
        if (c < nchunks) st16(dst + 16 * c, v[u]);
    }
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 22);
    const int reps = argc > 2 ? atoi(argv[2]) : 10, rounds = argc > 3 ? atoi(argv[3]) : 6;
    std::vector<uint64_t> oo(n + 1);
    uint64_t tin = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t L = (sm64_at(3, i) % 5) < 2 ? 64u : 1350u;
        oo[i] = tin + 8 * i;
        tin += L;
    }
    const uint64_t tout = tin + 8 * n;
    oo[n] = tout;
    // expected output (host): salts zero, payloads = input bytes (input byte b = b * 131 + 7)
    uint8_t *d_in, *d_out;
    uint64_t* d_oo;
    uint32_t* d_first;
    CK(hipMalloc(&d_in, tin + 64));
    CK(hipMalloc(&d_out, tout + 64));
    CK(hipMalloc(&d_oo, 8 * (n + 1)));
    std::vector<uint8_t> hin(tin + 64);
    for (uint64_t b = 0; b < tin + 64; ++b) hin[b] = (uint8_t)((b >= 16 ? b - 16 : 0) * 131 + 7);
    CK(hipMemcpy(d_in, hin.data(), tin + 64, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_oo, oo.data(), 8 * (n + 1), hipMemcpyHostToDevice));
    const uint8_t* in0 = d_in + 16;
    const uint64_t alg = 2 * tin + 8 * n;

    auto mkfirst = [&](uint64_t R) {
        const uint64_t nw = (tout + R - 1) / R;
        std::vector<uint32_t> f(nw);
        uint64_t d = 0;
        for (uint64_t w = 0; w < nw; ++w) {
            while (d + 1 < n && oo[d + 1] <= w * R) ++d;
            f[w] = (uint32_t)d;
        }
        return f;
    };
    uint32_t *f1, *f2, *f4, *f8, *f16;
    auto up = [&](uint64_t R, uint32_t** p) {
        auto f = mkfirst(R);
        CK(hipMalloc(p, 4 * f.size()));
        CK(hipMemcpy(*p, f.data(), 4 * f.size(), hipMemcpyHostToDevice));
    };
    up(1024, &f1);
    up(2048, &f2);
    up(4096, &f4);
    up(8192, &f8);
    up(16384, &f16);
    auto blocks_for = [](uint64_t waves) { return (uint32_t)((waves + 3) / 4); };
    auto run = [&](int which) {
        switch (which) {
        case 0: plain_copy<<<blocks_for((tin / 16 + 255) / 256), 256>>>(in0, d_out, tin / 16); break;
        case 1: wave_copy<32, 6><<<blocks_for((n + 31) / 32), 256>>>(in0, d_out, d_oo, n); break;
        case 2: wave_copy<16, 6><<<blocks_for((n + 15) / 16), 256>>>(in0, d_out, d_oo, n); break;
        case 3: wave_copy<8, 4><<<blocks_for((n + 7) / 8), 256>>>(in0, d_out, d_oo, n); break;
        case 4: flat_copy<1024><<<blocks_for((tout + 1023) / 1024), 256>>>(in0, d_out, d_oo, f1, n, tout); break;
        case 5: flat_copy<2048><<<blocks_for((tout + 2047) / 2048), 256>>>(in0, d_out, d_oo, f2, n, tout); break;
        case 6: flat_copy<4096><<<blocks_for((tout + 4095) / 4096), 256>>>(in0, d_out, d_oo, f4, n, tout); break;
        case 7: flat_lds_copy<8192><<<(uint32_t)((tout + 8191) / 8192), 256, 8192 + 64>>>(in0, d_out, d_oo, f8, n, tout); break;
        case 8: flat_lds_copy<16384><<<(uint32_t)((tout + 16383) / 16384), 256, 16384 + 64>>>(in0, d_out, d_oo, f16, n, tout); break;
        }
    };
    const char* names[] = {"copy (same bytes, 4 KiB/wave)", "wave<32> (wave kernel shape)", "wave<16>", "wave<8>",
                           "flat<1 KiB/wave>", "flat<2 KiB/wave>", "flat<4 KiB/wave>",
                           "flat_lds<8 KiB/workgroup>", "flat_lds<16 KiB/workgroup>"};
    const int NV = 9;
    // correctness of every shaped variant against the host
    std::vector<uint8_t> hout(tout);
    for (int v = 1; v < NV; ++v) {
        CK(hipMemset(d_out, 0xA5, tout + 64));
        run(v);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hout.data(), d_out, tout, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < n && bad < 5; ++i) {
            const uint64_t L = oo[i + 1] - oo[i] - 8, s = oo[i] - 8 * i;
            for (int j = 0; j < 8; ++j) bad += hout[oo[i] + j] != 0;
            for (uint64_t b = 0; b < L; ++b) bad += hout[oo[i] + 8 + b] != hin[16 + s + b];
        }
        if (bad) {
            fprintf(stderr, "%s: output differs\n", names[v]);
            return 1;
        }
    }
    std::vector<std::vector<float>> t(NV);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r <= rounds; ++r)
        for (int v = 0; v < NV; ++v) {
            run(v);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int k = 0; k < reps; ++k) run(v);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) t[v].push_back(ms / reps);
        }
    printf("{\"n\": %llu, \"input_bytes\": %llu, \"output_bytes\": %llu, \"algorithmic_bytes\": %llu, \"results\": [\n",
           (unsigned long long)n, (unsigned long long)tin, (unsigned long long)tout, (unsigned long long)alg);
    for (int v = 0; v < NV; ++v) {
        std::sort(t[v].begin(), t[v].end());
        const double med = t[v][t[v].size() / 2];
        const double bytes = v == 0 ? 2.0 * (double)tin : (double)alg;
        printf(" {\"kernel\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f, \"frac_of_8TBs\": %.4f}%s\n", names[v], med,
               bytes / med / 1e6, bytes / med / 1e6 / 8000.0, v + 1 < NV ? "," : "");
    }
    printf("]}\n");
    return 0;
}
