// salamander_uniform.h -- the uniform-batch Salamander kernel (gfx950).
//
// For the common batch shape of equal-length datagrams in dense slots: every
// datagram has the same length L (a multiple of 8), the input is the dense
// array in[p * L_in] and the output the dense array out[p * W] (slotted with
// out_stride == W, or packed, which is the same thing when nothing drops).
// The reference work per datagram is unchanged (extras/obfs/salamander.go:
// 59-91): obfuscate writes salt || in ^ key[i % 32], deobfuscate strips the
// salt and XORs back, key = BLAKE2b-256(PSK || salt).
//
// Shape.  Two neighbouring datagrams form a RUN.  Because L is a multiple of
// 8, a run's input (2 L_in bytes) and its output (2 W bytes) are both whole
// 16-byte chunks, so runs never share a chunk or a 128-byte line with another
// run.  In 8-byte words the run is: obfuscate output = salt0, D payload words,
// salt1, D payload words (D = L/8) from input words 0..2D-1; deobfuscate is
// the mirror image.  Every output word is an input word shifted by one or two
// words, so the kernel loads only ALIGNED 16-byte input chunks (one per lane)
// and rebuilds each output chunk from its own chunk and its left neighbour's
// (a DPP wavefront shift; lane 0 takes the left neighbour from the previous
// instruction).  No unaligned loads (round 1's wave kernel read ~10 % more HBM
// lines than the algorithm needs from them), no boundary bookkeeping, no
// partial-line stores.
//
// One wavefront owns 32 runs = 64 datagrams (lane l <-> datagram l for the
// key): wave w owns runs w, w + Wt, w + 2 Wt, ... (Wt = waves in the grid), so
// all waves in flight sweep neighbouring 2.4 KB runs and the chip's in-flight
// address window stays small (tools/region_copy.hip: a one-pass copy in 4 KiB
// regions per wave reaches 6.1 TB/s, in 77 KB regions 5.1 TB/s).  Phases:
//   1. metadata (offsets, widths) and the 64 keys, one BLAKE2b per lane, into
//      LDS with the salts;
//   2. sweep: the wave's runs back to back, 64 consecutive chunks per wave
//      instruction, kUU chunks per lane in flight; per chunk one aligned
//      non-temporal 16-byte load, a shift, two LDS key-word reads, XORs and one
//      aligned non-temporal 16-byte store.
#pragma once
#include "salamander_wave.h"

namespace hyobfs {

#ifndef HY_UNI_U
#define HY_UNI_U 6                   // chunks per lane in flight (8 spills in the hash phase)
#endif
#ifndef HY_UNI_MIN_WAVES
#define HY_UNI_MIN_WAVES 8           // __launch_bounds__ min waves per SIMD
#endif
constexpr int kUU = HY_UNI_U;
constexpr uint32_t kUniRuns = kGroup / 2;   // runs per wave group

struct UniformParams {
    uint32_t D;          // payload words per datagram (L / 8)
    uint32_t CC;         // chunks swept per run (D + 1 in both directions), > 64
    uint32_t pad_;
    uint32_t W;          // output bytes per datagram
    uint64_t LI;         // input bytes per datagram
    uint64_t run_in;     // input bytes per run (2 LI)
    uint64_t run_out;    // output bytes per run (2 W)
    uint64_t nruns;      // complete runs in this launch
    uint64_t nmeta;      // datagrams whose out_off/out_len/out_total this launch reports
};

struct UniGroup {                    // one wave's group in LDS (2.5 KiB)
    uint64_t key[kGroup][4];         // key words of datagram l (= lane l)
    uint64_t salt[kGroup];
};

// Left neighbour of each lane's value; lane 0 gets `first` (wave-uniform).
#ifdef HYOBFS_EMULATE
inline uint32_t wave_prev32(uint32_t x, uint32_t first) {
    const uint32_t r = __shfl_up(x, 1u, 64);
    return (threadIdx.x & 63) ? r : first;
}
inline uint32_t lane63(uint32_t x) { return __shfl(x, 63, 64); }
#else
__device__ __forceinline__ uint32_t wave_prev32(uint32_t x, uint32_t first) {
    // v_mov_b32_dpp wave_shr:1; lane 0 has no source lane and keeps `old`
    return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)x, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t lane63(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
#endif

__device__ __forceinline__ u128 load16a_nt(uint64_t addr) {   // 16-aligned global address
    return load16_nt(reinterpret_cast<const uint8_t*>(addr));
}
// non-temporal 16-byte store to a 16-aligned GLOBAL address (an integer address
// cast to a generic pointer would become a flat store)
__device__ __forceinline__ void store16a_nt(uint64_t addr, uint64_t lo, uint64_t hi) {
#ifdef HYOBFS_EMULATE
    std::memcpy(reinterpret_cast<uint8_t*>(addr), &lo, 8);
    std::memcpy(reinterpret_cast<uint8_t*>(addr) + 8, &hi, 8);
#else
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) v4u gv4u;
    v4u v;
    v.x = (uint32_t)lo;
    v.y = (uint32_t)(lo >> 32);
    v.z = (uint32_t)hi;
    v.w = (uint32_t)(hi >> 32);
    __builtin_nontemporal_store(v, (gv4u*)addr);
#endif
}
// x where !m, y where m (m: all ones or zero), without a branch
__device__ __forceinline__ uint64_t pick(uint64_t x, uint64_t y, bool m) {
    const uint64_t mm = 0ull - (uint64_t)m;
    return (x & ~mm) | (y & mm);
}

template <bool OBF, int SW>
__global__ __launch_bounds__(kGroup* kWavesPerBlock, HY_UNI_MIN_WAVES) void salamander_uniform_kernel(
    BatchParams B, KeyParams K, UniformParams P) {
    constexpr int U = kUU;
    __shared__ UniGroup ug[kWavesPerBlock];

    const int lane = threadIdx.x & 63;
    const uint32_t wid = uni32(threadIdx.x >> 6);
    UniGroup& G = ug[wid];
    const uint64_t Wt = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t w = (uint64_t)blockIdx.x * kWavesPerBlock + wid;
    if (w >= P.nruns) return;   // wave-uniform
    // runs j * Wt + w for j < nv (a prefix of the 32)
    const uint32_t nv = (uint32_t)min<uint64_t>(kUniRuns, (P.nruns - w + Wt - 1) / Wt);
    const uint8_t* __restrict__ in = B.in;
    const uint32_t D = P.D, CC = P.CC;

    // ---- 1. metadata and key of datagram `lane` (run lane/2, datagram lane%2 in it)
    {
        const uint32_t jl = (uint32_t)lane >> 1;
        const bool live = jl < nv;
        const uint64_t p = 2 * ((uint64_t)jl * Wt + w) + (lane & 1);
        uint64_t salt = 0;
        if (live) {
            salt = OBF ? B.salts[p] : load8u(in + p * P.LI);   // the wire's salt
            if (B.out_off) B.out_off[p] = p * P.W;
            if (B.out_len) B.out_len[p] = P.W;
        }
        // an odd datagram after the last run (n odd) is swept by another launch;
        // its metadata is reported here
        const bool tail = w == 0 && lane == 0 && P.nmeta > 2 * P.nruns;
        if (tail) {
            const uint64_t pt = 2 * P.nruns;
            if (B.out_off) B.out_off[pt] = pt * P.W;
            if (B.out_len) B.out_len[pt] = P.W;
        }
        if (B.out_total) {
            const uint64_t wr = uni64(wave_sum((live ? P.W : 0u) + (tail ? P.W : 0u)));
            if (lane == 0 && wr) atomicAdd(B.out_total, (unsigned long long)wr);
        }
        uint64_t key[4];
#ifdef HY_X_NOHASH   // ablation builds only (timing experiments; wrong output)
        key[0] = salt; key[1] = salt * 3; key[2] = salt ^ 7; key[3] = salt + 1;
#else
        wave_key<SW>(K, salt, key);
#endif
#pragma unroll
        for (int i = 0; i < 4; ++i) G.key[lane][i] = key[i];
        G.salt[lane] = salt;
    }
    hy_wave_sync();

    // ---- 2. sweep the wave's runs back to back: lane chunk c = run j, chunk k
    // of the run.  c advances by 64 per wave instruction and a run has CC > 64
    // chunks, so (j, k) and the run's base addresses step incrementally.
    const uint32_t nch = nv * CC;
    const uint64_t din = Wt * P.run_in, dout = Wt * P.run_out;   // one run further
    struct Pos {
        uint32_t c, k, j;
        uint64_t ib, ob;   // this run's input / output base
    };
    Pos s0;
    s0.c = (uint32_t)lane;
    s0.j = 0;
    s0.k = (uint32_t)lane;
    s0.ib = reinterpret_cast<uint64_t>(in) + w * P.run_in;
    s0.ob = reinterpret_cast<uint64_t>(B.out) + w * P.run_out;
    auto advance = [&](Pos& q) {
        q.c += kGroup;
        q.k += kGroup;
        const bool wrap = q.k >= CC;
        q.k = wrap ? q.k - CC : q.k;
        q.j += wrap ? 1u : 0u;
        q.ib += wrap ? din : 0ull;
        q.ob += wrap ? dout : 0ull;
    };
    // the previous instruction's lane-63 chunk: lane 0's left neighbour
    uint32_t cy0 = 0, cy1 = 0, cy2 = 0, cy3 = 0;
    for (uint32_t c0 = 0; c0 < nch; c0 += kGroup * U) {
        u128 v[U];
        Pos q = s0;
#pragma unroll
        for (int u = 0; u < U; ++u) {   // issue every load first
            // obfuscate: lane k holds input chunk k (k < D); deobfuscate: input chunk k (k <= D)
            v[u] = 0;
            if (q.c < nch && (!OBF || q.k < D))
                v[u] = load16a_nt(q.ib + 16ull * q.k);
            advance(q);
        }
        q = s0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t o0 = (uint32_t)v[u], o1 = (uint32_t)(v[u] >> 32);
            const uint32_t o2 = (uint32_t)(v[u] >> 64), o3 = (uint32_t)(v[u] >> 96);
            // left neighbour: chunk k - 1 of the same run whenever it is used
            // (all lanes active here: the shift reads every lane)
            const uint32_t p0 = OBF ? wave_prev32(o0, cy0) : 0u, p1 = OBF ? wave_prev32(o1, cy1) : 0u;
            const uint32_t p2 = wave_prev32(o2, cy2), p3 = wave_prev32(o3, cy3);
            if (OBF) {
                cy0 = lane63(o0);
                cy1 = lane63(o1);
            }
            cy2 = lane63(o2);
            cy3 = lane63(o3);
            const uint64_t own_lo = (uint64_t)o1 << 32 | o0, own_hi = (uint64_t)o3 << 32 | o2;
            const uint64_t prev_lo = (uint64_t)p1 << 32 | p0, prev_hi = (uint64_t)p3 << 32 | p2;
            // r2: key row of the run's first datagram (clamped for lanes past the end)
            const uint32_t k = q.k, r2 = 2 * min(q.j, kUniRuns - 1);
            uint64_t lo, hi, oaddr;
            // selections, not branches: the lanes of one instruction sit at every phase
            if (OBF) {
                // output words e = 2k, 2k+1 of the run: salt0 | payload0 (input
                // words 0..D-1) | salt1 | payload1 (input words D..2D-1)
                const uint32_t e = 2 * k;
                const bool d1l = e > D, d1h = e + 1 > D;   // word in the second datagram
                const uint64_t kl = G.key[r2 + d1l][(d1l ? e - D - 2 : e - 1) & 3];
                const uint64_t kh = G.key[r2 + d1h][(d1h ? e - D - 1 : e) & 3];
                const uint64_t s0w = G.salt[r2], s1w = G.salt[r2 + 1];
                lo = pick(pick(prev_hi, prev_lo, d1l) ^ kl, pick(s0w, s1w, d1l), e == 0 || e == D + 1);
                hi = pick(pick(own_lo, prev_hi, d1h) ^ kh, s1w, e == D);
                oaddr = q.ob + 16ull * k;
            } else {
                // input words of the run: salt0 | payload0 | salt1 | payload1;
                // lane k writes output chunk k - 1, words e = 2k-2, 2k-1
                const uint32_t e = 2 * k - 2;
                const bool d1l = e >= D, d1h = e + 1 >= D;
                const uint64_t kl = G.key[r2 + d1l][(d1l ? e - D : e) & 3];
                const uint64_t kh = G.key[r2 + d1h][(d1h ? e + 1 - D : e + 1) & 3];
                lo = (d1l ? own_lo : prev_hi) ^ kl;
                hi = (d1h ? own_hi : own_lo) ^ kh;
                oaddr = q.ob + 16ull * k - 16;
            }
            if (q.c < nch && (OBF || k != 0))
                store16a_nt(oaddr, lo, hi);
            advance(q);
        }
        s0 = q;
    }
}

// Host-side eligibility and parameters (launch_salamander, salamander.hip).
// The batch must be: uniform length, no in_off/in_len, input and output
// 16-byte aligned and dense (in_stride == input length, out_stride == W or
// packed), every datagram written (no cap drop), L a multiple of 8.
template <bool OBF>
inline bool uniform_params(const BatchParams& b, UniformParams& P) {
    if (b.in_off || b.in_len || b.n < 2) return false;
    const uint64_t LI = b.len_uniform;
    if (LI % 8 || LI > 65536) return false;
    // the sweep steps one run per wrap: a run must have more than 64 chunks
    // (payloads of 512 bytes and more; shorter ones take the wave kernel)
    if ((OBF ? LI : LI - 8) < 512) return false;
    const uint64_t W = OBF ? LI + 8 : LI - 8;
    if (b.in_stride != LI) return false;
    if (b.out_stride && b.out_stride != W) return false;
    if (b.pkt_cap && b.pkt_cap < W) return false;      // would drop every datagram
    if (b.out_cap < b.n * W) return false;            // would drop the tail
    if ((reinterpret_cast<uintptr_t>(b.in) | reinterpret_cast<uintptr_t>(b.out)) & 15) return false;
    P.D = (uint32_t)((OBF ? LI : W) / 8);
    P.CC = P.D + 1;
    P.W = (uint32_t)W;
    P.LI = LI;
    P.run_in = 2 * LI;
    P.run_out = 2 * W;
    P.nruns = b.n / 2;
    P.nmeta = b.n;
    return true;
}

template <bool OBF, int SW>
void launch_uniform_sw(const BatchParams& bp, const KeyParams& k, const UniformParams& P, hipStream_t s) {
    const uint64_t waves = div_up(P.nruns, kUniRuns);
    const uint64_t blocks = div_up(waves, kWavesPerBlock);
    hipLaunchKernelGGL((salamander_uniform_kernel<OBF, SW>), dim3((uint32_t)blocks), dim3(kGroup * kWavesPerBlock),
                       0, s, bp, k, P);
}

}  // namespace hyobfs
