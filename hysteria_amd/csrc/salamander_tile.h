// salamander_tile.h -- the one-shot tile kernel for slotted batches whose region
// edges all fall on 8-byte boundaries (gfx950).
//
// Reference: extras/obfs/salamander.go:59-91 (Obfuscate, Deobfuscate, keyLocked).
//
// A workgroup of four waves owns a TILE of 16 consecutive datagrams and exits
// when it is done.  16 slots of a multiple of 8 bytes are whole 128-byte lines,
// so no output line is shared by two workgroups (which may sit on different XCDs).
//   1. waves 1-3 copy the tile's input range (16 x in_stride bytes at most) into
//      LDS with LDS-DMA (global_load_lds_dwordx4, non-temporal): 1 KiB per
//      instruction, 16-byte aligned and contiguous -- the loads of a plain
//      copy, with nothing held in registers.
//   2. meanwhile wave 0 loads the 16 salts and hashes BLAKE2b-256(PSK || salt)
//      with four lanes per key (one G column each, the diagonal step by DPP
//      quad permutes): about 1k VALU instructions for all 16 keys, into LDS.
//   3. after one barrier, all four waves compose the output: with every region
//      edge on an 8-byte boundary each 8-byte half of a 16-byte output chunk is
//      a salt, 8 payload bytes of one datagram (one 8-byte LDS read XOR one key
//      word) or nothing; one 16-byte non-temporal store per chunk, 1 KiB per
//      wave instruction, whole lines.
// Slots larger than 256 x kTSU x 16 / 16 bytes take several passes of step 3.
// Applies when tile_params() holds; everything else runs the wave kernel.
#pragma once
#include "salamander_wave.h"

namespace hyobfs {

constexpr int kTileMaxD = 16;        // datagrams per tile: one wave hashes 16 keys, 4 lanes each;
                                     // 16 slots of a multiple of 8 bytes are whole 128-byte lines
constexpr uint64_t kMaxTileSlot = 1u << 20;
#ifndef HY_TILE_MIN_WAVES
#define HY_TILE_MIN_WAVES 8
#endif

struct TileParams {
    uint32_t S;      // output slot (out_stride), a multiple of 8
    uint32_t W;      // output width, a multiple of 8, 16 <= W <= S
    uint32_t LI;     // input bytes per datagram (len_uniform)
    float invS;      // 1 / S
    uint64_t t0;     // first tile of this launch (launch_tile_sw splits big batches)
};

#ifndef HY_TILE_SU
#define HY_TILE_SU 5             // staged: output chunks per thread and pass (256 x 5 x 16 B = 20 KiB)
#endif
constexpr int kTSU = HY_TILE_SU;
#ifndef HY_TILE_DMA_AUX
#define HY_TILE_DMA_AUX 2        // cache policy of the staging loads: 2 = nt (streamed once; 4 % faster
                                 // than the default policy, profiles/r03_ab_tile_stage.txt)
#endif

// BLAKE2b sigma, for compile-time placement of message words on the lanes
struct B2Sigma {
    static constexpr uint8_t s[12][16] = {
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
};

// Lane (0..3) of a quad whose G takes message word w in slot SLOT of round R
// (SLOT 0/1: column step x/y, 2/3: diagonal step x/y), or -1.
template <int R, int SLOT>
constexpr int quad_lane_of(int w) {
    for (int i = 0; i < 4; ++i)
        if (B2Sigma::s[R][(SLOT >> 1) * 8 + 2 * i + (SLOT & 1)] == w) return i;
    return -1;
}

// Message word of slot SLOT for this lane: the device block is PSK words
// (uniform) 0..SW-1, word SW = PSK tail | salt << sb, word SW+1 = salt's
// remaining bytes (SW < 15), zeros after; the second block (SW == 15 with
// K.nblk == 2) holds only the salt's tail in word 0 (as msg_word).
template <int R, int SLOT, int SW, int BLK, int WD>
__device__ __forceinline__ void quad_msg_acc(uint64_t& m, const KeyParams& K, uint64_t lo, uint64_t hi,
                                             uint32_t qi) {
    constexpr int kLast = BLK ? 0 : (SW < 15 ? SW + 1 : 15);
    if constexpr (WD <= kLast) {
        constexpr int li = quad_lane_of<R, SLOT>(WD);
        if constexpr (li >= 0) {
            uint64_t val;
            if constexpr (BLK) val = hi;
            else if constexpr (WD < SW) val = K.m[WD];
            else if constexpr (WD == SW) val = K.m[WD] | lo;
            else val = K.m[WD] | hi;
            m = qi == (uint32_t)li ? val : m;
        }
        quad_msg_acc<R, SLOT, SW, BLK, WD + 1>(m, K, lo, hi, qi);
    }
}

template <int R, int SLOT, int SW, int BLK>
__device__ __forceinline__ uint64_t quad_msg(const KeyParams& K, uint64_t lo, uint64_t hi, uint32_t qi) {
    uint64_t m = 0;
    quad_msg_acc<R, SLOT, SW, BLK, 0>(m, K, lo, hi, qi);
    return m;
}

// quad_perm DPP move of a 64-bit value (lane i of each quad reads lane CTRL[i])
template <int CTRL>
__device__ __forceinline__ uint64_t qperm(uint64_t x) {
    return (uint64_t)qperm32<CTRL>((uint32_t)(x >> 32)) << 32 | qperm32<CTRL>((uint32_t)x);
}

#define HY_QG(a, b, c, d, x, y)   \
    do {                          \
        a = a + b + (x);          \
        d = rotr64<32>(d ^ a);    \
        c = c + d;                \
        b = rotr64<24>(b ^ c);    \
        a = a + b + (y);          \
        d = rotr64<16>(d ^ a);    \
        c = c + d;                \
        b = rotr64<63>(b ^ c);    \
    } while (0)

// One BLAKE2b round on a quad: lane i holds v[i], v[4+i], v[8+i], v[12+i].
template <int R, int SW, int BLK>
__device__ __forceinline__ void quad_round(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, const KeyParams& K,
                                           uint64_t lo, uint64_t hi, uint32_t qi) {
#ifndef HYOBFS_EMULATE
    // the per-lane message selects of this round are computed here, not hoisted
    // into registers for all twelve rounds at once (long PSKs: up to 17 words)
    asm volatile("" : "+v"(qi));
#endif
    HY_QG(a, b, c, d, (quad_msg<R, 0, SW, BLK>(K, lo, hi, qi)), (quad_msg<R, 1, SW, BLK>(K, lo, hi, qi)));
    b = qperm<kQRot1>(b);   // diagonals: lane i takes v[4+(i+1)%4], v[8+(i+2)%4], v[12+(i+3)%4]
    c = qperm<kQRot2>(c);
    d = qperm<kQRot3>(d);
    HY_QG(a, b, c, d, (quad_msg<R, 2, SW, BLK>(K, lo, hi, qi)), (quad_msg<R, 3, SW, BLK>(K, lo, hi, qi)));
    b = qperm<kQRot3>(b);   // back to columns
    c = qperm<kQRot2>(c);
    d = qperm<kQRot1>(d);
}

template <int SW, int BLK>
__device__ __forceinline__ void quad_rounds(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, const KeyParams& K,
                                            uint64_t lo, uint64_t hi, uint32_t qi) {
    quad_round<0, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<1, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<2, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<3, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<4, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<5, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<6, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<7, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<8, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<9, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<10, SW, BLK>(a, b, c, d, K, lo, hi, qi);
    quad_round<11, SW, BLK>(a, b, c, d, K, lo, hi, qi);
}

__device__ __forceinline__ uint64_t sel4(uint64_t x0, uint64_t x1, uint64_t x2, uint64_t x3, uint32_t i) {
    return i == 0 ? x0 : i == 1 ? x1 : i == 2 ? x2 : x3;
}

// keyLocked (salamander.go:88-91) on a quad: lane 4k+qi returns key word qi of
// BLAKE2b-256(PSK || salt), salt being the same in the quad's four lanes.
template <int SW>
__device__ __forceinline__ uint64_t quad_key(const KeyParams& K, uint64_t salt, uint32_t qi) {
    const uint32_t sb = (K.salt_pos & 7) * 8;
    const uint64_t lo = salt << sb;
    const uint64_t hi = sb ? (salt >> (64 - sb)) : 0ull;
    const uint64_t h0 = sel4(K.h[0], K.h[1], K.h[2], K.h[3], qi);
    const uint64_t h1 = sel4(K.h[4], K.h[5], K.h[6], K.h[7], qi);
    const uint64_t iv0 = sel4(kIV[0], kIV[1], kIV[2], kIV[3], qi);
    const uint64_t iv1 = sel4(kIV[4], kIV[5], kIV[6], kIV[7], qi);
    uint64_t a = h0, b = h1, c = iv0, d = iv1;
    if (qi == 0) d ^= K.t[0];
    if (qi == 2 && K.nblk == 1) d = ~d;
    quad_rounds<SW, 0>(a, b, c, d, K, lo, hi, qi);
    if constexpr (SW == 15) {
        if (K.nblk == 2) {   // salt_pos 121..127: chain into the salt's second block
            const uint64_t g0 = h0 ^ a ^ c, g1 = h1 ^ b ^ d;
            a = g0;
            b = g1;
            c = iv0;
            d = iv1;
            if (qi == 0) d ^= K.t[1];
            if (qi == 2) d = ~d;
            quad_rounds<SW, 1>(a, b, c, d, K, lo, hi, qi);
            return g0 ^ a ^ c;
        }
    }
    return h0 ^ a ^ c;
}

// Orders LDS writes before other waves' LDS reads without waiting for this
// wave's global loads (a __syncthreads() fence would add vmcnt(0)).
__device__ __forceinline__ void hy_lds_barrier() {
#ifdef HYOBFS_EMULATE
    __syncthreads();
#else
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#endif
}

__device__ __forceinline__ void store8_global(uint8_t* p, uint64_t v) {   // 8-aligned
#ifdef HYOBFS_EMULATE
    std::memcpy(p, &v, 8);
#else
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(1))) v2u gv2u;
    v2u x;
    x.x = (uint32_t)v;
    x.y = (uint32_t)(v >> 32);
    __builtin_nontemporal_store(x, (gv2u*)p);
#endif
}

__device__ __forceinline__ void store16_global(uint8_t* p, uint64_t lo, uint64_t hi) {   // 16-aligned
#ifdef HYOBFS_EMULATE
    std::memcpy(p, &lo, 8);
    std::memcpy(p + 8, &hi, 8);
#else
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) v4u gv4u;
    v4u x;
    x.x = (uint32_t)lo;
    x.y = (uint32_t)(lo >> 32);
    x.z = (uint32_t)hi;
    x.w = (uint32_t)(hi >> 32);
    __builtin_nontemporal_store(x, (gv4u*)p);
#endif
}

// The wire salt the key wave reads while the DMA waves stage the same line
// (deobfuscate): a temporal load, so the line is allocated in L2 and the DMA's request
// for it hits there; a non-temporal load fetched those lines twice from HBM (uniform
// deobfuscate: reads 1.042 x the input against 1.0016 x, 0.4181 against 0.3962 ms per
// launch, profiles/r04_ab_uniform_saltt.txt)
__device__ __forceinline__ uint64_t load8_wire_salt(const uint8_t* p) {   // 8-aligned
#ifdef HYOBFS_EMULATE
    return load8_nt(p);
#else
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    typedef const __attribute__((address_space(1))) v2u gv2u;
    const v2u v = *(gv2u*)(p);
    return (uint64_t)v.y << 32 | v.x;
#endif
}

__device__ __forceinline__ void glds16(const uint8_t* g, uint8_t* l) {   // LDS-DMA: l = wave base + lane * 16
#ifdef HYOBFS_EMULATE
    std::memcpy(l + 16 * (threadIdx.x & 63), g, 16);
#else
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, HY_TILE_DMA_AUX);
#endif
}

// Obfuscate: the key wave's early temporal loads of each datagram's input (two per
// datagram, at payload offsets 0 and ~L/2 rounded down to a line) warm the L2 for the
// staging DMA (78.8 -> 81.7 %).  HY_TILE_PREFETCH = loads per datagram.
#ifndef HY_TILE_PREFETCH
#define HY_TILE_PREFETCH 2
#endif

// One 8-byte half of an output chunk: datagram q, slot offset rr.  Branch-free:
// every lane does one data read and one key read from LDS whatever the half holds
// (salt: data = the salt, key masked off; payload: 8 staged bytes and the key word;
// outside the region: reads of word 0, not stored), so a wave never splits on the
// one salt / datagram-edge chunk per datagram.
template <bool OBF>
__device__ __forceinline__ uint64_t tile_half(const uint8_t* s_in, const uint64_t* s_key, const uint64_t* s_salt,
                                              uint32_t q, uint32_t rr, bool valid, uint32_t in_stride) {
    constexpr uint32_t SALT = OBF ? 8u : 0u, SKIP = OBF ? 0u : 8u;
    const bool salt = OBF && rr < 8u;
    const uint32_t j = rr - SALT;   // payload offset (wraps for the salt; unused then)
    const uint32_t qq = valid ? q : 0u;
    const uint64_t* d = salt ? s_salt + qq
                             : reinterpret_cast<const uint64_t*>(s_in + (valid ? q * in_stride + SKIP + j : 0u));
    const uint64_t k = s_key[qq * 8u + ((j >> 3) & 3u)];
    return *d ^ (salt ? 0ull : k);
}

template <bool OBF, int SW>
__global__ __launch_bounds__(256, HY_TILE_MIN_WAVES) void salamander_tile_kernel(BatchParams B, KeyParams K,
                                                                                  TileParams T) {
#ifdef HYOBFS_EMULATE
    uint8_t* s_in = hyemu_dyn_lds();
#else
    extern __shared__ __attribute__((aligned(16))) uint8_t s_in[];   // the tile's input range
#endif
    __shared__ uint64_t s_key[kTileMaxD * 8];   // each key twice: word w and w + 4 equal
    __shared__ uint64_t s_salt[kTileMaxD];
    constexpr int U = kTSU;

    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = uni32(tid >> 6);
    const uint32_t S = T.S, W = T.W;
    const uint64_t p0 = (T.t0 + blockIdx.x) * kTileMaxD;
    const uint32_t nt = (uint32_t)min<uint64_t>((uint64_t)kTileMaxD, B.n - p0);
    const uint32_t tbytes = (nt - 1) * S + W;   // tile-local end of the last region
    const uint8_t* __restrict__ ib = B.in + p0 * B.in_stride;
    const uint32_t in_stride = (uint32_t)B.in_stride;

    if (wid == 0) {
        // ---- the key wave: salts, BLAKE2b-256 on quads (lane 4k+i: word i of key k), LDS
        const uint32_t qk = lane >> 2, qi = lane & 3;
        uint64_t salt = 0;
        if (qk < nt) salt = OBF ? B.salts[p0 + qk] : load8_wire_salt(ib + qk * in_stride);
#if HY_TILE_PREFETCH
        // offset qi * in_stride / HY_TILE_PREFETCH, down to a line, and never past the
        // datagram's own L bytes (the caller promises only those at the last slot)
        uint32_t pf = 0;
        if (OBF && qk < nt && qi < HY_TILE_PREFETCH) {
            const uint32_t po = min((qi * in_stride / HY_TILE_PREFETCH) & ~127u, (T.LI - 4u) & ~3u);
            pf = *reinterpret_cast<const uint32_t*>(ib + qk * in_stride + po);
        }
#endif
        const uint64_t kw = quad_key<SW>(K, salt, qi);
#if HY_TILE_PREFETCH && !defined(HYOBFS_EMULATE)
        asm volatile("" ::"v"(pf));
#elif HY_TILE_PREFETCH
        hyemu_sink(pf);   // the emulated tier performs the load too: ASan checks its address
#endif
        if (qk < nt) {
            s_key[qk * 8 + qi] = kw;
            s_key[qk * 8 + 4 + qi] = kw;
            if (qi == 0) s_salt[qk] = salt;
        }
        if (lane < nt) {
            if (B.out_off) B.out_off[p0 + lane] = (p0 + lane) * S;
            if (B.out_len) B.out_len[p0 + lane] = W;
        }
        if (B.out_total && lane == 0) atomicAdd(B.out_total, (unsigned long long)nt * W);
    } else {
        // ---- waves 1-3: the tile's input range (16 * in_stride bytes at most, 16-aligned)
        // into LDS, 1 KiB per instruction, nothing held in registers
        const uint32_t in_end = (nt - 1) * in_stride + T.LI;
        const uint32_t nfull = in_end >> 4;
        for (uint32_t i = wid - 1; i * 64u < nfull; i += 3) {
            const uint32_t ch = i * 64u + lane;
            if (ch < nfull) glds16(ib + 16u * ch, s_in + 1024u * i);
        }
        if ((in_end & 15u) && wid == 3 && lane == 0)   // an 8-byte tail (inputs end on 8-byte boundaries)
            *reinterpret_cast<uint64_t*>(s_in + 16u * nfull) = load8_nt(ib + 16u * nfull);
    }
    __syncthreads();   // every wave's LDS-DMA has landed (vmcnt(0)), the keys are published

    // ---- every thread: compose its output chunks from LDS, 1 KiB per wave instruction
    uint8_t* __restrict__ ob = B.out + p0 * S;
    const uint32_t nch = (tbytes + 15u) >> 4;
    for (uint32_t c0 = 0; c0 < nch; c0 += 256u * U) {
        uint64_t lo[U], hi[U];
        uint32_t st[U];   // bit 0 low half written, bit 1 high half written
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + (uint32_t)u * 256u + tid, x = c << 4;
            st[u] = 0;
            lo[u] = hi[u] = 0;
            if (c >= nch) continue;
            uint32_t p = (uint32_t)((float)x * T.invS);
            int32_t r = (int32_t)(x - p * S);
            if (r < 0) {
                --p;
                r += (int32_t)S;
            } else if (r >= (int32_t)S) {
                ++p;
                r -= (int32_t)S;
            }
            uint32_t r2 = (uint32_t)r + 8u, p2 = p;
            if (r2 >= S) {
                r2 -= S;
                ++p2;
            }
            const bool vlo = (uint32_t)r < W, vhi = p2 < nt && r2 < W;
            st[u] = (vlo ? 1u : 0u) | (vhi ? 2u : 0u);
            lo[u] = tile_half<OBF>(s_in, s_key, s_salt, p, (uint32_t)r, vlo, in_stride);
            hi[u] = tile_half<OBF>(s_in, s_key, s_salt, p2, r2, vhi, in_stride);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t x = (c0 + (uint32_t)u * 256u + tid) << 4;
            if (st[u] == 3u)
                store16_global(ob + x, lo[u], hi[u]);
            else if (st[u] == 1u)
                store8_global(ob + x, lo[u]);
            else if (st[u] == 2u)
                store8_global(ob + x + 8, hi[u]);
        }
    }
}

// The tile kernel applies to slotted batches where every datagram has one
// length, the slot, the input stride and the input base are multiples of 8
// (every 8-byte half of an output chunk then belongs to one region: tile_half),
// the input base is 16-aligned and a tile's input fits 64 KiB of LDS, the payload
// is at least 16 bytes and nothing is dropped.
template <bool OBF>
inline bool tile_params(const BatchParams& b, TileParams& T) {
    if (b.out_stride == 0 || b.in_len || b.in_off || b.n == 0) return false;
    if (reinterpret_cast<uintptr_t>(b.out) & 15u) return false;
    const uint64_t L = b.len_uniform;
    if (L > kMaxDatagram || L < (OBF ? 16u : 24u)) return false;
    if ((L | b.out_stride | b.in_stride | reinterpret_cast<uintptr_t>(b.in)) & 7u) return false;
    if (b.in_stride > 0xFFFFFFFFull / kTileMaxD) return false;
    // the staged input range: 16-aligned (LDS-DMA moves 16-byte chunks), at most 64 KiB of LDS
    if ((reinterpret_cast<uintptr_t>(b.in) & 15u) || b.in_stride > 4096 || L > 4096) return false;
    const uint64_t W = OBF ? L + 8 : L - 8, S = b.out_stride;
    if ((b.pkt_cap && W > b.pkt_cap) || W > S) return false;
    if ((b.n - 1) * S + W > b.out_cap) return false;
    if (S > kMaxTileSlot) return false;   // tile-local offsets stay 32-bit, float estimate exact enough
    T.S = (uint32_t)S;
    T.W = (uint32_t)W;
    T.LI = (uint32_t)L;
    T.invS = 1.0f / (float)S;
    T.t0 = 0;
    return true;
}

// Tiles per launch: a big batch goes out as consecutive launches of at most this
// many tiles (HYOBFS_TILE_LAUNCH_TILES overrides; 0 = one launch).  On an 8M x 1200 B
// batch one launch ran at 70.5-72.6 % of 8 TB/s and launches of 1M at 75.4-76.8 %
// (profiles/r03_size_probe.txt): within one long launch the XCDs drift apart in the
// address space, every launch boundary lines them up again.  Launches of 512K
// datagrams measured another ~0.8 % faster (78.2-78.4 %; 256K 77.5-77.7 %, 128K
// 74.5-74.7 %: launch gaps), and 512K is the default.  The 1M-datagram bench batch is
// therefore two launches: per-call figures sum the launches of one call
// (scripts/rocprof_per_call.py, scripts/pmc_traffic.py); a rocprofv3 per-kernel average
// describes half a call.
#ifndef HY_TILE_LAUNCH_TILES
#define HY_TILE_LAUNCH_TILES 32768   // 512K datagrams
#endif
inline uint64_t tile_launch_tiles() {   // read once, thread-safe (a function-local static)
    static const uint64_t v = [] {
        const char* e = std::getenv("HYOBFS_TILE_LAUNCH_TILES");
        const long long x = e ? std::atoll(e) : HY_TILE_LAUNCH_TILES;
        return (uint64_t)(x < 0 ? 0 : x);
    }();
    return v;
}

template <bool OBF, int SW>
void launch_tile_sw(const BatchParams& b, const KeyParams& k, const TileParams& T, hipStream_t s) {
    const uint64_t tiles = div_up(b.n, kTileMaxD);
    const uint64_t per = tile_launch_tiles() ? tile_launch_tiles() : tiles;
    // dynamic LDS: the longest tile input range, 15 strides plus one datagram (in_stride may be
    // smaller than the length, e.g. 0 for one datagram)
    const uint32_t shm = (uint32_t)(((kTileMaxD - 1) * b.in_stride + T.LI + 15) & ~15ull);
    for (uint64_t t0 = 0; t0 < tiles; t0 += per) {
        TileParams Tl = T;
        Tl.t0 = t0;
        const uint64_t blocks = min(per, tiles - t0);
        hipLaunchKernelGGL((salamander_tile_kernel<OBF, SW>), dim3((uint32_t)blocks), dim3(256), shm, s, b, k, Tl);
    }
}

}  // namespace hyobfs
