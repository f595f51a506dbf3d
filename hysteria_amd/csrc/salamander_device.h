// salamander_device.h -- device code of the Salamander kernels (templates).
// Included by salamander.hip (non-template kernels, dispatch) and by
// salamander_inst.hip, which instantiates the main kernel for one salt word
// (-DHY_SW=n) per translation unit so the 64 instantiations build in parallel.
#pragma once
#include <algorithm>

#include "kernels.h"

namespace hyobfs {

inline uint64_t div_up(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// ------------------------------------------------------------------ BLAKE2b
// RFC 7693; golang.org/x/crypto@v0.54.0 blake2b.Sum256 is the reference's
// implementation (extras/go.mod:18).
__device__ constexpr uint64_t kIV[8] = {
    0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
    0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
    0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

__device__ constexpr uint8_t kSigma[12][16] = {
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

// 64-bit rotate right on the 32-bit VALU: two v_alignbit_b32 for 24, 16 and
// 63, a register swap for 32.
template <int N>
__device__ __forceinline__ uint64_t rotr64(uint64_t x) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    uint32_t rl, rh;
    if (N == 32) {
        rl = hi;
        rh = lo;
    } else if (N < 32) {
        rl = __builtin_amdgcn_alignbit(hi, lo, N);
        rh = __builtin_amdgcn_alignbit(lo, hi, N);
    } else {
        rl = __builtin_amdgcn_alignbit(lo, hi, N - 32);
        rh = __builtin_amdgcn_alignbit(hi, lo, N - 32);
    }
    return ((uint64_t)rh << 32) | rl;
}

#define HY_G(v, a, b, c, d, x, y)              \
    do {                                       \
        v[a] = v[a] + v[b] + (x);              \
        v[d] = rotr64<32>(v[d] ^ v[a]);        \
        v[c] = v[c] + v[d];                    \
        v[b] = rotr64<24>(v[b] ^ v[c]);        \
        v[a] = v[a] + v[b] + (y);              \
        v[d] = rotr64<16>(v[d] ^ v[a]);        \
        v[c] = v[c] + v[d];                    \
        v[b] = rotr64<63>(v[b] ^ v[c]);        \
    } while (0)

// RFC 7693 section 3.2 F(h, m, t, f), fully unrolled (used by keys_kernel).
__device__ __forceinline__ void b2b_compress(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                             bool last) {
    uint64_t v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = h[i];
        v[i + 8] = kIV[i];
    }
    v[12] ^= t;
    v[14] = last ? ~v[14] : v[14];
#pragma unroll
    for (int r = 0; r < 12; ++r) {
        HY_G(v, 0, 4, 8, 12, m[kSigma[r][0]], m[kSigma[r][1]]);
        HY_G(v, 1, 5, 9, 13, m[kSigma[r][2]], m[kSigma[r][3]]);
        HY_G(v, 2, 6, 10, 14, m[kSigma[r][4]], m[kSigma[r][5]]);
        HY_G(v, 3, 7, 11, 15, m[kSigma[r][6]], m[kSigma[r][7]]);
        HY_G(v, 0, 5, 10, 15, m[kSigma[r][8]], m[kSigma[r][9]]);
        HY_G(v, 1, 6, 11, 12, m[kSigma[r][10]], m[kSigma[r][11]]);
        HY_G(v, 2, 7, 8, 13, m[kSigma[r][12]], m[kSigma[r][13]]);
        HY_G(v, 3, 4, 9, 14, m[kSigma[r][14]], m[kSigma[r][15]]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

// keyLocked (salamander.go:88-91): BLAKE2b-256(PSK || salt) from the host's
// PSK-only prefix state.  Returns the 4 little-endian key words.
__device__ __forceinline__ void salamander_key(const KeyParams& K, uint64_t salt, uint64_t key[4]) {
    const uint32_t sw = K.salt_pos >> 3;
    const uint32_t sb = (K.salt_pos & 7) * 8;
    const uint64_t lo = salt << sb;
    const uint64_t hi = sb ? (salt >> (64 - sb)) : 0ull;
    uint64_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = K.h[i];
    for (uint32_t b = 0; b < K.nblk; ++b) {
        uint64_t m[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t idx = 16 * b + j;
            uint64_t w = K.m[idx];
            w |= (idx == sw) ? lo : 0ull;
            w |= (idx == sw + 1) ? hi : 0ull;
            m[j] = w;
        }
        b2b_compress(h, m, K.t[b], b + 1 == K.nblk);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) key[i] = h[i];
}

// ---- the same hash, one round per call, for the pipelined main kernel.
// SW = message word holding salt[0] (K.salt_pos / 8, a template parameter so
// that only the one or two salt words are per-lane registers; the PSK words
// stay uniform).  SW == 15 also covers the two-block case (salt_pos 121..127:
// the salt's tail is word 0 of a second, otherwise empty block).
template <int SW>
struct HashState {
    uint64_t v[16];
    uint64_t lo, hi;                 // salt shifted into words SW and SW+1
    uint64_t h[SW == 15 ? 4 : 1];    // per-lane chaining value (two-block case)
};

template <int SW, int BLK>
__device__ __forceinline__ uint64_t msg_word(const KeyParams& K, uint64_t lo, uint64_t hi, int idx) {
    if (BLK == 0) {
        if (idx == SW) return K.m[idx] | lo;
        if (SW < 15 && idx == SW + 1) return K.m[idx] | hi;
        return K.m[idx];
    }
    return idx == 0 ? hi : 0ull;   // second block: only the salt's tail
}

template <int R, int SW, int BLK>
__device__ __forceinline__ void b2b_round(HashState<SW>& S, const KeyParams& K) {
    uint64_t* v = S.v;
#define HY_M(k) msg_word<SW, BLK>(K, S.lo, S.hi, kSigma[R][k])
    HY_G(v, 0, 4, 8, 12, HY_M(0), HY_M(1));
    HY_G(v, 1, 5, 9, 13, HY_M(2), HY_M(3));
    HY_G(v, 2, 6, 10, 14, HY_M(4), HY_M(5));
    HY_G(v, 3, 7, 11, 15, HY_M(6), HY_M(7));
    HY_G(v, 0, 5, 10, 15, HY_M(8), HY_M(9));
    HY_G(v, 1, 6, 11, 12, HY_M(10), HY_M(11));
    HY_G(v, 2, 7, 8, 13, HY_M(12), HY_M(13));
    HY_G(v, 3, 4, 9, 14, HY_M(14), HY_M(15));
#undef HY_M
}

template <int SW, int BLK>
__device__ __forceinline__ void b2b_round_rt(HashState<SW>& S, const KeyParams& K, uint32_t r) {
    switch (r) {   // r is wave-uniform: a scalar jump
        case 0: b2b_round<0, SW, BLK>(S, K); break;
        case 1: b2b_round<1, SW, BLK>(S, K); break;
        case 2: b2b_round<2, SW, BLK>(S, K); break;
        case 3: b2b_round<3, SW, BLK>(S, K); break;
        case 4: b2b_round<4, SW, BLK>(S, K); break;
        case 5: b2b_round<5, SW, BLK>(S, K); break;
        case 6: b2b_round<6, SW, BLK>(S, K); break;
        case 7: b2b_round<7, SW, BLK>(S, K); break;
        case 8: b2b_round<8, SW, BLK>(S, K); break;
        case 9: b2b_round<9, SW, BLK>(S, K); break;
        case 10: b2b_round<10, SW, BLK>(S, K); break;
        default: b2b_round<11, SW, BLK>(S, K); break;
    }
}

template <int SW>
__device__ __forceinline__ void hash_begin(HashState<SW>& S, const KeyParams& K, uint64_t salt) {
    const uint32_t sb = (K.salt_pos & 7) * 8;
    S.lo = salt << sb;
    S.hi = sb ? (salt >> (64 - sb)) : 0ull;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        S.v[i] = K.h[i];
        S.v[i + 8] = kIV[i];
    }
    S.v[12] ^= K.t[0];
    S.v[14] = (K.nblk == 1) ? ~S.v[14] : S.v[14];
    if (SW == 15) {
#pragma unroll
        for (int i = 0; i < 4; ++i) S.h[i] = K.h[i];
    }
}

// One step = one round; 12 * K.nblk steps per key.
template <int SW>
__device__ __forceinline__ void hash_step(HashState<SW>& S, const KeyParams& K, uint32_t step) {
    if (SW == 15 && step >= 12) {
        b2b_round_rt<SW, 1>(S, K, step - 12);
        return;
    }
    b2b_round_rt<SW, 0>(S, K, step);
    if (SW == 15 && step == 11 && K.nblk == 2) {   // chain into the second block
        uint64_t h1[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) h1[i] = (i < 4 ? S.h[i] : K.h[i]) ^ S.v[i] ^ S.v[i + 8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            S.v[i] = h1[i];
            S.v[i + 8] = kIV[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) S.h[i] = h1[i];
        S.v[12] ^= K.t[1];
        S.v[14] = ~S.v[14];
    }
}

template <int SW>
__device__ __forceinline__ void hash_key(const HashState<SW>& S, const KeyParams& K, uint64_t key[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) key[i] = (SW == 15 ? S.h[i] : K.h[i]) ^ S.v[i] ^ S.v[i + 8];
}

// 256-bit rotate left by 8*r bits (r = 0..31): byte j of the result is byte
// (j - r) mod 32 of the key, so the result indexed by an output address
// modulo 32 gives the key byte of that address.
__device__ __forceinline__ void rotl_key_bytes(const uint64_t k[4], uint32_t r, uint64_t o[4]) {
    const uint32_t wr = r >> 3;
    const uint32_t s = (r & 7) * 8;
    uint64_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t a0 = k[i], a1 = k[(i + 3) & 3], a2 = k[(i + 2) & 3], a3 = k[(i + 1) & 3];
        w[i] = wr == 0 ? a0 : wr == 1 ? a1 : wr == 2 ? a2 : a3;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        o[i] = s ? ((w[i] << s) | (w[(i + 3) & 3] >> (64 - s))) : w[i];
}

// ------------------------------------------------------------------ helpers
typedef unsigned __int128 u128;

__device__ __forceinline__ u128 load16u(const uint8_t* p) {   // any alignment
    u128 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ uint64_t load8u(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
__device__ __forceinline__ u128 bytemask(uint32_t lo, uint32_t hi) {  // bytes [lo, hi), hi <= 16
    const uint32_t nb = hi - lo;
    const u128 ones = ~(u128)0;
    const u128 m = nb >= 16 ? ones : (((u128)1 << (8 * nb)) - 1);
    return m << (8 * lo);
}

template <bool OBF>
__device__ __forceinline__ uint32_t out_width(uint32_t L, uint32_t cap) {
    if (L > kMaxDatagram) return 0;
    if (OBF) {
        const uint32_t W = L + 8;                       // salamander.go:60
        return (cap == 0 || W <= cap) ? W : 0u;          // :61-62
    } else {
        if (L <= 8) return 0;                           // :75-76, outLen <= 0
        const uint32_t W = L - 8;
        return (cap == 0 || W <= cap) ? W : 0u;          // :76-77
    }
}

__device__ __forceinline__ uint32_t pkt_len(const BatchParams& B, uint64_t p) {
    return B.in_len ? B.in_len[p] : B.len_uniform;
}
__device__ __forceinline__ uint64_t pkt_in_off(const BatchParams& B, uint64_t p) {
    return B.in_off ? B.in_off[p] : p * B.in_stride;
}

// wavefront-inclusive scan (64 lanes)
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x = max(x, (uint32_t)__shfl_xor(x, d, 64));
    return x;
}

// --------------------------------------------------------------- main kernel
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef HY_PERSIST_PARK
#define HY_PERSIST_PARK 0   // A/B: 1 = complete boundary chunks parked in LDS, stored by the sweep
#endif

struct TileBuf {                 // one sub-tile of <= kTile datagrams, in LDS
    uint32_t o[kTile];           // output region start, relative to base
    uint32_t w[kTile];           // output region width, 0 = dropped
    uint32_t pe[kTile];          // max region end over earlier datagrams of the sub-tile
    uint32_t pad_[kTile];
    uint64_t io[kTile];          // input payload start (absolute byte offset)
    uint64_t salt[kTile];        // salt (obfuscate)
    uint4 key[2 * kTile];        // key rotated to the output's 32-byte phase, 2 halves
    uint64_t base;               // absolute output offset of relative 0 (16-aligned)
    uint32_t nchunks;            // 16-byte chunks from base to the last region end
    uint32_t cnt;                // datagrams in the sub-tile
};

#ifdef HY_BOUNDS_CHECK
// Debug builds: record the first out-of-range global access (and skip it).
__device__ __forceinline__ bool hy_ok(const BatchParams& B, int kind, bool in_range, uint64_t v0,
                                      uint64_t v1, uint64_t v2, uint64_t v3) {
    if (in_range || !B.dbg) return in_range;
    if (atomicCAS(&B.dbg[0], 0ull, (unsigned long long)kind) == 0ull) {
        B.dbg[1] = blockIdx.x;
        B.dbg[2] = threadIdx.x;
        B.dbg[3] = v0;
        B.dbg[4] = v1;
        B.dbg[5] = v2;
        B.dbg[6] = v3;
    }
    return false;
}
#define HY_OK(kind, cond, a, b, c, d) hy_ok(B, kind, (cond), (a), (b), (c), (d))
#else
#define HY_OK(kind, cond, a, b, c, d) true
#endif

// All bytes one datagram k contributes to the 16-byte chunk at relative a.
template <bool OBF>
__device__ __forceinline__ void chunk_contrib(const BatchParams& B, const TileBuf& T,
                                              const uint8_t* __restrict__ in, uint32_t k, uint32_t a, u128& r,
                                              uint32_t& cov) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;
    const uint32_t oq = T.o[k], wq = T.w[k];
    if (wq == 0 || oq + wq <= a || oq >= a + 16) return;
    if (OBF) {   // salt bytes [oq, oq + 8)
        const uint32_t sb = max(oq, a), se = min(oq + 8u, a + 16u);
        if (sb < se) {
            u128 S = (u128)T.salt[k];
            S = oq >= a ? (S << (8 * (oq - a))) : (S >> (8 * (a - oq)));
            r |= S & bytemask(sb - a, se - a);
            cov |= ((1u << (se - sb)) - 1u) << (sb - a);
        }
    }
    const uint32_t op = oq + SALT, pend = oq + wq;
    const uint32_t ps = max(op, a), pe = min(pend, a + 16u);
    if (ps < pe) {
        const uint32_t PL = wq - SALT;
        const int base = (int)a - (int)op;   // payload index of chunk byte 0
        const uint8_t* src = in + T.io[k];
        u128 X = 0;
        if (PL >= 16) {   // one 16-byte window inside the payload, shifted into place
            const int ws = min(max(base, 0), (int)PL - 16);
            if (!HY_OK(4, T.io[k] + ws + 16 <= B.dbg_in_bytes, T.io[k], ws, PL, k)) return;
            const u128 V = load16u(src + ws);
            const int d = ws - base;
            X = d >= 0 ? (V << (8 * d)) : (V >> (8 * -d));
        } else {
            for (uint32_t j = ps - a; j < pe - a; ++j) X |= (u128)src[base + (int)j] << (8 * j);
        }
        const uint4 kk = T.key[2 * k + ((a >> 4) & 1)];
        u128 k128;
        __builtin_memcpy(&k128, &kk, 16);
        r |= (X ^ k128) & bytemask(ps - a, pe - a);
        cov |= ((1u << (pe - ps)) - 1u) << (ps - a);
    }
}

// Streamed input: read exactly once.  HY_NT_LOADS=1 marks it non-temporal
// (the hardware handles the byte misalignment either way).
#ifndef HY_NT_LOADS
#define HY_NT_LOADS 0
#endif
__device__ __forceinline__ u128 load16_stream(const uint8_t* p) {
#if HY_NT_LOADS
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    u128 r;
    __builtin_memcpy(&r, &v, 16);
    return r;
#else
    return load16u(p);
#endif
}

#ifndef HY_NT_STORES
#define HY_NT_STORES 1
#endif
__device__ __forceinline__ void store16_stream(uint8_t* dst, u128 r) {   // dst 16-aligned
    u32x4 v;
    __builtin_memcpy(&v, &r, 16);
#if HY_NT_STORES
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
#else
    *reinterpret_cast<u32x4*>(dst) = v;
#endif
}

__device__ __forceinline__ void store_masked(uint8_t* dst, u128 r, uint32_t cov) {
    if (cov == 0xFFFFu) {
        __builtin_memcpy(dst, &r, 16);
        return;
    }
#pragma unroll
    for (int dw = 0; dw < 4; ++dw) {
        const uint32_t m4 = (cov >> (4 * dw)) & 0xFu;
        const uint32_t word = (uint32_t)(r >> (32 * dw));
        if (m4 == 0xFu) {
            *reinterpret_cast<uint32_t*>(dst + 4 * dw) = word;
        } else if (m4) {
            for (int b = 0; b < 4; ++b)
                if (m4 & (1u << b)) dst[4 * dw + b] = (uint8_t)(word >> (8 * b));
        }
    }
}

#ifndef HY_KU
#define HY_KU 4
#endif
constexpr int kU = HY_KU;   // chunks per lane per sweep iteration



// Values that are equal in every lane (read from LDS, reduced) made scalar, so
// loop bounds and base pointers live in SGPRs and loops stay wave-uniform.
// (the builtin returns int: convert each half to uint32_t before widening)
__device__ __forceinline__ uint32_t uni32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    return ((uint64_t)hi << 32) | lo;
}

struct SweepRegs {      // one sweep iteration's loads in flight
    u128 v[kU];
    uint32_t q[kU];
    bool fast[kU];
};

// Persistent kernel: workgroup g owns datagrams [g*n/G, (g+1)*n/G) (equal
// work for equal lengths; every workgroup is resident, so they finish
// together).  It walks them in sub-tiles of kTile datagrams:
//   sweep(s)    -- 16-byte chunks of sub-tile s that lie inside one payload:
//                  one unaligned 16 B load, one LDS key read, XOR, one
//                  non-temporal store; iteration i+1's loads are issued
//                  before iteration i's stores
//   boundary(s) -- lane t finishes the chunks datagram t owns that are not
//                  inside one payload (salt, datagram edges, sub-tile edges)
//   prep(s+1)   -- widths, offsets (scan), salts of the next sub-tile; its 12
//                  (or 24) BLAKE2b rounds run one per sweep iteration
#ifdef HY_MIN_WAVES_PER_EU   // occupancy experiments: force a register budget
#define HY_MAIN_BOUNDS __launch_bounds__(kTile, HY_MIN_WAVES_PER_EU)
#else
#define HY_MAIN_BOUNDS __launch_bounds__(kTile)
#endif
template <bool OBF, bool PACKED, int SW>
__global__ HY_MAIN_BOUNDS void salamander_kernel(BatchParams B, KeyParams K) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;   // salt bytes in front of the output payload
    constexpr uint32_t SKIP = OBF ? 0u : 8u;   // salt bytes in front of the input payload
    constexpr int U = kU;

    __shared__ TileBuf buf[2];
#if HY_PERSIST_PARK
    // packed layout: complete boundary chunks parked here by their owner (up to 3
    // per datagram: first, second, last chunk), stored by the sweep lane that
    // covers them, so their lines leave in the sweep's own store instructions
    __shared__ uint4 s_park[3 * kTile];
    __shared__ uint32_t s_parkm[kTile];   // bit i: candidate i of datagram t is parked
#endif
    __shared__ uint64_t s_sum[kTile / 64];
    __shared__ uint32_t s_max[kTile / 64];

    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint64_t g = blockIdx.x;
    // Work order.  Contiguous: a balanced static partition (the first part_rem
    // workgroups take one extra datagram), sub-tiles of 256 from P0.  Strided
    // (tile_stride = G): sub-tile s is the batch's tile g + s G, so the resident
    // workgroups sweep neighbouring tiles at any moment (an address window of
    // G tiles instead of the whole batch) and a packed tile's output offset is
    // its tile prefix.
    const uint64_t G = B.tile_stride;
    const bool strided = G != 0;
    uint64_t P0 = 0, P1 = B.n;
    uint32_t nsub;
    if (strided) {
        const uint64_t ntiles = (B.n + kTile - 1) / kTile;
        if (g >= ntiles) return;
        nsub = (uint32_t)((ntiles - 1 - g) / G + 1);
    } else {
        P0 = g * B.part_len + min<uint64_t>(g, B.part_rem);
        P1 = P0 + B.part_len + (g < B.part_rem ? 1 : 0);
        if (P0 >= P1) return;
        nsub = (uint32_t)((P1 - P0 + kTile - 1) / kTile);
    }
    // first datagram of sub-tile s, and one past its last
    auto sub_first = [&](uint32_t s) -> uint64_t {
        return strided ? (g + (uint64_t)s * G) * kTile : P0 + (uint64_t)s * kTile;
    };
    auto sub_end = [&](uint64_t ps) -> uint64_t { return min<uint64_t>(ps + kTile, P1); };
    const uint8_t* __restrict__ in = B.in;
    const uint32_t nsteps = 12 * K.nblk;

    // block-wide exclusive scan (sum); every thread must call
    auto block_scan = [&](uint64_t x, uint64_t& total) -> uint64_t {
        const uint64_t inc = wave_incl_scan(x, lane);
        if (lane == 63) s_sum[wid] = inc;
        __syncthreads();
        uint64_t pre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kTile / 64; ++w) {
            const uint64_t v = s_sum[w];
            pre += (w < wid) ? v : 0;
            tot += v;
        }
        __syncthreads();
        total = uni64(tot);
        return pre + inc - x;
    };

    // output offset of datagram P0 (packed layout)
    uint64_t carry = 0;
    if (PACKED && !strided) {
        const uint64_t tb = P0 / kTile * kTile;
        uint32_t Wt = 0;
        if (tb + t < P0) Wt = out_width<OBF>(pkt_len(B, tb + t), B.pkt_cap);
        uint64_t tot;
        (void)block_scan(Wt, tot);
        carry = B.tile_prefix[P0 / kTile] + tot;
    }
    uint64_t written = 0;

    // ---- per-lane state of the datagram being prepared (next sub-tile)
    uint64_t pp = 0, pioff = 0, psalt = 0;
    uint32_t pL = 0;
    HashState<SW> hs;

    auto prep_load = [&](uint32_t s) {   // issue the global loads of sub-tile s
        pp = sub_first(s) + t;
        pL = 0;
        pioff = 0;
        psalt = 0;
        if (pp < sub_end(sub_first(s))) {
            pL = pkt_len(B, pp);
            pioff = pkt_in_off(B, pp);
            if (OBF) psalt = B.salts[pp];
        }
    };
    // widths, offsets, drop rules, LDS metadata of sub-tile s (has __syncthreads)
    auto prep_finish = [&](uint32_t s, TileBuf& T) {
        const uint64_t ps = sub_first(s);
        const uint32_t cnt = (uint32_t)(sub_end(ps) - ps);
        const bool live = (uint32_t)t < cnt;
        uint32_t W = live ? out_width<OBF>(pL, B.pkt_cap) : 0u;
        uint64_t ooff, first;
        if (PACKED) {
            uint64_t tot;
            if (strided) carry = B.tile_prefix[ps / kTile];   // ps is a tile start
            ooff = carry + block_scan(W, tot);
            first = carry;
            carry += tot;
        } else {
            ooff = pp * B.out_stride;
            first = ps * B.out_stride;
        }
        if (W && ooff + W > B.out_cap) W = 0;   // does not fit: dropped, offsets unchanged
        if (live) {
            if (B.out_off) B.out_off[pp] = ooff;
            if (B.out_len) B.out_len[pp] = W;
        }
        written += W;
        if (!OBF && W) psalt = load8u(in + pioff);   // the wire's salt; used at the first round
        const uint64_t base = first & ~15ull;
        const uint32_t rel = live ? (uint32_t)(ooff - base) : 0xFFFFFFFFu;
        const uint32_t end = W ? rel + W : 0u;
        // exclusive max-scan of region ends (ownership of shared chunks)
        uint32_t incm = end;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incm, d, 64);
            if (lane >= d) incm = max(incm, y);
        }
        const uint32_t prevl = __shfl_up(incm, 1, 64);
        if (lane == 63) s_max[wid] = incm;
        __syncthreads();
        uint32_t prem = 0, totm = 0;
#pragma unroll
        for (int w = 0; w < kTile / 64; ++w) {
            const uint32_t v = s_max[w];
            prem = (w < wid) ? max(prem, v) : prem;
            totm = max(totm, v);
        }
        totm = uni32(totm);
        T.o[t] = rel;
        T.w[t] = W;
        T.pe[t] = lane ? max(prem, prevl) : prem;
        T.io[t] = pioff + SKIP;
        if (OBF) T.salt[t] = psalt;
        if (t == 0) {
            T.base = base;
            T.nchunks = (totm + 15u) >> 4;
            T.cnt = cnt;
        }
    };
    auto finish_key = [&](TileBuf& T) {   // all rounds done: rotate and publish the key
        uint64_t key[4], kr[4];
        hash_key<SW>(hs, K, key);
        rotl_key_bytes(key, (T.o[t] + SALT) & 31u, kr);
        T.key[2 * t] = make_uint4((uint32_t)kr[0], (uint32_t)(kr[0] >> 32), (uint32_t)kr[1],
                                  (uint32_t)(kr[1] >> 32));
        T.key[2 * t + 1] = make_uint4((uint32_t)kr[2], (uint32_t)(kr[2] >> 32), (uint32_t)kr[3],
                                      (uint32_t)(kr[3] >> 32));
    };

    // Sub-tile s is swept while sub-tile s+1 is prepared and hashed.  s = -1
    // sweeps nothing: it only prepares sub-tile 0 (the one hash not overlapped
    // with the stream).  Each piece of code below is inlined once, to keep the
    // kernel small for the instruction cache.
    for (int s = -1; s < (int)nsub; ++s) {
        const TileBuf& T = buf[s & 1];
        TileBuf& N = buf[(s + 1) & 1];
        const bool has_next = s + 1 < (int)nsub;
        const uint32_t nchunks = s >= 0 ? uni32(T.nchunks) : 0u;
        const uint32_t cnt = s >= 0 ? uni32(T.cnt) : 0u;
        const uint32_t d0 = s >= 0 ? uni32(T.o[0]) : 0u;
        uint8_t* __restrict__ outb = B.out + (s >= 0 ? uni64(T.base) : 0ull);
        const uint32_t n_iters = (nchunks + kTile * U - 1) / (kTile * U);

        auto issue = [&](uint32_t it, SweepRegs& R) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = it * (kTile * U) + u * kTile + t;
                const uint32_t a = c << 4;
                uint32_t q;
                if (PACKED) {   // last datagram whose region starts at or before a
                    q = 0;
#pragma unroll
                    for (uint32_t step = kTile / 2; step; step >>= 1)
                        q = (T.o[q + step] <= a) ? q + step : q;
                } else {
                    const uint32_t x = a >= d0 ? a - d0 : 0u;
                    q = (uint32_t)((double)x * B.inv_stride);
                    const uint64_t stv = B.out_stride;
                    if ((uint64_t)(q + 1) * stv <= x) ++q;
                    if ((uint64_t)q * stv > x) --q;
                    q = min(q, cnt - 1);
                }
                R.q[u] = q;
                const uint32_t oq = T.o[q], wq = T.w[q];
                R.fast[u] = (c < nchunks) && wq != 0 && oq + SALT <= a && a + 16 <= oq + wq;
                R.v[u] = 0;
                if (R.fast[u] && HY_OK(1, T.io[q] + (a - oq - SALT) + 16 <= B.dbg_in_bytes, T.io[q], a, oq,
                                       ((uint64_t)q << 32) | (uint32_t)s))
                    R.v[u] = load16_stream(in + T.io[q] + (a - oq - SALT));
            }
        };
        auto retire = [&](uint32_t it, const SweepRegs& R) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                u128 v = R.v[u];
#if HY_PERSIST_PARK
                bool parked = false;
                if (PACKED && !R.fast[u]) {   // a parked boundary chunk of datagram q?
                    const uint32_t c = it * (kTile * U) + u * kTile + t;
                    const uint32_t q = R.q[u], m = c < nchunks ? s_parkm[q] : 0u;
                    if (m) {
                        const uint32_t cs = T.o[q] >> 4, ce = (T.o[q] + T.w[q] - 1) >> 4;
                        const int i = c == cs ? 0 : c == cs + 1 ? 1 : c == ce ? 2 : 3;
                        if (i < 3 && (m >> i & 1)) {   // stored pre-XORed with the key half below
                            const uint4 pv = s_park[3 * q + i];
                            __builtin_memcpy(&v, &pv, 16);
                            parked = true;
                        }
                    }
                }
                if (!R.fast[u] && !parked) continue;   // one store instruction for both
#else
                if (!R.fast[u]) continue;
#endif
                const uint32_t a = (it * (kTile * U) + u * kTile + t) << 4;
                const uint4 kk = T.key[2 * R.q[u] + ((a >> 4) & 1)];
                u128 k128;
                __builtin_memcpy(&k128, &kk, 16);
                if (HY_OK(2, (uint64_t)(outb - B.out) + a + 16 <= B.out_cap, (uint64_t)(outb - B.out), a,
                          nchunks, ((uint64_t)R.q[u] << 32) | (uint32_t)s))
                    store16_stream(outb + a, v ^ k128);
            }
        };

        const uint32_t steps = has_next ? nsteps : 0u;
        if (has_next) prep_load(s + 1);
        auto boundary = [&]() {   // chunks datagram t owns that are not inside one payload
#if HY_PERSIST_PARK
            uint32_t pm = 0;
#endif
            if ((uint32_t)t < cnt && T.w[t]) {
                const uint32_t st = T.o[t], en = st + T.w[t];
                const uint32_t cs = st >> 4, ce = (en - 1) >> 4;
                const bool own_cs = T.pe[t] <= (cs << 4);
                const uint32_t cand[3] = {cs, cs + 1, ce};
                const bool use[3] = {own_cs, cs + 1 <= ce, ce > cs + 1};
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    if (!use[i]) continue;
                    const uint32_t a = cand[i] << 4;
                    if (st + SALT <= a && a + 16 <= en) continue;   // inside the payload: swept
                    u128 r = 0;
                    uint32_t cov = 0;
                    for (uint32_t k = t; k < cnt && T.o[k] < a + 16; ++k) chunk_contrib<OBF>(B, T, in, k, a, r, cov);
#if HY_PERSIST_PARK
                    if (PACKED && cov == 0xFFFFu) {   // complete: the sweep stores it (XORing the key half again)
                        const uint4 kk = T.key[2 * t + ((a >> 4) & 1)];
                        u128 k128;
                        __builtin_memcpy(&k128, &kk, 16);
                        const u128 x = r ^ k128;
                        s_park[3 * t + i] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64),
                                                       (uint32_t)(x >> 96));
                        pm |= 1u << i;
                        continue;
                    }
#endif
                    if (cov && HY_OK(3, (uint64_t)(outb - B.out) + a + 16 <= B.out_cap + 15, (uint64_t)(outb - B.out),
                                     a, cov, s))
                        store_masked(outb + a, r, cov);
                }
            }
#if HY_PERSIST_PARK
            s_parkm[t] = pm;
#endif
        };
        // Sweep iteration it: issue its loads; while they fly, finish the
        // boundary chunks (iteration 0) and run one round of the next
        // sub-tile's hash; then XOR and store.  (A one-iteration-ahead prefetch
        // measured slower: its registers cost a wave per SIMD.)
        const uint32_t n_loop = max(max(n_iters, steps + 1), cnt ? 1u : 0u);
        for (uint32_t it = 0; it < n_loop; ++it) {
            SweepRegs R;
            if (it < n_iters) issue(it, R);
            if (it == 0) {
                boundary();
#if HY_PERSIST_PARK
                if (PACKED) __syncthreads();   // parked chunks visible to every sweep lane
#endif
            }
            if (it >= 1 && it <= steps) hash_step<SW>(hs, K, it - 1);
            if (it < n_iters) retire(it, R);
            if (it == 0 && has_next) {
                prep_finish(s + 1, N);
                hash_begin<SW>(hs, K, psalt);
            }
        }
        if (has_next) finish_key(N);
        __syncthreads();
    }

    // bytes written by this workgroup
    if (B.out_total) {
        const uint64_t ws = wave_sum(written);
        if (lane == 0 && ws) atomicAdd(B.out_total, (unsigned long long)ws);
    }
}

#ifndef HY_PERSIST_STRIDED
#define HY_PERSIST_STRIDED 0
#endif

// Resident workgroups per CU of one main-kernel instantiation (persistent grid).
template <bool OBF, bool PACKED, int SW>
int resident_per_cu() {
    static int cached = 0;
    if (!cached) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, salamander_kernel<OBF, PACKED, SW>, kTile, 0) !=
                hipSuccess ||
            nb < 1)
            nb = 1;
        cached = nb;
    }
    return cached;
}

inline int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    return cus;
}

template <bool OBF, bool PACKED, int SW>
void launch_main_sw(const BatchParams& bp, const KeyParams& k, hipStream_t s) {
    // every workgroup resident (static partition), at least a wave of datagrams each
    const uint64_t full = (uint64_t)device_cus() * resident_per_cu<OBF, PACKED, SW>();
    // HYOBFS_PERSIST_ORDER=strided|contiguous (read per launch: in-process A/B)
    const char* e = std::getenv("HYOBFS_PERSIST_ORDER");
    const bool strided = e ? std::strcmp(e, "strided") == 0 : HY_PERSIST_STRIDED;
    const uint64_t grid = std::min<uint64_t>(full, strided ? div_up(bp.n, kTile) : div_up(bp.n, 64));
    BatchParams b = bp;
    b.part_len = bp.n / grid;
    b.part_rem = bp.n % grid;
    b.tile_stride = strided ? (uint32_t)grid : 0u;
    hipLaunchKernelGGL((salamander_kernel<OBF, PACKED, SW>), dim3((uint32_t)grid), dim3(kTile), 0, s, b, k);
}


}  // namespace hyobfs
