// salamander_device.h -- device helpers shared by the Salamander kernels
// (salamander_wave.h, salamander_tile.h) and the Gecko encoder: BLAKE2b,
// byte-window arithmetic, the reference's width rules, wave scans, stores.
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

// 16 readable bytes for loads whose value is discarded (sweeps that issue their
// loads unconditionally, so the compiler's vmcnt waits stay exact)
__device__ __forceinline__ const uint8_t* hy_safe_line() {
#ifdef HYOBFS_EMULATE
    static const uint8_t z[64] = {};
    return z;
#else
    static __device__ uint8_t z[64];
    return z;
#endif
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
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t y = __shfl_xor(x, d, 64);
        x = x > y ? x : y;
    }
    return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x = max(x, (uint32_t)__shfl_xor(x, d, 64));
    return x;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

// quad_perm DPP move (lane i of each quad reads lane CTRL[i]): the diagonal steps of
// four-lanes-per-state BLAKE2b (salamander_tile.h) and ChaCha (gecko.hip)
// update_dpp with bound_ctrl (zero fill; quad_perm never reads out of bounds, so the
// result is the plain permute): that lets the compiler fold the permute into the VALU
// instruction that reads it (v_add_u32_dpp, v_xor_b32_dpp) instead of a separate
// v_mov_b32_dpp -- 207 of the Gecko kernel's 216 such moves (ChaCha diagonals)
#ifndef HY_DPP_FUSE
#define HY_DPP_FUSE 1
#endif
template <int CTRL>
__device__ __forceinline__ uint32_t qperm32(uint32_t x) {
#if HY_DPP_FUSE
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
#else
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
#endif
}
constexpr int kQRot1 = 0x39;   // quad_perm [1,2,3,0]: lane i reads lane i+1
constexpr int kQRot2 = 0x4E;   // [2,3,0,1]
constexpr int kQRot3 = 0x93;   // [3,0,1,2]

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

}  // namespace hyobfs
