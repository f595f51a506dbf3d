// gecko_device.h -- device helpers shared by the Gecko encode kernels (gecko.hip,
// gecko_tile.h): 16-byte helpers and the padding keystream (include/hyobfs_gecko.h).
#pragma once
#include "kernels.h"
#include "salamander_device.h"
#include "../../include/hyobfs_gecko.h"

namespace hyobfs {

typedef unsigned __int128 gk_u128;
__device__ __forceinline__ gk_u128 gk_load16u(const uint8_t* p) {   // any alignment
    gk_u128 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ void gk_store16u(uint8_t* p, gk_u128 v) { __builtin_memcpy(p, &v, 16); }
__device__ __forceinline__ gk_u128 gk_mask(uint32_t lo, uint32_t hi) {   // bytes [lo, hi) of 16
    const uint32_t nb = hi - lo;
    const gk_u128 m = nb >= 16 ? ~(gk_u128)0 : (((gk_u128)1 << (8 * nb)) - 1);
    return m << (8 * lo);
}

// ---- padding keystream (include/hyobfs_gecko.h): ChaCha, 8 rounds, RFC 8439 block
// (constants, 8 key words, 32-bit counter, 3 nonce words), each 64-byte block's
// bytes in column order: keystream bytes 64 blk + 16 c .. + 15 are state words c,
// c + 4, c + 8, c + 12.  Pad byte j of frame i is keystream byte out_off[i] + 13 + j.
// Column order lets four lanes compute one block, a column each, with no transpose.
#ifndef HY_GK_PAD_ROUNDS
#define HY_GK_PAD_ROUNDS 8
#endif
struct GkPad {
    uint32_t k[8], n[3];
};
__device__ __forceinline__ GkPad gk_pad_params(const hyobfs_gecko_batch& B) {
    GkPad P;
    __builtin_memcpy(P.k, B.pad_key, 32);
    __builtin_memcpy(P.n, B.pad_nonce, 12);
    return P;
}
__device__ __forceinline__ uint32_t gk_rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
#define GK_QR(a, b, c, d)         \
    do {                          \
        a += b;                   \
        d = gk_rotl(d ^ a, 16);   \
        c += d;                   \
        b = gk_rotl(b ^ c, 12);   \
        a += b;                   \
        d = gk_rotl(d ^ a, 8);    \
        c += d;                   \
        b = gk_rotl(b ^ c, 7);    \
    } while (0)
constexpr uint32_t kChaC0 = 0x61707865u, kChaC1 = 0x3320646Eu, kChaC2 = 0x79622D32u, kChaC3 = 0x6B206574u;
__device__ __forceinline__ uint32_t gk_sel4(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, uint32_t i) {
    return i == 0 ? x0 : i == 1 ? x1 : i == 2 ? x2 : x3;
}

// Column qi (= this lane's place in its quad) of keystream block blk: the four lanes
// of a quad compute one block, a column each, the diagonal step by DPP quad
// permutes.  Every lane of the wave must execute it (the permutes read neighbours).
__device__ __forceinline__ gk_u128 gk_ks_quad(const GkPad& P, uint32_t blk, uint32_t qi) {
    const uint32_t a0 = gk_sel4(kChaC0, kChaC1, kChaC2, kChaC3, qi);
    const uint32_t b0 = gk_sel4(P.k[0], P.k[1], P.k[2], P.k[3], qi);
    const uint32_t c0 = gk_sel4(P.k[4], P.k[5], P.k[6], P.k[7], qi);
    const uint32_t d0 = gk_sel4(blk, P.n[0], P.n[1], P.n[2], qi);
    uint32_t a = a0, b = b0, c = c0, d = d0;
#pragma unroll
    for (int r = 0; r < HY_GK_PAD_ROUNDS / 2; ++r) {
        GK_QR(a, b, c, d);   // column round
        b = qperm32<kQRot1>(b);
        c = qperm32<kQRot2>(c);
        d = qperm32<kQRot3>(d);
        GK_QR(a, b, c, d);   // diagonal round
        b = qperm32<kQRot3>(b);
        c = qperm32<kQRot2>(c);
        d = qperm32<kQRot1>(d);
    }
    return (gk_u128)(d + d0) << 96 | (gk_u128)(c + c0) << 64 | (gk_u128)(b + b0) << 32 | (a + a0);
}

// The same column computed by one lane alone (edge chunks, divergent code).
__device__ __forceinline__ gk_u128 gk_ks_single(const GkPad& P, uint32_t blk, uint32_t col) {
    uint32_t x[16] = {kChaC0, kChaC1, kChaC2, kChaC3, P.k[0], P.k[1], P.k[2], P.k[3],
                      P.k[4], P.k[5], P.k[6], P.k[7], blk,    P.n[0], P.n[1], P.n[2]};
    uint32_t s[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = x[i];
#pragma unroll
    for (int r = 0; r < HY_GK_PAD_ROUNDS / 2; ++r) {
        GK_QR(x[0], x[4], x[8], x[12]);
        GK_QR(x[1], x[5], x[9], x[13]);
        GK_QR(x[2], x[6], x[10], x[14]);
        GK_QR(x[3], x[7], x[11], x[15]);
        GK_QR(x[0], x[5], x[10], x[15]);
        GK_QR(x[1], x[6], x[11], x[12]);
        GK_QR(x[2], x[7], x[8], x[13]);
        GK_QR(x[3], x[4], x[9], x[14]);
    }
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = gk_sel4(x[4 * j] + s[4 * j], x[4 * j + 1] + s[4 * j + 1], x[4 * j + 2] + s[4 * j + 2],
                                               x[4 * j + 3] + s[4 * j + 3], col);
    return (gk_u128)w[3] << 96 | (gk_u128)w[2] << 64 | (gk_u128)w[1] << 32 | w[0];
}

// Keystream bytes [W0, W0 + 16) for any W0 (one or two columns).
__device__ __forceinline__ gk_u128 gk_ks_at(const GkPad& P, uint64_t W0) {
    const uint64_t c0 = W0 & ~15ull;
    const uint32_t sh = (uint32_t)(W0 & 15);
    const gk_u128 x0 = gk_ks_single(P, (uint32_t)(c0 >> 6), (uint32_t)(c0 >> 4) & 3u);
    if (!sh) return x0;
    const gk_u128 x1 = gk_ks_single(P, (uint32_t)((c0 + 16) >> 6), (uint32_t)((c0 + 16) >> 4) & 3u);
    return (x0 >> (8 * sh)) | (x1 << (8 * (16 - sh)));
}

}  // namespace hyobfs
