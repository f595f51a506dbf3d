// salamander_tile.h -- the one-shot tile kernel for slotted batches whose region
// edges all fall on 8-byte boundaries (gfx950).
//
// Reference: extras/obfs/salamander.go:59-91 (Obfuscate, Deobfuscate, keyLocked).
//
// A workgroup of four waves owns a TILE of 16 consecutive datagrams and exits
// when it is done.  16 slots of a multiple of 8 bytes are whole 128-byte lines,
// so no line is shared by two workgroups (which may sit on different XCDs).
//   * wave 0 (keys): loads the 16 salts and hashes BLAKE2b-256(PSK || salt)
//     with four lanes per key (one G column each, the diagonal step by DPP
//     quad permutes), about 1k VALU instructions for all 16 keys, into LDS.
//   * waves 1-3 (data): each thread classifies its kTU output chunks (16 bytes,
//     1 KiB per wave instruction) and issues their loads at once.  With every
//     region edge on an 8-byte boundary, each 8-byte half of a chunk is a salt,
//     8 payload bytes of one datagram, or nothing, and one 16-byte window inside
//     a payload holds every payload half of the chunk.  After one LDS-only
//     barrier (the loads stay in flight across it, so they overlap the hash),
//     each payload half is XORed with its key word and the chunk is stored.
// The access shape is the one-shot region copy of a few KiB per wave, the
// fastest copy shape measured on MI355X (tools/region_copy.hip).  Slots larger
// than 16 x 192 x kTU / 16 bytes take several passes.  Applies when
// tile_params() holds; everything else runs the wave kernel.
#pragma once
#include "salamander_wave.h"

namespace hyobfs {

constexpr int kTileMaxD = 16;        // datagrams per tile: one wave hashes 16 keys, 4 lanes each;
                                     // 16 slots of a multiple of 8 bytes are whole 128-byte lines
#ifndef HY_TILE_U
#define HY_TILE_U 7
#endif
constexpr int kTU = HY_TILE_U;       // output chunks per data thread and pass (192 x 7 x 16 B = 21 KiB:
                                     // one pass for 16 slots of up to 1344 bytes)
constexpr uint64_t kMaxTileSlot = 1u << 20;
#ifndef HY_TILE_MIN_WAVES
#define HY_TILE_MIN_WAVES 8
#endif

struct TileParams {
    uint32_t S;      // output slot (out_stride), a multiple of 8
    uint32_t W;      // output width, a multiple of 8, 16 <= W <= S
    float invS;      // 1 / S
};

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
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, false);
    return (uint64_t)hi << 32 | lo;
}
constexpr int kQRot1 = 0x39;   // quad_perm [1,2,3,0]: lane i reads lane i+1
constexpr int kQRot2 = 0x4E;   // [2,3,0,1]
constexpr int kQRot3 = 0x93;   // [3,0,1,2]

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

// Per-chunk record kept across the barrier (one register):
//   bits 0-7  key word index of the low half in s_key (datagram * 8 + word; the
//             high half's word follows it, keys are stored twice in a row)
//   bits 8-11 datagram whose salt the chunk carries
//   bit 12/13 low/high half written; bit 14/15 low/high half is a salt
//   bit 16    low half from the window's high 8 bytes; bit 17 high half from its low 8
constexpr uint32_t kTcVlo = 1u << 12, kTcVhi = 1u << 13, kTcSlo = 1u << 14, kTcShi = 1u << 15;
constexpr uint32_t kTcLoFromHi = 1u << 16, kTcHiFromLo = 1u << 17;

// One output chunk: classification (tc record) and its 16-byte input window.
template <bool OBF>
__device__ __forceinline__ uint32_t tile_chunk(const uint8_t* __restrict__ ib, uint32_t in_stride, uint32_t S,
                                               uint32_t W, float invS, uint32_t nt, uint32_t tbytes, uint32_t x,
                                               u128& v) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;   // salt bytes in front of the output payload
    constexpr uint32_t SKIP = OBF ? 0u : 8u;   // salt bytes in front of the input payload
    v = 0;
    if (x >= tbytes) return 0;
    uint32_t p = (uint32_t)((float)x * invS);   // datagram of the low half (float estimate, fixed below)
    int32_t r = (int32_t)(x - p * S);
    if (r < 0) {
        --p;
        r += (int32_t)S;
    } else if (r >= (int32_t)S) {
        ++p;
        r -= (int32_t)S;
    }
    uint32_t r2 = (uint32_t)r + 8u, p2 = p;   // the high half
    if (r2 >= S) {
        r2 -= S;
        ++p2;
    }
    const bool vlo = (uint32_t)r < W;   // (then p < nt: x < tbytes)
    const bool vhi = p2 < nt && r2 < W;
    const bool slo = OBF && (uint32_t)r < 8u, shi = OBF && r2 < 8u;
    const bool plo = vlo && !slo, phi = vhi && !shi;
    const uint32_t jlo = (uint32_t)r - SALT, jhi = r2 - SALT;   // payload offsets (when payload)
    uint32_t f = (vlo ? kTcVlo : 0u) | (vhi ? kTcVhi : 0u) | (slo ? kTcSlo : 0u) | (shi ? kTcShi : 0u);
    f |= ((slo ? p : p2) & 15u) << 8;   // (p2 may be nt when no half is a salt)
    uint32_t wp = p, wj = jlo;          // window: datagram, payload offset
    if (plo) {
        // tile_params: a payload half next to another datagram's payload half never occurs
        if (!(phi && p2 == p)) {   // the payload's last word: the window ends with it
            wj = jlo - 8u;
            f |= kTcLoFromHi;
        }
        f |= p * 8u + ((jlo >> 3) & 3u);
    } else if (phi) {
        wp = p2;
        wj = jhi;
        f |= kTcHiFromLo | (p2 * 8u + ((jhi >> 3) & 3u) + 3u);
    }
#ifdef HY_X_TILE_ALIGN   // ablation builds only (wrong output): every window 16-aligned
    if (plo || phi) v = load16_nt(ib + ((wp * in_stride + SKIP + wj) & ~15u));
#elif defined(HY_X_TILE_PLAIN_LOADS)
    if (plo || phi) v = load16u(ib + (wp * in_stride + SKIP + wj));
#else
    if (plo || phi) v = load16_nt(ib + (wp * in_stride + SKIP + wj));
#endif
    return f;
}

// XOR with the key words (and salts) from LDS, store the chunk.
__device__ __forceinline__ void tile_store(uint8_t* __restrict__ ob, const uint64_t* s_key, const uint64_t* s_salt,
                                           uint32_t f, uint32_t x, u128 v) {
    if (!(f & (kTcVlo | kTcVhi))) return;
    const uint32_t ki = f & 0xFFu;
    const uint64_t k0 = s_key[ki], k1 = s_key[ki + 1];
    const uint64_t wlo = (uint64_t)v, whi = (uint64_t)(v >> 64);
    uint64_t lo = ((f & kTcLoFromHi) ? whi : wlo) ^ k0;
    uint64_t hi = ((f & kTcHiFromLo) ? wlo : whi) ^ k1;
    if (f & (kTcSlo | kTcShi)) {
        const uint64_t sv = s_salt[(f >> 8) & 15u];
        if (f & kTcSlo) lo = sv;
        if (f & kTcShi) hi = sv;
    }
    if ((f & (kTcVlo | kTcVhi)) == (kTcVlo | kTcVhi))
#ifdef HY_X_TILE_PLAIN_STORES
        __builtin_memcpy(ob + x, &lo, 8), __builtin_memcpy(ob + x + 8, &hi, 8);
#else
        store16_global(ob + x, lo, hi);
#endif
    else if (f & kTcVlo)
        store8_global(ob + x, lo);
    else
        store8_global(ob + x + 8, hi);
}

template <bool OBF, int SW>
__global__ __launch_bounds__(256, HY_TILE_MIN_WAVES) void salamander_tile_kernel(BatchParams B, KeyParams K,
                                                                                  TileParams T) {
    __shared__ uint64_t s_key[kTileMaxD * 8];   // each key twice: word w and w + 4 equal
    __shared__ uint64_t s_salt[kTileMaxD];

    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = uni32(tid >> 6);
    const uint32_t S = T.S, W = T.W;
    const uint64_t p0 = (uint64_t)blockIdx.x * kTileMaxD;
    const uint32_t nt = (uint32_t)min<uint64_t>((uint64_t)kTileMaxD, B.n - p0);
    const uint32_t tbytes = (nt - 1) * S + W;   // tile-local end of the last region
    const uint8_t* __restrict__ ib = B.in + p0 * B.in_stride;
    const uint32_t in_stride = (uint32_t)B.in_stride;

    if (wid == 0) {
        // ---- the key wave: salts, BLAKE2b-256 on quads (lane 4k+i: word i of key k), LDS
        const uint32_t qk = lane >> 2, qi = lane & 3;
        uint64_t salt = 0;
        if (qk < nt) salt = OBF ? B.salts[p0 + qk] : load8_nt(ib + qk * in_stride);
#if defined(HY_X_NOHASH) || defined(HY_X_TILE_NOHASH)   // ablation builds only (wrong output)
        const uint64_t kw = salt * (qi + 3);
#else
        const uint64_t kw = quad_key<SW>(K, salt, qi);
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
#ifndef HY_X_TILE_NOBAR
        hy_lds_barrier();
#endif
        return;
    }

    // ---- the three data waves: 1 KiB of output per wave instruction, kTU chunks
    // per thread in flight; the first pass's loads are issued before the barrier
    // that publishes the keys, so they overlap the hash
    constexpr uint32_t kPass = 192u * kTU;      // chunks per pass
    const uint32_t dt = tid - 64u;
    uint8_t* __restrict__ ob = B.out + p0 * S;
    const uint32_t nch = (tbytes + 15u) >> 4;
    for (uint32_t c0 = 0; c0 < nch; c0 += kPass) {
        u128 v[kTU];
        uint32_t tc[kTU];
#pragma unroll
        for (int u = 0; u < kTU; ++u)
            tc[u] = tile_chunk<OBF>(ib, in_stride, S, W, T.invS, nt, tbytes, (c0 + (uint32_t)u * 192u + dt) << 4, v[u]);
#ifndef HY_X_TILE_NOBAR   // (ablation builds only: keys not waited for, wrong output)
        if (c0 == 0) hy_lds_barrier();
#endif
#pragma unroll
        for (int u = 0; u < kTU; ++u)
            tile_store(ob, s_key, s_salt, tc[u], (c0 + (uint32_t)u * 192u + dt) << 4, v[u]);
    }
}

// The tile kernel applies to slotted batches where every datagram has one
// length, the slot, the input stride and the input base are multiples of 8, the
// payload is at least 16 bytes, nothing is dropped, and no 16-byte chunk holds
// payload bytes of two datagrams (deobfuscate into dense slots of 8 mod 16).
template <bool OBF>
inline bool tile_params(const BatchParams& b, TileParams& T) {
    if (b.out_stride == 0 || b.in_len || b.in_off || b.n == 0) return false;
    if (reinterpret_cast<uintptr_t>(b.out) & 15u) return false;
    const uint64_t L = b.len_uniform;
    if (L > kMaxDatagram || L < (OBF ? 16u : 24u)) return false;
    if ((L | b.out_stride | b.in_stride | reinterpret_cast<uintptr_t>(b.in)) & 7u) return false;
    if (b.in_stride > 0xFFFFFFFFull / kTileMaxD) return false;
    const uint64_t W = OBF ? L + 8 : L - 8, S = b.out_stride;
    if ((b.pkt_cap && W > b.pkt_cap) || W > S) return false;
    if ((b.n - 1) * S + W > b.out_cap) return false;
    if (!OBF && S == W && (W & 15u)) return false;
    if (S > kMaxTileSlot) return false;   // tile-local offsets stay 32-bit, float estimate exact enough
    T.S = (uint32_t)S;
    T.W = (uint32_t)W;
    T.invS = 1.0f / (float)S;
    return true;
}

template <bool OBF, int SW>
void launch_tile_sw(const BatchParams& b, const KeyParams& k, const TileParams& T, hipStream_t s) {
    const uint64_t blocks = div_up(b.n, kTileMaxD);
    hipLaunchKernelGGL((salamander_tile_kernel<OBF, SW>), dim3((uint32_t)blocks), dim3(256), 0, s, b, k, T);
}

}  // namespace hyobfs
