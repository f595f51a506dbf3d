// salamander_flat.h -- the flat kernel: CONTIGUOUS input (datagram i at
// in + in_len[0] + ... + in_len[i-1], include/hyobfs.h) into PACKED output (gfx950).
// The layout of BASELINE configs[2] and of any batch a reader fills back to back.
//
// Reference: extras/obfs/salamander.go:59-91 (Obfuscate, Deobfuscate, keyLocked).
//
// The output is cut into tiles of kFT bytes (16 KiB), each written by one one-shot
// workgroup, so every 128-byte line leaves whole from one workgroup.  With contiguous
// input the payload bytes behind a tile are one contiguous input window, known from
// the tile's first datagram alone:
//   prepass: width and length sums per 256 datagrams and their scan (shared with the
//     wave kernel, salamander.hip), then flat_locate_kernel: per datagram its output
//     offset and width (the reference's return values, out_off / out_len) and, for
//     every tile whose first byte it holds, the tile's descriptor (the datagram, its
//     output and input offsets);
//   flat kernel, one workgroup of four waves per tile:
//     1. every wave issues its rows of the window's LDS-DMA (global_load_lds_dwordx4,
//        non-temporal, 1 KiB per wave instruction) first, so the copy is in flight
//        during everything else;
//     2. wave 0 loads the lengths and salts of the tile's datagrams (lane per
//        datagram), scans them (32-bit, tile-relative) and takes their keys from the
//        key records the launch's hasher workgroups write (flat_hasher, one lane per
//        key; a record not yet written after a bounded wait is hashed in place, four
//        lanes per key), rotated to the output's 32-byte phase, into the table;
//     3. one barrier, then every thread composes four 16-byte output chunks:
//        * inside one payload (the common case): two 8-byte LDS reads of the stage --
//          with contiguous input the stage offset of a datagram's payload is a
//          multiple of 8 away from its output offset -- XOR one 16-byte key read;
//        * across one region edge (a datagram's end, the next one's salt and start):
//          the two datagrams' stage reads, keys and salts, merged per 8-byte half by
//          three byte boundaries with bit-field selects (v_bfi_b32);
//        * anything else (three or more datagrams in a chunk, payload bytes outside
//          the window or off the 8-byte grid): a byte-masked merge that may read
//          global memory -- correct for every batch, rare for real traffic;
//        and stores each with one non-temporal 16-byte store (the batch's last chunk
//        byte-masked).
// A tile reached by more than kFD datagrams takes several passes of 2-3; a chunk two
// passes share gets each pass's bytes by a byte-masked store.  Applies to contiguous input with packed
// output and 16-byte aligned `in` and `out` (flat_eligible, salamander.hip); the wave
// kernel takes every other packed layout.
#pragma once
#include "salamander_tile.h"

namespace hyobfs {

#ifndef HY_FLAT_T
#define HY_FLAT_T 16384
#endif
constexpr uint32_t kFT = HY_FLAT_T;   // output bytes per tile
static_assert(kFT % 4096 == 0 && kFT <= 65536, "a tile is four 16-byte chunks per thread");
constexpr uint32_t kFThreads = kFT / 64;   // threads per workgroup: four output chunks each
constexpr uint32_t kFWaves = kFThreads / 64;
constexpr int kFU = 4;                     // output chunks per thread
constexpr int kFD = 64;                  // datagrams per pass (a lane each)
constexpr uint32_t kFGuard = 32;         // LDS bytes on both sides of the stage (reads of masked bytes)
// staged input bytes: a tile's payload bytes (obfuscate: at most kFT), plus the wire
// salts between them (deobfuscate: 8 per datagram of a pass), plus 16-byte rounding
template <bool OBF>
constexpr uint32_t flat_stage_bytes() { return kFT + (OBF ? 32u : 8u * kFD + 32u); }
// waves per SIMD the register budget is sized for: 7 (72 VGPRs) -- LDS allows about 8
// workgroups per CU anyway, and at 8 (64 VGPRs) the tile path spilled 21-31 VGPRs;
// 7 / 6 / 5 ran configs[2] in 1.541 / 1.597 / 1.665 ms against 1.640 at 8
// (profiles/r06_bimodal/ab_flat_vgpr_cap.txt)
#ifndef HY_FLAT_MIN_WAVES
#define HY_FLAT_MIN_WAVES 7
#endif
// w[] flag bits above the width (widths are < 2^24)
constexpr uint32_t kFlatOffWin = 1u << 31;   // some payload byte of the tile lies outside the staged window
constexpr uint32_t kFlatOffGrid = 1u << 30;  // stage offset not a multiple of 8 from the output offset
constexpr uint32_t kFlatWMask = kFlatOffGrid - 1u;

struct FlatDesc {       // one output tile: the first valid datagram reaching into it
    uint64_t d;         // its index
    uint64_t o;         // its output offset
    uint64_t i;         // its input offset
};

struct FlatParams {
    FlatDesc* desc;     // ntiles_max + 1 entries
    // the first datagram that does not fit out_cap (written by the one wave holding
    // it, ~0 = none): [0] its output offset = the end of the valid output, [1] its index
    uint64_t* cut;
    uint64_t ntiles_max;
    const uint64_t* in_total;    // input bytes: the length scan's total (device)
    const uint64_t* out_total;   // the width scan's total: the valid output's end without a cut
    uint8_t* krec;      // key records: per datagram 4 granules {key word, epoch} (krec_*)
    uint64_t epoch;     // this call's tag (never 0)
    uint32_t nhash;     // hasher workgroups in front of the tile workgroups
};

inline uint64_t flat_ntiles_max(uint64_t out_cap) { return (out_cap + kFT - 1) / kFT; }
constexpr uint64_t kKeyRec = 64;   // key record bytes per datagram
// the prepass's scratch: two header words, the descriptor of every tile out_cap allows,
// then (256-aligned) the key records
inline uint64_t flat_desc_bytes(uint64_t out_cap) { return 16 + sizeof(FlatDesc) * (flat_ntiles_max(out_cap) + 1); }
inline uint64_t flat_workspace_bytes(uint64_t out_cap, uint64_t n) {
    return ((flat_desc_bytes(out_cap) + 255) & ~255ull) + 256 + kKeyRec * n;
}

// Hasher workgroups per launch (HYOBFS_FLAT_HASHERS overrides; 0: every tile hashes its
// own keys).  They are the launch's first workgroups, so they start ahead of the tiles.
#ifndef HY_FLAT_HASHERS
#define HY_FLAT_HASHERS 256
#endif
#ifndef HY_FLAT_HASH_PRIO
#define HY_FLAT_HASH_PRIO 3
#endif
inline uint32_t flat_hashers() {
    static const uint32_t v = [] {
        const char* e = std::getenv("HYOBFS_FLAT_HASHERS");
        const long x = e ? std::atol(e) : HY_FLAT_HASHERS;
        return (uint32_t)(x < 0 ? 0 : x > 4096 ? 4096 : x);
    }();
    return v;
}

// ---- key records: the hand-off from the hasher workgroups to the tile workgroups
// inside one launch (MI355X_MICROARCH.md, inter-workgroup visibility; the per-XCD L2s
// are not coherent).  Datagram k's record is four 16-byte granules {key word w,
// epoch}, each written by ONE write-through (sc1) 16-byte store and read by ONE sc1
// 16-byte load: a granule carries its own tag, so a reader never needs a flag or a
// fence -- a tag equal to this call's epoch means that word is this call's key
// (records of earlier calls carry other epochs).
#ifdef HYOBFS_EMULATE
__device__ __forceinline__ void krec_store(uint8_t* blk, uint32_t off, uint64_t w, uint64_t tag) {
    std::memcpy(blk + off, &w, 8);
    std::memcpy(blk + off + 8, &tag, 8);
}
__device__ __forceinline__ void krec_load(const uint8_t* blk, uint32_t off, uint64_t& w, uint64_t& tag) {
    std::memcpy(&w, blk + off, 8);
    std::memcpy(&tag, blk + off + 8, 8);
}
#else
typedef uint32_t krec_v4 __attribute__((ext_vector_type(4)));
// blk: wave-uniform base of a 64-record (4 KiB) block
__device__ __forceinline__ __amdgpu_buffer_rsrc_t krec_rsrc(const uint8_t* blk) {
    const uint64_t a = uni64(reinterpret_cast<uint64_t>(blk));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(a), 0, (int)(64 * kKeyRec), 0x00020000);
}
__device__ __forceinline__ void krec_store(uint8_t* blk, uint32_t off, uint64_t w, uint64_t tag) {
    krec_v4 v;
    v.x = (uint32_t)w;
    v.y = (uint32_t)(w >> 32);
    v.z = (uint32_t)tag;
    v.w = (uint32_t)(tag >> 32);
    __builtin_amdgcn_raw_buffer_store_b128(v, krec_rsrc(blk), (int)off, 0, 16);   // aux 16: sc1
}
__device__ __forceinline__ void krec_load(const uint8_t* blk, uint32_t off, uint64_t& w, uint64_t& tag) {
    const krec_v4 v = __builtin_amdgcn_raw_buffer_load_b128(krec_rsrc(blk), (int)off, 0, 16);   // sc1
    w = (uint64_t)v.y << 32 | v.x;
    tag = (uint64_t)v.w << 32 | v.z;
}
#endif

// Per datagram: width (drop rules), output and input offsets from the scans, the
// reference's return values, and the descriptor of every tile whose first byte the
// datagram holds.  One wave per 256-datagram tile of the scan, four datagrams per lane.
// The valid output ends at the first datagram with a width that does not fit out_cap
// (every later one is dropped too); exactly one wave holds it -- the one whose first
// datagram's offset still fits -- and records it with plain stores.
template <bool OBF>
__global__ __launch_bounds__(256) void flat_locate_kernel(BatchParams B, FlatParams F, uint64_t ntiles) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t tile = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= ntiles) return;   // whole waves
    const uint64_t p0 = tile * kTile + 4ull * lane;
    uint32_t L[4], W[4];
    uint64_t sl = 0, sw = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        L[k] = p0 + k < B.n ? B.in_len[p0 + k] : 0u;
        W[k] = p0 + k < B.n ? out_width<OBF>(L[k], B.pkt_cap) : 0u;
        sl += L[k];
        sw += W[k];
    }
    const uint64_t wave_o = B.tile_prefix[tile];   // every earlier datagram with a width fits iff <= out_cap
    uint64_t o = wave_o + wave_incl_scan(sw, (int)lane) - sw;
    uint64_t i = B.in_tile_prefix[tile] + wave_incl_scan(sl, (int)lane) - sl;
    uint64_t cut = ~0ull;   // index of this lane's first datagram that does not fit
    uint64_t cut_o = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t p = p0 + k;
        if (p < B.n) {
            const bool fits = W[k] && o + W[k] <= B.out_cap;   // else dropped; offsets never move
            if (B.out_off) B.out_off[p] = o;
            if (B.out_len) B.out_len[p] = fits ? W[k] : 0u;
            if (fits) {
                for (uint64_t t = (o + kFT - 1) / kFT; t * kFT < o + W[k]; ++t) F.desc[t] = FlatDesc{p, o, i};
            } else if (W[k] && cut == ~0ull) {
                cut = p;
                cut_o = o;
            }
        }
        o += W[k];
        i += L[k];
    }
    // the first cut in this wave; the batch's first if everything before the wave fit
    const unsigned long long m = __ballot(cut != ~0ull);
    if (m && wave_o <= B.out_cap) {
        const int l0 = __builtin_ctzll(m);
        const uint64_t c = __shfl(cut, l0, 64), co = __shfl(cut_o, l0, 64);
        if (lane == 0) {
            F.cut[0] = co;
            F.cut[1] = c;
        }
    }
}

template <bool OBF>
struct FlatLDS {
    uint8_t stage[kFGuard + flat_stage_bytes<OBF>() + kFGuard];   // input window, byte 0 at stage[kFGuard]
    uint64_t key[kFD][4];     // key rotated to the output's 32-byte phase
    uint64_t salt[kFD];
    int32_t o[kFD + 1];       // output start relative to the tile ([m..] = INT_MAX)
    int32_t dlt[kFD];         // stage index of the payload byte at tile-relative output x: x + dlt
    uint32_t w[kFD];          // width (0: dropped) | kFlatOffWin | kFlatOffGrid
};

// The helpers below take any LDS layout with the fields of FlatLDS (stage with kFGuard
// bytes on both sides, key, salt, o, dlt, w).
// 16 bytes of the stage from stage index q (>= -kFGuard, < stage bytes + kFGuard - 16)
template <class LDS>
__device__ __forceinline__ u128 flat_stage16(const LDS& S, int32_t q) {
    const int32_t a = q + (int32_t)kFGuard;
    const int32_t b = a & ~15;
    const uint32_t sh = (uint32_t)(a & 15);
    const u128 A = *reinterpret_cast<const u128*>(S.stage + b);
    const u128 C = *reinterpret_cast<const u128*>(S.stage + b + 16);
    return sh ? (A >> (8 * sh)) | (C << (128 - 8 * sh)) : A;
}

// Payload bytes [base, base + 16) of the datagram whose PL payload bytes start at
// input position ip, of which the caller keeps [.., need) (the rest is masked): from
// the stage when the window holds the kept bytes, else one in-bounds global load.
template <class LDS>
__device__ __forceinline__ u128 flat_payload16(const LDS& S, const uint8_t* __restrict__ in, uint64_t ws,
                                               uint32_t wlen, uint64_t ip, uint32_t PL, int32_t base, int32_t need) {
    const int64_t pos = (int64_t)ip + base;
    if (pos >= (int64_t)ws - 16 && pos + need <= (int64_t)(ws + wlen)) return flat_stage16(S, (int32_t)(pos - (int64_t)ws));
    const uint8_t* src = in + ip;
    if (PL >= 16) {
        const int32_t w = min(max(base, 0), (int32_t)PL - 16);
        const u128 V = load16u(src + w);
        const int32_t d = w - base;
        return d >= 0 ? (V << (8 * d)) : (V >> (8 * -d));
    }
    u128 X = 0;
    for (int32_t j = max(base, 0); j < min(base + 16, (int32_t)PL); ++j) X |= (u128)src[j] << (8 * (j - base));
    return X;
}

// Everything datagram k of the table contributes to the chunk at tile-relative rel
// (the general merge: any alignment, any number of datagrams per chunk); kh = the
// chunk's key half (its output offset / 16, mod 2).
template <bool OBF, class LDS>
__device__ __forceinline__ void flat_contrib(const LDS& S, const uint8_t* __restrict__ in, uint64_t ws,
                                             uint32_t wlen, uint32_t k, int32_t rel, uint32_t kh, u128& r, uint32_t& cov) {
    constexpr int32_t SALT = OBF ? 8 : 0;
    const uint32_t W = S.w[k] & kFlatWMask;
    const int32_t o = S.o[k];
    if (W == 0 || o >= rel + 16 || o + (int32_t)W <= rel) return;
    if (OBF) {   // salt bytes [o, o + 8)
        const int32_t sb = max(o, rel), se = min(o + 8, rel + 16);
        if (sb < se) {
            u128 Sv = (u128)S.salt[k];
            Sv = o >= rel ? (Sv << (8 * (o - rel))) : (Sv >> (8 * (rel - o)));
            r |= Sv & bytemask((uint32_t)(sb - rel), (uint32_t)(se - rel));
            cov |= ((1u << (se - sb)) - 1u) << (sb - rel);
        }
    }
    const int32_t ps = max(o + SALT, rel), pe = min(o + (int32_t)W, rel + 16);
    if (ps < pe) {
        // the payload's input position: stage index of payload byte 0, back to input
        const uint64_t ip = (uint64_t)((int64_t)ws + (int64_t)(o + SALT) + S.dlt[k]);
        const u128 X = flat_payload16(S, in, ws, wlen, ip, W - (uint32_t)SALT, rel - (o + SALT), pe - rel);
        const uint64_t* kw = S.key[k] + 2 * kh;
        const u128 K = (u128)kw[1] << 64 | kw[0];
        r |= (X ^ K) & bytemask((uint32_t)(ps - rel), (uint32_t)(pe - rel));
        cov |= ((1u << (pe - ps)) - 1u) << (ps - rel);
    }
}

// Bytes [0, b) of an 8-byte half (b clamped to 0..8), as a 64-bit mask.
__device__ __forceinline__ uint64_t flat_lomask(int32_t b) {
    const uint32_t c = (uint32_t)min(max(b, 0), 8);
    return c ? ~0ull >> (64u - 8u * c) : 0ull;
}
// (m & x) | (~m & y) per bit: v_bfi_b32 on each half
__device__ __forceinline__ uint64_t flat_bfi(uint64_t m, uint64_t x, uint64_t y) { return (m & x) | (~m & y); }

// One 16-byte output chunk at tile-relative rel from the table of m datagrams (ND
// entries, o[ND] a sentinel), kh = 2 x its key half: true with the value when the chunk
// lies inside one payload, or across one region edge (q's salt or end, then at most the
// datagram after it) with both datagrams staged on the 8-byte grid; false when it needs
// the general merge.
template <bool OBF, int ND, class LDS>
__device__ __forceinline__ bool flat_chunk(const LDS& S, int32_t rel, uint32_t kh, uint32_t m, u128& value) {
    constexpr int32_t SALT = OBF ? 8 : 0;
    uint32_t q = 0;   // last datagram whose output starts at or before rel
#pragma unroll
    for (uint32_t s = ND / 2; s; s >>= 1) q = S.o[q + s] <= rel ? q + s : q;
    const int32_t oq = S.o[q];
    const uint32_t wq = S.w[q];
    const int32_t eq = oq + (int32_t)(wq & kFlatWMask);   // q's region end
    // q's region holds byte 0; at most q+1 (starting right at q's end, staged, on the
    // grid) holds the rest
    const uint32_t q1 = q + 1;
    const int32_t o1 = S.o[q1];   // == eq unless q is the last of the pass
    const uint32_t w1 = q1 < m ? S.w[q1] : 0u;
    const int32_t e1 = o1 + (int32_t)(w1 & kFlatWMask);
    const bool fast = oq <= rel && (wq & (kFlatOffWin | kFlatOffGrid)) == 0 && eq > rel &&
                      (eq >= rel + 16 || (o1 == eq && (w1 & (kFlatOffWin | kFlatOffGrid)) == 0 && e1 >= rel + 16));
    if (!fast) return false;
    const uint64_t* dq = reinterpret_cast<const uint64_t*>(S.stage + (rel + S.dlt[q] + (int32_t)kFGuard));
    const uint64_t xl = dq[0] ^ S.key[q][kh], xh = dq[1] ^ S.key[q][kh + 1];
    if (oq + SALT <= rel && rel + 16 <= eq) {   // inside q's payload
        value = (u128)xh << 64 | xl;
        return true;
    }
    // q's salt [oq, oq + 8), q's payload [oq + 8, eq), q+1's salt [eq, eq + 8),
    // q+1's payload: byte boundaries b1 <= b2 <= b3, chunk-relative
    uint64_t lo = 0, hi = 0;
    const int32_t b1 = oq + SALT - rel, b2 = eq - rel, b3 = b2 + SALT;
    if (eq < rel + 16) {   // q+1 starts in this chunk (b2 in 1..15)
        const uint64_t* d1 = reinterpret_cast<const uint64_t*>(S.stage + (rel + S.dlt[q1] + (int32_t)kFGuard));
        lo = d1[0] ^ S.key[q1][kh];
        hi = d1[1] ^ S.key[q1][kh + 1];
        if (OBF) {   // q+1's salt at byte b2
            const uint64_t s1 = S.salt[q1];
            const uint32_t e8 = 8u * (uint32_t)b2;
            const uint64_t s1l = e8 < 64 ? s1 << e8 : 0ull;
            const uint64_t s1h = e8 < 64 ? s1 >> (64 - e8) : s1 << (e8 - 64);
            lo = flat_bfi(flat_lomask(b3), s1l, lo);
            hi = flat_bfi(flat_lomask(b3 - 8), s1h, hi);
        }
    }
    lo = flat_bfi(flat_lomask(b2), xl, lo);
    hi = flat_bfi(flat_lomask(b2 - 8), xh, hi);
    if (OBF) {   // q's salt ends at byte b1 <= 8: low half only
        const uint32_t c8 = 8u * (uint32_t)min(rel - oq, 8);
        const uint64_t sq = c8 < 64 ? S.salt[q] >> c8 : 0ull;
        lo = flat_bfi(flat_lomask(b1), sq, lo);
    }
    value = (u128)hi << 64 | lo;
    return true;
}

// A hasher workgroup: its waves take 64-datagram blocks in index order (block
// h * waves + wave, then every nhash * waves), one lane per key (wave_key,
// salamander_wave.h: the fewest instructions per key), and publish each key as a
// record of four tagged granules.  Deobfuscate reads the wire salts at the offsets
// from the length scan.  Hashers never wait on anything.
template <bool OBF, int SW>
__device__ __forceinline__ void flat_hasher(const BatchParams& B, const KeyParams& K, const FlatParams& F, uint32_t h,
                                            uint32_t wid) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t step = (uint64_t)F.nhash * kFWaves;
#ifndef HYOBFS_EMULATE
    __builtin_amdgcn_s_setprio(HY_FLAT_HASH_PRIO);   // VALU-only waves among streaming ones: issue first
#endif
    for (uint64_t blk = (uint64_t)h * kFWaves + wid; blk * 64 < B.n; blk += step) {
        const uint64_t k = blk * 64 + lane;
        const bool live = k < B.n;
        uint64_t salt = 0;
        if (OBF) {
            salt = live ? B.salts[k] : 0ull;
        } else {   // the wire's salt at the datagram's input offset
            const uint64_t g = blk / 4;   // its 256-datagram scan tile
            uint64_t pre = 0;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const uint64_t q = g * kTile + 64ull * j + lane;
                if (q < blk * 64) pre += B.in_len[q];
            }
            const uint32_t L = live ? B.in_len[k] : 0u;
            const uint64_t i = B.in_tile_prefix[g] + wave_sum(pre) + wave_incl_scan32(L, (int)lane) - L;
            if (L > 8u) salt = load8u(B.in + i);
        }
        uint64_t key[4];
        wave_key<SW>(K, salt, key);
        uint8_t* kb = F.krec + kKeyRec * blk * 64;
        if (live) {
#pragma unroll
            for (int w = 0; w < 4; ++w) krec_store(kb, (uint32_t)(kKeyRec * lane + 16 * w), key[w], F.epoch);
        }
    }
}

template <bool OBF, int SW>
__global__ __launch_bounds__(kFThreads, HY_FLAT_MIN_WAVES) void salamander_flat_kernel(BatchParams B, KeyParams K,
                                                                                  FlatParams F) {
    constexpr int32_t SALT = OBF ? 8 : 0;   // salt bytes in front of the output payload
    constexpr uint32_t SKIP = OBF ? 0u : 8u;   // salt bytes in front of the input payload
    __shared__ __attribute__((aligned(16))) FlatLDS<OBF> S;
    const uint32_t wid = uni32(threadIdx.x >> 6);
    const uint8_t* __restrict__ in = B.in;
    if (blockIdx.x < F.nhash) {   // a hasher workgroup (whole workgroup)
        flat_hasher<OBF, SW>(B, K, F, blockIdx.x, wid);
        return;
    }
    const uint64_t t = blockIdx.x - F.nhash;
    const uint64_t E = uni64(min<uint64_t>(F.cut[0], *F.out_total));   // end of the valid output
    if (t == 0 && threadIdx.x == 0 && B.out_total) atomicAdd(B.out_total, (unsigned long long)E);
    const uint64_t tT = t * kFT;
    if (tT >= E) return;   // past the valid output (whole workgroup)
    const int32_t tl = (int32_t)min<uint64_t>(kFT, E - tT);   // the tile's bytes
    const FlatDesc D0 = F.desc[t];
    const uint64_t d0 = uni64(D0.d), o0 = uni64(D0.o), i0 = uni64(D0.i);
    // the tile's datagrams [d0, dend): the next tile's first one may start in this one
    const uint64_t dend = uni64(tT + kFT < E ? F.desc[t + 1].d + 1 : min<uint64_t>(F.cut[1], B.n));

    // ---- 1. the input window: from the payload byte behind output byte tT (16-aligned
    // down), cut at the input's end (a partial last 16 bytes by single lanes)
    const int64_t first = (int64_t)tT - (int64_t)o0 - SALT;   // payload index of byte tT in d0
    const uint64_t ws = (i0 + SKIP + (uint64_t)max<int64_t>(first, 0)) & ~15ull;
    const uint64_t in_total = uni64(*F.in_total);
    const uint32_t wlen = (uint32_t)min<uint64_t>(flat_stage_bytes<OBF>(), in_total > ws ? in_total - ws : 0);
    {
        const uint32_t lane = threadIdx.x & 63;
        const uint32_t nfull = wlen >> 4;
        for (uint32_t c = wid; c * 64u < nfull; c += kFWaves) {
            const uint32_t ch = c * 64u + lane;
            if (ch < nfull) glds16(in + ws + 16ull * ch, S.stage + kFGuard + 1024u * c);
        }
        const uint32_t tail = wlen & 15u;
        if (tail && wid == kFWaves - 1 && lane < tail) S.stage[kFGuard + 16u * nfull + lane] = in[ws + 16ull * nfull + lane];
    }

    uint8_t* __restrict__ ob = B.out + tT;
    uint64_t og = o0, ig = i0;   // offsets of the pass's first datagram
    for (uint64_t g0 = d0; g0 < dend; g0 += kFD) {
        const uint32_t m = (uint32_t)min<uint64_t>((uint64_t)kFD, dend - g0);
        // the thread index made opaque per pass: values derived from it (the quad's
        // BLAKE2b selects, chunk addresses) are recomputed in each pass, not hoisted out
        // of the (almost always single-trip) loop and spilled
        uint32_t tid = threadIdx.x;
#ifndef HYOBFS_EMULATE
        asm volatile("" : "+v"(tid));
#endif
        const uint32_t lane = tid & 63;
        if (wid == 0) {
            // ---- 2. wave 0: the pass's lengths, widths, offsets, salts and key records
            // (lane l: datagram g0 + l), all loaded in one round trip
            const bool live = lane < m;
            const uint64_t p = g0 + lane;
            const uint32_t L = live ? B.in_len[p] : 0u;
            uint64_t salt = live && OBF ? B.salts[p] : 0ull;
            uint8_t* kb = F.krec + kKeyRec * g0;   // the pass's first record (64 records: one 4 KiB block)
            uint64_t kw[4], tg[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                kw[w] = tg[w] = 0;
                if (live && F.nhash) krec_load(kb, (uint32_t)(kKeyRec * lane + 16 * w), kw[w], tg[w]);
            }
            uint32_t W = live ? out_width<OBF>(L, B.pkt_cap) : 0u;
            // tile-relative 32-bit scans: a pass spans at most 64 x 2^24 bytes
            const uint32_t iw = wave_incl_scan32(W, (int)lane);
            const uint32_t il = wave_incl_scan32(L, (int)lane);
            const uint64_t o = og + iw - W, i = ig + il - L;
            og += uni32((uint32_t)__shfl(iw, 63, 64));
            ig += uni32((uint32_t)__shfl(il, 63, 64));
            if (W && o + W > B.out_cap) W = 0;   // past out_cap: dropped (not in [d0, dend) unless cut)
            const int32_t orel = (int32_t)((int64_t)o - (int64_t)tT);
            const int32_t dlt = (int32_t)((int64_t)(i + SKIP) - (int64_t)ws) - (orel + SALT);
            // ---- keys: the hashers' records; a record not published yet is polled a
            // while, then the wave hashes the pass's keys itself (four lanes per key;
            // at once when the launch has no hashers)
            bool miss = W && (tg[0] != F.epoch || tg[1] != F.epoch || tg[2] != F.epoch || tg[3] != F.epoch);
            const int spins = F.nhash ? 48 : 0;
            for (int spin = 0; spin < spins && __ballot(miss); ++spin) {
#ifndef HYOBFS_EMULATE
                __builtin_amdgcn_s_sleep(8);
#endif
                if (miss) {
                    miss = false;
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        krec_load(kb, (uint32_t)(kKeyRec * lane + 16 * w), kw[w], tg[w]);
                        miss |= tg[w] != F.epoch;
                    }
                }
            }
            if (__ballot(miss)) {   // fallback: quad hashes, 16 keys per pass of the wave
                if (!OBF && W) salt = load8u(in + i);   // the wire's salt
                for (uint32_t k0 = 0; k0 < m; k0 += 16) {
                    const uint32_t k = k0 + (lane >> 2), qi = lane & 3u;
                    const uint64_t x = quad_key<SW>(K, __shfl(salt, (int)(k < 64 ? k : 0), 64), qi);
                    // lane l collects words 0..3 of key l from lanes 4(l - k0) + w
                    const uint32_t src = 4u * ((lane - k0) & 15u);
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const uint64_t y = __shfl(x, (int)(src + (uint32_t)w), 64);
                        if (miss && lane >= k0 && lane < k0 + 16) kw[w] = y;
                    }
                }
            }
            // rotated to the output's 32-byte phase: row byte x = key byte x - (o + SALT) mod 32
            uint64_t kr[4];
            rotl_key_bytes(kw, ((uint32_t)o + (uint32_t)SALT) & 31u, kr);
            // the tile's part of the payload inside the staged window, on the 8-byte grid
            uint32_t fl = 0;
            if (W) {
                const int32_t ps = max(orel + SALT, 0), pe = min(orel + (int32_t)W, (int32_t)kFT);
                if (ps < pe && (ps + dlt < 0 || pe + dlt > (int32_t)wlen)) fl |= kFlatOffWin;
                if (dlt & 7) fl |= kFlatOffGrid;
            }
            S.o[lane] = live ? orel : 0x7FFFFFFF;
            if (lane == 0) S.o[kFD] = 0x7FFFFFFF;
            S.w[lane] = W | fl;
            S.dlt[lane] = dlt;
            S.salt[lane] = salt;
#pragma unroll
            for (int w = 0; w < 4; ++w) S.key[lane][w] = kr[w];
        }
        __syncthreads();   // the stage has landed (every wave's vmcnt(0)), the table and keys are published

        // ---- 3. compose: the chunks inside one payload or across one region edge
        // first, stored together; the rest (gen) by the general merge afterwards, one at
        // a time (its registers are not live beside the four values)
        u128 r[kFU];
        uint32_t gen = 0;   // bit u: chunk u takes the general merge
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
            const int32_t rel = 16 * (int32_t)(u * kFThreads + tid);
            r[u] = 0;
            if (rel >= tl) continue;
            if (!flat_chunk<OBF, kFD>(S, rel, 2u * (((uint32_t)rel >> 4) & 1u), m, r[u])) gen |= 1u << u;
        }
        // ---- store: one non-temporal 16-byte store per chunk, all values finished first
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
            const int32_t rel = 16 * (int32_t)(u * kFThreads + tid);
            if (rel < tl && !((gen >> u) & 1u)) store16_stream(ob + rel, r[u]);
        }
        // ---- the general merge: this pass's datagrams' bytes of the chunk; a chunk it
        // covers in part (the output's last chunk, a chunk shared with the next pass)
        // byte-masked
        while (gen) {
            const int u = __builtin_ctz(gen);
            gen &= gen - 1;
            const int32_t rel = 16 * (int32_t)(u * kFThreads + tid);
            uint32_t q = 0;
            for (uint32_t s = kFD / 2; s; s >>= 1) q = S.o[q + s] <= rel ? q + s : q;
            u128 v = 0;
            uint32_t cov = 0;
            for (uint32_t k = q; k < m && S.o[k] < rel + 16; ++k)
                flat_contrib<OBF>(S, in, ws, wlen, k, rel, ((uint32_t)rel >> 4) & 1u, v, cov);
            if (cov == 0xFFFFu)
                store16_stream(ob + rel, v);
            else if (cov)
                store_masked(ob + rel, v, cov);
        }
        if (g0 + kFD < dend) __syncthreads();   // the next pass overwrites the table and keys
    }
}

template <bool OBF, int SW>
void launch_flat_sw(const BatchParams& b, const KeyParams& k, const FlatParams& F, hipStream_t s) {
    // the hashers, then one workgroup per tile out_cap allows (those past the valid
    // output exit at once; at least one, which writes out_total)
    const uint64_t nt = F.ntiles_max < 1 ? 1 : F.ntiles_max;
    hipLaunchKernelGGL((salamander_flat_kernel<OBF, SW>), dim3((uint32_t)(F.nhash + nt)), dim3(kFThreads), 0, s, b, k,
                       F);
}

}  // namespace hyobfs
