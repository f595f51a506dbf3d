// salamander_flat.h -- the flat kernel: CONTIGUOUS input (datagram i at
// in + in_len[0] + ... + in_len[i-1], include/hyobfs.h) into PACKED output (gfx950).
// The layout of BASELINE configs[2] and of any batch that arrives back to back.
//
// Reference: extras/obfs/salamander.go:59-91 (Obfuscate, Deobfuscate, keyLocked).
//
// The output is cut into tiles of kFT bytes (8 KiB; a tile's lines are written by
// one workgroup only).  Because the input is contiguous, the input bytes behind a
// tile are one contiguous window, known from the tile's first datagram alone:
//   prepass: the width and length sums per 256 datagrams and their scan (shared with
//     the wave kernel, salamander.hip), then flat_locate_kernel: per datagram its
//     output offset and width (the reference's return values, out_off / out_len) and,
//     for every tile whose first byte it holds, the tile's descriptor (the datagram,
//     its output and input offsets);
//   flat kernel, one workgroup of four waves per tile: all waves issue the LDS-DMA of
//     the tile's input window (global_load_lds_dwordx4, non-temporal, 1 KiB per wave
//     instruction) and load the lengths and salts of the tile's datagrams (lane per
//     datagram; every wave scans them for the offsets), wave w hashes the keys of
//     datagrams 16w .. 16w + 15 four lanes per key (quad_key, salamander_tile.h),
//     rotated to the output's 32-byte phase; one barrier; every thread composes its
//     16-byte output chunks from LDS (a chunk is the contributions of the one or two
//     datagrams that touch it: salt bytes, payload bytes XOR the key) and stores each
//     with one non-temporal 16-byte store.
// A tile with more than kFD datagrams takes several passes (its chunks accumulate in
// registers across them); payload bytes outside the staged window (a tile whose input
// span holds long dropped datagrams) are read from global memory.  Both are correct
// and slower; neither happens for input without drops and datagrams >= 128 B on average.
// Applies to contiguous input with packed output and a 16-byte aligned `in`
// (flat_eligible, salamander.hip); the wave kernel takes every other layout.
#pragma once
#include "salamander_tile.h"

namespace hyobfs {

#ifndef HY_FLAT_T
#define HY_FLAT_T 8192
#endif
constexpr uint32_t kFT = HY_FLAT_T;                     // output bytes per tile
static_assert(kFT % 4096 == 0, "a tile is whole 16-byte chunks for 256 threads");
constexpr int kFD = 64;                                 // datagrams per pass
constexpr uint32_t kFStage = kFT + kFT / 8 + 256;       // staged input bytes (deobfuscate: + 8 per datagram)
constexpr uint32_t kFGuard = 32;                        // LDS bytes on both sides of the stage
constexpr int kFU = (int)(kFT / 4096);                  // output chunks per thread
#ifndef HY_FLAT_MIN_WAVES
#define HY_FLAT_MIN_WAVES 5   // 84 VGPRs, no spills (8 waves: 64 VGPRs and 80 B/lane of scratch)
#endif
#ifndef HY_FLAT_ABL
#define HY_FLAT_ABL 0                                   // ablations (wrong output, timing only): 1 hash, 2 compose, 4 DMA
#endif
#ifndef HY_FLAT_LAUNCH_TILES
#define HY_FLAT_LAUNCH_TILES 65536                      // tiles per launch (512 MiB of output)
#endif

struct FlatDesc {       // one output tile: the first valid datagram reaching into it
    uint64_t d;         // its index
    uint64_t o;         // its output offset
    uint64_t i;         // its input offset
};

struct FlatParams {
    FlatDesc* desc;     // ntiles_max entries
    // the first datagram that does not fit out_cap (written by the one wave holding
    // it, ~0 = none): [0] its output offset = the end of the valid output, [1] its index
    uint64_t* cut;
    uint64_t ntiles_max;
    const uint64_t* in_total;    // input bytes: the length scan's total (device)
    const uint64_t* out_total;   // the width scan's total: the valid output's end without a cut
    uint64_t t0;        // first tile of this launch
};

inline uint64_t flat_ntiles_max(uint64_t out_cap) { return (out_cap + kFT - 1) / kFT; }

// Per datagram: width (drop rules), output and input offsets from the scans, the
// reference's return values, and the descriptor of every tile whose first byte the
// datagram holds.  One wave per 256-datagram tile of the scan, four datagrams per lane.
// The valid output ends at the first datagram with a width that does not fit out_cap
// (every later one is dropped too); exactly one wave holds it -- the one whose first
// datagram's offset still fits -- and records it with plain stores (no atomics: one
// word updated by every wave serialised the whole prepass).
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

struct FlatLDS {
    uint8_t stage[kFGuard + kFStage + kFGuard];   // input window, stage byte 0 at stage[kFGuard]
    int32_t o[kFD + 1];                          // output start relative to the tile ([m..] = INT_MAX)
    uint32_t w[kFD];                             // width (0: dropped)
    uint64_t ip[kFD];                            // input position of payload byte 0
    uint64_t salt[kFD];
    u128 key[2 * kFD];                           // key rotated to the output's 32-byte phase, 2 halves
};

// 16 bytes of the stage from stage position q (>= -kFGuard, < kFStage + kFGuard - 16)
__device__ __forceinline__ u128 flat_stage16(const FlatLDS& S, int32_t q) {
    const int32_t a = q + (int32_t)kFGuard;
    const int32_t b = a & ~15;
    const uint32_t sh = (uint32_t)(a & 15);
    const u128 A = *reinterpret_cast<const u128*>(S.stage + b);
    const u128 C = *reinterpret_cast<const u128*>(S.stage + b + 16);
    return sh ? (A >> (8 * sh)) | (C << (128 - 8 * sh)) : A;
}

// Payload bytes [base, base + 16) of the datagram whose payload is the PL bytes at
// input position ip, of which the caller keeps [.., need) (the rest is garbage,
// masked): from the stage when the window holds the kept bytes (never below ws: the
// tile's payload bytes start there), else one in-bounds global load.
__device__ __forceinline__ u128 flat_payload16(const FlatLDS& S, const uint8_t* __restrict__ in, uint64_t ws,
                                               uint64_t wend, uint64_t ip, uint32_t PL, int32_t base, int32_t need) {
    const int64_t pos = (int64_t)ip + base;
    if (pos >= (int64_t)ws - 16 && pos + need <= (int64_t)wend) return flat_stage16(S, (int32_t)(pos - (int64_t)ws));
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

// Everything datagram k of the table contributes to the chunk at tile-relative rel.
template <bool OBF>
__device__ __forceinline__ void flat_contrib(const FlatLDS& S, const uint8_t* __restrict__ in, uint64_t ws, uint64_t wend,
                                             uint32_t k, int32_t rel, u128& r, uint32_t& cov) {
    constexpr int32_t SALT = OBF ? 8 : 0;
    const uint32_t W = S.w[k];
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
        const u128 X = flat_payload16(S, in, ws, wend, S.ip[k], W - (uint32_t)SALT, rel - (o + SALT), pe - rel);
        r |= (X ^ S.key[2 * k + (((uint32_t)rel >> 4) & 1u)]) & bytemask((uint32_t)(ps - rel), (uint32_t)(pe - rel));
        cov |= ((1u << (pe - ps)) - 1u) << (ps - rel);
    }
}

template <bool OBF, int SW>
__global__ __launch_bounds__(256, HY_FLAT_MIN_WAVES) void salamander_flat_kernel(BatchParams B, KeyParams K,
                                                                                  FlatParams F) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;   // salt bytes in front of the output payload
    constexpr uint32_t SKIP = OBF ? 0u : 8u;   // salt bytes in front of the input payload
    __shared__ __attribute__((aligned(16))) FlatLDS S;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = uni32(tid >> 6);
    const uint8_t* __restrict__ in = B.in;
    const uint64_t t = F.t0 + blockIdx.x;
    const uint64_t E = uni64(min<uint64_t>(F.cut[0], *F.out_total));   // end of the valid output
    if (t == 0 && tid == 0 && B.out_total) *B.out_total = E;
    const uint64_t tT = t * kFT;
    if (tT >= E) return;   // past the valid output
    const int32_t tl = (int32_t)min<uint64_t>(kFT, E - tT);   // the tile's bytes
    const FlatDesc D0 = F.desc[t];
    const uint64_t d0 = uni64(D0.d), o0 = uni64(D0.o), i0 = uni64(D0.i);
    // the tile's datagrams [d0, d1]: the next tile's first one may start here too
    const uint64_t d1 = uni64(tT + kFT < E ? F.desc[t + 1].d : min<uint64_t>(F.cut[1], B.n) - 1);

    // ---- the input window: from the payload byte behind output byte tT (16-aligned
    // down), kFStage bytes, cut at the input's end (a partial last 16 bytes by one lane)
    const int64_t first = (int64_t)tT - (int64_t)o0 - (int64_t)SALT;   // payload index of byte tT in d0
    const uint64_t ws = (i0 + SKIP + (uint64_t)max<int64_t>(first, 0)) & ~15ull;
    const uint64_t wend = min<uint64_t>(ws + kFStage, uni64(*F.in_total));
    {
        const uint32_t nfull = (uint32_t)((wend - ws) >> 4);
        for (uint32_t c = wid; c * 64u < nfull && !(HY_FLAT_ABL & 4); c += 4) {
            const uint32_t ch = c * 64u + lane;
            if (ch < nfull) glds16(in + ws + 16ull * ch, S.stage + kFGuard + 1024u * c);
        }
        const uint32_t tail = (uint32_t)((wend - ws) & 15);
        if (tail && wid == 3 && lane < tail) S.stage[kFGuard + 16u * nfull + lane] = in[ws + 16ull * nfull + lane];
    }

    u128 r[kFU];
    uint32_t cov[kFU];
#pragma unroll
    for (int u = 0; u < kFU; ++u) {
        r[u] = 0;
        cov[u] = 0;
    }
    uint64_t og = o0, ig = i0;   // offsets of the pass's first datagram
    for (uint64_t g0 = d0; g0 <= d1; g0 += kFD) {
        const uint32_t m = (uint32_t)min<uint64_t>((uint64_t)kFD, d1 - g0 + 1);
        // ---- every wave: the pass's lengths, widths and offsets (lane l: datagram g0 + l)
        const bool live = lane < m;
        const uint64_t p = g0 + lane;
        const uint32_t L = live ? B.in_len[p] : 0u;
        uint32_t W = live ? out_width<OBF>(L, B.pkt_cap) : 0u;
        const uint64_t iw = wave_incl_scan((uint64_t)W, (int)lane), il = wave_incl_scan((uint64_t)L, (int)lane);
        const uint64_t o = og + iw - W, i = ig + il - L;
        og += uni64(__shfl(iw, 63, 64));
        ig += uni64(__shfl(il, 63, 64));
        if (W && o + W > B.out_cap) W = 0;   // past out_cap: dropped
        if (wid == 0) {
            S.o[lane] = live ? (int32_t)((int64_t)o - (int64_t)tT) : 0x7FFFFFFF;
            if (lane == 0) S.o[kFD] = 0x7FFFFFFF;
            S.w[lane] = W;
            S.ip[lane] = i + SKIP;
        }
        // ---- keys: wave w hashes datagrams 16w .. 16w + 15, four lanes each
        if (16u * wid < m) {
            const uint32_t k = 16u * wid + (lane >> 2), qi = lane & 3u;
            const uint32_t kk = k < m ? k : 16u * wid;
            uint64_t salt;
            if (OBF) {
                salt = B.salts[g0 + kk];
            } else {   // the wire's salt: the datagram's first 8 bytes
                const uint64_t ik = __shfl(i, (int)kk, 64);
                const uint32_t Wk = __shfl(W, (int)kk, 64);
                salt = Wk ? load8u(in + ik) : 0ull;
            }
            const uint64_t ok = __shfl(o, (int)kk, 64);
#if HY_FLAT_ABL & 1
            const uint64_t kw = salt ^ qi;
#else
            const uint64_t kw = quad_key<SW>(K, salt, qi);
#endif
            const uint32_t rr = ((uint32_t)ok + SALT) & 31u;
            const uint32_t st = (8u * qi - rr) & 31u, w0 = st >> 3, sh = (st & 7u) * 8u;
            const uint64_t a = __shfl(kw, (int)((lane & ~3u) | w0), 64);
            const uint64_t b = __shfl(kw, (int)((lane & ~3u) | ((w0 + 1) & 3u)), 64);
            if (k < m) {
                reinterpret_cast<uint64_t*>(S.key)[4 * k + qi] = sh ? (a >> sh) | (b << (64 - sh)) : a;
                if (qi == 0) S.salt[k] = salt;
            }
        }
        __syncthreads();   // the stage has landed (every wave's vmcnt(0)), the table and keys are published

        // ---- compose: the one or two datagrams touching each chunk (more: a loop)
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
            const int32_t rel = 16 * (int32_t)(u * 256 + tid);
            if (rel >= tl) continue;
#if HY_FLAT_ABL & 2
            r[u] = flat_stage16(S, rel) ^ S.key[tid & 127];
            cov[u] = 0xFFFFu;
            continue;
#endif
            uint32_t q = 0;   // last datagram whose output starts at or before rel
#pragma unroll
            for (uint32_t s = kFD / 2; s; s >>= 1) q = S.o[q + s] <= rel ? q + s : q;
            flat_contrib<OBF>(S, in, ws, wend, q, rel, r[u], cov[u]);
            for (uint32_t k = q + 1; k < m && S.o[k] < rel + 16; ++k) flat_contrib<OBF>(S, in, ws, wend, k, rel, r[u], cov[u]);
        }
        if (g0 + kFD <= d1) __syncthreads();   // the next pass overwrites the table and keys
    }

    // ---- store: whole chunks in one non-temporal 16-byte store, the last one masked
    uint8_t* __restrict__ ob = B.out + tT;
#pragma unroll
    for (int u = 0; u < kFU; ++u) {
        const int32_t rel = 16 * (int32_t)(u * 256 + tid);
        if (cov[u] == 0xFFFFu)
            store16_stream(ob + rel, r[u]);
        else if (cov[u])
            store_masked(ob + rel, r[u], cov[u]);
    }
}

// The prepass's scratch: the descriptor of every tile out_cap allows, two header words.
inline uint64_t flat_workspace_bytes(uint64_t out_cap) { return 16 + sizeof(FlatDesc) * (flat_ntiles_max(out_cap) + 1); }

template <bool OBF, int SW>
void launch_flat_sw(const BatchParams& b, const KeyParams& k, const FlatParams& F, hipStream_t s) {
    // one workgroup per tile out_cap allows (those past the valid output exit at once);
    // at least one, which writes out_total
    const uint64_t nt = F.ntiles_max < 1 ? 1 : F.ntiles_max;
    for (uint64_t t0 = 0; t0 < nt; t0 += HY_FLAT_LAUNCH_TILES) {
        FlatParams Fl = F;
        Fl.t0 = t0;
        const uint64_t g = nt - t0 < (uint64_t)HY_FLAT_LAUNCH_TILES ? nt - t0 : (uint64_t)HY_FLAT_LAUNCH_TILES;
        hipLaunchKernelGGL((salamander_flat_kernel<OBF, SW>), dim3((uint32_t)g), dim3(256), 0, s, b, k, Fl);
    }
}

}  // namespace hyobfs
