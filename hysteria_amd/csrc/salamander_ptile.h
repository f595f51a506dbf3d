// salamander_ptile.h -- the packed tile kernel: ragged batches with packed output
// (gfx950).  BASELINE configs[2] (40 % 64 B / 60 % 1350 B, packed) runs here.
//
// Reference: extras/obfs/salamander.go:59-91 (Obfuscate, Deobfuscate, keyLocked).
//
// The salamander_tile.h design for any lengths and alignments.  A workgroup of
// four waves owns a tile of 16 consecutive datagrams and exits when done:
//   1. every wave reads the tile's lengths and input offsets; waves 1-3 copy the
//      16-byte blocks holding each datagram's input into LDS with LDS-DMA
//      (global_load_lds_dwordx4, non-temporal), back to back;
//   2. wave 0 meanwhile derives the tile's output offset (the scan's tile prefix
//      plus the widths of the scan tile's earlier datagrams), the widths and
//      drop rules (salamander.go:60-62, :75-77), loads the 16 salts and hashes the
//      16 keys on quads (salamander_tile.h quad_key), all into LDS;
//   3. after one barrier, all four waves sweep the tile's output range in 16-byte
//      chunks on the global 16-byte grid, 1 KiB per wave instruction: a chunk
//      inside one payload is one unaligned 16-byte LDS read of the staged input,
//      one of the key (stored twice in a row, so any 16 key bytes are contiguous),
//      an XOR and a store;
//   4. then each datagram's two or three other chunks (salt, edges) are merged by
//      one thread each, every datagram touching the chunk under byte masks.  The
//      first and last chunks of a tile are shared with the neighbouring tiles:
//      masked stores.
// A tile whose staged input would not fit the LDS budget (datagrams of more than
// ~1.2 KiB on average) reads its inputs from global memory in the same compose
// step instead (16-byte windows, as the wave kernel does).
#pragma once
#include "salamander_tile.h"

namespace hyobfs {

#ifndef HY_PT_LDS
#define HY_PT_LDS 20480          // staged input bytes per tile (dynamic LDS): 7 workgroups per CU
#endif
#ifndef HY_PT_U
#define HY_PT_U 5                // output chunks per thread and compose pass
#endif
#ifndef HY_PT_MIN_WAVES
#define HY_PT_MIN_WAVES 7
#endif
constexpr uint32_t kPtSlack = 32;   // LDS bytes in front of the staged input (windows may start before it)

struct PtMeta {                     // the tile's datagrams (wave 0 writes, everyone reads after the barrier)
    uint32_t os[kTileMaxD + 1];     // output region start relative to the tile's first region; [nt] = end
    uint32_t w[kTileMaxD];          // output width, 0 = dropped
    uint32_t src[kTileMaxD];        // staged: LDS offset of input byte 0
    uint64_t io[kTileMaxD];         // direct: input offset (bytes from B.in)
    uint64_t base;                  // absolute output offset of the tile's first region
    uint32_t staged;                // 1: inputs staged in LDS
};

// Bytes of datagram k in the 16-byte output chunk whose first byte is at
// tile-relative output offset a (salt, payload XOR key), merged into r / cov.
template <bool OBF>
__device__ __forceinline__ void pt_contrib(const BatchParams& B, const PtMeta& M, const uint8_t* s_in,
                                           const uint8_t* s_keyb, const uint64_t* s_salt, uint32_t k, int32_t a,
                                           u128& r, uint32_t& cov) {
    constexpr int32_t SALT = OBF ? 8 : 0;
    constexpr uint32_t SKIP = OBF ? 0u : 8u;
    const int32_t os = (int32_t)M.os[k], W = (int32_t)M.w[k];
    if (W == 0 || os + W <= a || os >= a + 16) return;
    if (OBF) {   // salt bytes [os, os + 8)
        const int32_t sb = max(os, a), se = min(os + 8, a + 16);
        if (sb < se) {
            u128 S = (u128)s_salt[k];
            S = os >= a ? (S << (8 * (os - a))) : (S >> (8 * (a - os)));
            r |= S & bytemask((uint32_t)(sb - a), (uint32_t)(se - a));
            cov |= ((1u << (se - sb)) - 1u) << (sb - a);
        }
    }
    const int32_t ps = max(os + SALT, a), pe = min(os + W, a + 16);
    if (ps >= pe) return;
    const int32_t jb = a - os - SALT;   // payload index of chunk byte 0 (may be negative)
    u128 V;
    if (M.staged) {
        __builtin_memcpy(&V, s_in + (int32_t)(M.src[k] + SKIP) + jb, 16);   // unaligned LDS read
    } else {   // one in-bounds 16-byte window of the payload (or bytes), shifted into place
        const int32_t PL = W - SALT;
        const uint8_t* g = B.in + M.io[k] + SKIP;
        if (PL >= 16) {
            const int32_t ws = min(max(jb, 0), PL - 16), d = ws - jb;
            const u128 X = load16u(g + ws);
            V = d >= 0 ? (X << (8 * d)) : (X >> (8 * -d));
        } else {
            V = 0;
            for (int32_t j = ps - a; j < pe - a; ++j) V |= (u128)g[jb + j] << (8 * j);
        }
    }
    u128 Kb;   // key bytes for payload indices jb .. jb + 15 (the key stored twice: 64 bytes)
    __builtin_memcpy(&Kb, s_keyb + 64 * k + (uint32_t)(jb & 31), 16);
    r |= (V ^ Kb) & bytemask((uint32_t)(ps - a), (uint32_t)(pe - a));
    cov |= ((1u << (pe - ps)) - 1u) << (ps - a);
}

template <bool OBF, int SW>
__global__ __launch_bounds__(256, HY_PT_MIN_WAVES) void salamander_ptile_kernel(BatchParams B, KeyParams K) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;
#ifdef HYOBFS_EMULATE
    uint8_t* s_in = hyemu_dyn_lds();
#else
    extern __shared__ __attribute__((aligned(16))) uint8_t s_in[];   // kPtSlack + HY_PT_LDS + kPtSlack
#endif
    __shared__ uint64_t s_key[kTileMaxD * 8];   // each key twice in a row
    __shared__ uint64_t s_salt[kTileMaxD];
    __shared__ PtMeta M;
    constexpr int U = HY_PT_U;

    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = uni32(tid >> 6);
    const uint64_t p0 = (uint64_t)blockIdx.x * kTileMaxD;
    const uint32_t nt = (uint32_t)min<uint64_t>((uint64_t)kTileMaxD, B.n - p0);

    // ---- every wave: the tile's lengths, widths, input blocks (lanes 0..15)
    const bool mine = lane < nt;
    const uint64_t p = p0 + lane;
    const uint32_t L = mine ? pkt_len(B, p) : 0u;
    const uint64_t io = mine ? pkt_in_off(B, p) : 0ull;
    const uint32_t W0 = mine ? out_width<OBF>(L, B.pkt_cap) : 0u;   // the scan's width (before out_cap)
    const uint32_t os_incl = (uint32_t)wave_incl_scan(W0, (int)lane);
    const uint32_t os = os_incl - W0;
    const uint32_t total = uni32(__shfl(os_incl, 63, 64));
    // input blocks on the absolute 16-byte grid: [ga >> 4, (ga + L + 15) >> 4)
    const uintptr_t ga = reinterpret_cast<uintptr_t>(B.in) + io;
    const uint32_t nb = (W0 && L) ? (uint32_t)(((ga + L + 15) >> 4) - (ga >> 4)) : 0u;
    const uint32_t nb_incl = (uint32_t)wave_incl_scan(nb, (int)lane);
    const uint32_t bstart = nb_incl - nb;
    const uint32_t NB = uni32(__shfl(nb_incl, 63, 64));
    const bool staged = 16u * NB <= (uint32_t)HY_PT_LDS;

    if (wid == 0) {
        // ---- keys on quads: lane 4k+i holds word i of datagram k's key.  The salt and
        // offset loads are issued together, before the hash.
        const uint32_t qk = lane >> 2, qi = lane & 3;
        const uint64_t ioq = __shfl(io, (int)qk, 64);
        const uint32_t Wq = __shfl(W0, (int)qk, 64);
        uint64_t salt = 0;
        if (qk < nt && (OBF || Wq)) salt = OBF ? B.salts[p0 + qk] : load8u(B.in + ioq);   // the wire's salt
        // output offset of the tile: its scan tile's prefix plus its offset inside it
        const uint64_t base = uni64(B.tile_prefix[p0 / kTile] + B.sub_prefix[p0 / kTileMaxD]);
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
        // drops: a region past out_cap is dropped, offsets unchanged (include/hyobfs.h)
        const uint32_t W = (W0 && base + os + W0 <= B.out_cap) ? W0 : 0u;
        if (mine) {
            M.os[lane] = os;
            M.w[lane] = W;
            M.src[lane] = kPtSlack + 16u * bstart + (uint32_t)(ga & 15);
            M.io[lane] = io;
            if (B.out_off) B.out_off[p] = base + os;
            if (B.out_len) B.out_len[p] = W;
        }
        if (lane == 0) {
            M.os[nt] = total;
            M.base = base;
            M.staged = staged ? 1u : 0u;
        }
        if (B.out_total) {
            const uint64_t written = uni64(wave_sum(W));
            if (lane == 0 && written) atomicAdd(B.out_total, (unsigned long long)written);
        }
    } else if (staged) {
        // ---- waves 1-3: the datagrams' input blocks into LDS, 1 KiB per instruction.
        // Block b belongs to the last datagram whose first block is <= b (block starts
        // in scalar registers, no LDS round trips); its global block is b + delta.
        const uint64_t dlt = (uint64_t)(ga >> 4) - bstart;
        uint32_t bsd[kTileMaxD];
        uint64_t dd[kTileMaxD];
#pragma unroll
        for (int d = 0; d < (int)kTileMaxD; ++d) {
            bsd[d] = (uint32_t)__builtin_amdgcn_readlane((int)bstart, d);
            dd[d] = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)dlt, d) |
                    (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(dlt >> 32), d) << 32;
        }
        for (uint32_t i = wid - 1; i * 64u < NB; i += 3) {
            const uint32_t b = i * 64u + lane;
            uint64_t delta = dd[0];
#pragma unroll
            for (int d = 1; d < (int)kTileMaxD; ++d)
                if (bsd[d] <= b) delta = dd[d];
            if (b < NB) glds16(reinterpret_cast<const uint8_t*>((b + delta) << 4), s_in + kPtSlack + 1024u * i);
        }
    }
    __syncthreads();   // every wave's LDS-DMA has landed (vmcnt(0)); keys and metadata are published

    // ---- every thread: compose the tile's output range on the global 16-byte grid
    const uint64_t base = M.base;
    const uint32_t tend = M.os[nt];
    if (tend == 0) return;
    const uint32_t head = (uint32_t)(base & 15);   // bytes of the first chunk before the tile
    const uint32_t nch = (head + tend + 15) >> 4;
    uint8_t* __restrict__ ob = B.out + (base - head);
    const uint8_t* s_keyb = reinterpret_cast<const uint8_t*>(s_key);
    // region starts in registers (lane d: datagram d, past nt: never reached)
    const int32_t osl = lane < nt ? (int32_t)M.os[lane] : 0x7fffffff;
    int32_t osd[kTileMaxD];
#pragma unroll
    for (int d = 1; d < (int)kTileMaxD; ++d) osd[d] = __builtin_amdgcn_readlane(osl, d);
    // ---- sweep: the chunks inside one payload (every lane on the same path)
    const bool stg = M.staged != 0;
    for (uint32_t c0 = 0; c0 < nch; c0 += 256u * U) {
        u128 r[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + (uint32_t)u * 256u + tid;
            const int32_t a = (int32_t)(16u * c) - (int32_t)head;   // tile-relative offset of chunk byte 0
            uint32_t k = 0;   // the last datagram whose region starts at or before a
#pragma unroll
            for (int d = 1; d < (int)kTileMaxD; ++d) k += osd[d] <= a ? 1u : 0u;
            const int32_t os = (int32_t)M.os[k], W = (int32_t)M.w[k];
            ok[u] = c < nch && W && os + (int32_t)SALT <= a && a + 16 <= os + W;
            r[u] = 0;
            if (ok[u]) {
                const int32_t jb = a - os - (int32_t)SALT;
                u128 V, Kb;
                if (stg)
                    __builtin_memcpy(&V, s_in + (int32_t)(M.src[k] + (OBF ? 0u : 8u)) + jb, 16);
                else
                    V = load16u(B.in + M.io[k] + (OBF ? 0u : 8u) + (uint32_t)jb);
                __builtin_memcpy(&Kb, s_keyb + 64 * k + (uint32_t)(jb & 31), 16);
                r[u] = V ^ Kb;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) {
                const uint32_t c = c0 + (uint32_t)u * 256u + tid;
                store16_global(ob + 16u * c, (uint64_t)r[u], (uint64_t)(r[u] >> 64));
            }
    }
    // ---- edges: a region's other chunks are its first, the one holding its last salt
    // byte (obfuscate) and its last.  Thread e takes candidate e % NC of datagram e / NC;
    // the first region touching a chunk merges every region touching it.  (Merging
    // inside the sweep made every wave instruction run the merge for a few lanes.)
    constexpr uint32_t NC = OBF ? 3u : 2u;
    if (tid < NC * nt) {
        const uint32_t v = tid / NC, w = tid % NC;
        const int32_t os = (int32_t)M.os[v], W = (int32_t)M.w[v];
        auto cand = [&](uint32_t i) -> int32_t {   // chunk index on the tile's grid
            const int32_t x = i == 0 ? os : (i == NC - 1 ? os + W - 1 : os + 7);
            return (x + (int32_t)head) >> 4;
        };
        const int32_t c = cand(w), a = 16 * c - (int32_t)head;
        bool skip = W == 0 || (w > 0 && cand(0) == c) || (w == 2 && cand(1) == c) ||
                    (os + (int32_t)SALT <= a && a + 16 <= os + W);   // inside the payload: the sweep's
        // an earlier region reaching into the chunk owns it (regions are back to back:
        // region u ends at or before os[u + 1])
        for (int32_t u = (int32_t)v - 1; !skip && u >= 0 && (int32_t)M.os[u + 1] > a; --u)
            skip = M.w[u] && (int32_t)(M.os[u] + M.w[u]) > a;
        if (!skip) {
            u128 r = 0;
            uint32_t cov = 0;
            for (uint32_t kk = v; kk < nt && (int32_t)M.os[kk] < a + 16; ++kk)
                pt_contrib<OBF>(B, M, s_in, s_keyb, s_salt, kk, a, r, cov);
            if (cov == 0xFFFFu)
                store16_global(ob + 16 * c, (uint64_t)r, (uint64_t)(r >> 64));
            else if (cov)
                store_masked(ob + 16 * c, r, cov);
        }
    }
}

// The packed tile kernel: every packed batch (the scan's tile prefix is in
// B.tile_prefix).  Tile-local offsets are 32-bit: a tile's 16 regions span less
// than 2^31 bytes (kMaxDatagram = 16 MiB).
template <bool OBF, int SW>
void launch_ptile_sw(const BatchParams& b, const KeyParams& k, hipStream_t s) {
    const uint64_t blocks = div_up(b.n, kTileMaxD);
    hipLaunchKernelGGL((salamander_ptile_kernel<OBF, SW>), dim3((uint32_t)blocks), dim3(256),
                       kPtSlack + HY_PT_LDS + kPtSlack, s, b, k);
}

}  // namespace hyobfs
