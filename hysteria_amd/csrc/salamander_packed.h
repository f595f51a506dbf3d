// salamander_packed.h -- the pipelined packed kernel: ragged batches with packed
// output (gfx950).  BASELINE configs[2] (40 % 64 B / 60 % 1350 B, packed).
//
// Reference: extras/obfs/salamander.go:59-91 (Obfuscate, Deobfuscate, keyLocked).
//
// Persistent workgroups of four waves walk tiles of 16 consecutive datagrams
// (tile t, t + G, t + 2G, ... for grid size G, so the resident workgroups sweep
// neighbouring addresses).  Per tile:
//   1. wave 0 holds the tile's lengths, input offsets, salts and output offset in
//      registers, loaded during the previous tile.  It derives widths, drops and
//      the input's 16-byte blocks, issues the LDS-DMA of every block
//      (global_load_lds_dwordx4, non-temporal), issues the NEXT tile's loads, and
//      hashes the 16 keys on quads (salamander_tile.h quad_key) while both are in
//      flight; then it publishes keys and metadata to LDS and waits for its DMA;
//   2. one barrier; all four waves sweep the tile's output range in 16-byte chunks
//      on the global 16-byte grid (a chunk inside one payload: one unaligned LDS read
//      of the staged input, one of the key stored twice in a row, an XOR, a store);
//      then each datagram's two or three other chunks (salt, edges) are merged by one
//      thread each under byte masks; a second barrier frees the LDS.
// So one tile costs one exposed HBM round trip (its DMA, overlapped with the hash)
// instead of the one-shot tile's two plus the key wave (the one-shot
// packed tile kernel was latency-bound at 13 us per tile).  A tile whose input would
// not fit the LDS budget reads its inputs from global memory in the same sweep.
#pragma once
#include "salamander_tile.h"

namespace hyobfs {

#ifndef HY_PK_LDS
#define HY_PK_LDS 20480          // staged input bytes per tile (dynamic LDS)
#endif
#ifndef HY_PK_U
#define HY_PK_U 5                // output chunks per thread and sweep pass
#endif
#ifndef HY_PK_MIN_WAVES
#define HY_PK_MIN_WAVES 7
#endif
constexpr uint32_t kPkSlack = 32;   // LDS bytes in front of the staged input (windows may start before it)

struct PkMeta {                     // the tile's datagrams (wave 0 writes, everyone reads after the barrier)
    uint32_t os[kTileMaxD + 1];     // output region start relative to the tile's first region; [nt] = end
    uint32_t w[kTileMaxD];          // output width, 0 = dropped
    uint32_t src[kTileMaxD];        // staged: LDS offset of input byte 0
    uint64_t io[kTileMaxD];         // direct: input offset (bytes from B.in)
    uint64_t base;                  // absolute output offset of the tile's first region
    uint32_t nt;                    // datagrams in the tile
    uint32_t staged;                // 1: inputs staged in LDS
};

// Bytes of datagram k in the 16-byte output chunk whose first byte is at
// tile-relative output offset a (salt, payload XOR key), merged into r / cov.
template <bool OBF>
__device__ __forceinline__ void pk_contrib(const BatchParams& B, const PkMeta& M, const uint8_t* s_in,
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

__device__ __forceinline__ void pk_wait_vm() {   // this wave's vector memory operations (incl. LDS-DMA) done
#ifndef HYOBFS_EMULATE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}

// One tile's registers in wave 0: lane k < 16 the length and input offset of
// datagram k, quad k (lanes 4k..4k+3) its salt, every lane the tile's output offset.
struct PkRegs {
    uint32_t L;
    uint64_t io, salt, base;
};

template <bool OBF>
__device__ __forceinline__ void pk_load(const BatchParams& B, uint64_t t, uint32_t lane, PkRegs& R) {
    const uint64_t p0 = t * kTileMaxD;
    const uint32_t nt = (uint32_t)min<uint64_t>((uint64_t)kTileMaxD, B.n - p0);
    R.L = lane < nt ? pkt_len(B, p0 + lane) : 0u;
    R.io = lane < nt ? pkt_in_off(B, p0 + lane) : 0ull;
    R.salt = 0;
    if (OBF && (lane >> 2) < nt) R.salt = B.salts[p0 + (lane >> 2)];
    R.base = B.tile_prefix[p0 / kTile] + B.sub_prefix[t];
}

// Deobfuscate: the salt is the wire's first 8 bytes, loaded once the offsets are in.
template <bool OBF>
__device__ __forceinline__ void pk_load_salt(const BatchParams& B, uint64_t t, uint32_t lane, PkRegs& R) {
    if (OBF) return;
    const uint64_t p0 = t * kTileMaxD;
    const uint32_t nt = (uint32_t)min<uint64_t>((uint64_t)kTileMaxD, B.n - p0);
    const uint32_t qk = lane >> 2;
    const uint32_t Lq = __shfl(R.L, (int)qk, 64);
    const uint64_t ioq = __shfl(R.io, (int)qk, 64);
    if (qk < nt && out_width<false>(Lq, B.pkt_cap)) R.salt = load8u(B.in + ioq);
}

template <bool OBF, int SW>
__global__ __launch_bounds__(256, HY_PK_MIN_WAVES) void salamander_packed_kernel(BatchParams B, KeyParams K) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;
#ifdef HYOBFS_EMULATE
    uint8_t* s_in = hyemu_dyn_lds();
#else
    extern __shared__ __attribute__((aligned(16))) uint8_t s_in[];   // kPkSlack + HY_PK_LDS + kPkSlack
#endif
    __shared__ uint64_t s_key[kTileMaxD * 8];   // each key twice in a row
    __shared__ uint64_t s_salt[kTileMaxD];
    __shared__ PkMeta M;
    constexpr int U = HY_PK_U;

    const uint32_t wid = uni32(threadIdx.x >> 6);
    const uint64_t ntiles = (B.n + kTileMaxD - 1) / kTileMaxD;
    const uint8_t* s_keyb = reinterpret_cast<const uint8_t*>(s_key);

    PkRegs R{};
    if (wid == 0 && blockIdx.x < ntiles) {   // the first tile's registers
        pk_load<OBF>(B, blockIdx.x, threadIdx.x & 63, R);
        pk_load_salt<OBF>(B, blockIdx.x, threadIdx.x & 63, R);
    }
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        // lane-derived values are rebuilt per tile: hoisted out of the loop, the
        // per-lane addresses of every phase stay live across it and spill
        uint32_t tid = threadIdx.x;
#ifndef HYOBFS_EMULATE
        asm volatile("" : "+v"(tid));
#endif
        const uint32_t lane = tid & 63;
        if (wid == 0) {
            const uint64_t p0 = t * kTileMaxD;
            const uint32_t nt = (uint32_t)min<uint64_t>((uint64_t)kTileMaxD, B.n - p0);
            const bool mine = lane < nt;
            const uint32_t L = R.L;
            const uint64_t io = R.io;
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
            const bool staged = 16u * NB <= (uint32_t)HY_PK_LDS;
            // drops: a region past out_cap is dropped, offsets unchanged (include/hyobfs.h)
            const uint64_t base = uni64(R.base);
            const uint32_t W = (W0 && base + os + W0 <= B.out_cap) ? W0 : 0u;
            if (mine) {
                M.os[lane] = os;
                M.w[lane] = W;
                M.src[lane] = kPkSlack + 16u * bstart + (uint32_t)(ga & 15);
                M.io[lane] = io;
                if (B.out_off) B.out_off[p0 + lane] = base + os;
                if (B.out_len) B.out_len[p0 + lane] = W;
            }
            if (lane == 0) {
                M.os[nt] = total;
                M.base = base;
                M.nt = nt;
                M.staged = staged ? 1u : 0u;
            }
            if (B.out_total) {
                const uint64_t written = uni64(wave_sum(W));
                if (lane == 0 && written) atomicAdd(B.out_total, (unsigned long long)written);
            }
            if (staged) {   // ---- the tile's input blocks into LDS, 1 KiB per instruction
                // block b belongs to the last datagram whose first block is <= b (block
                // starts in scalar registers); its global block is b + delta
                const uint64_t dlt = (uint64_t)(ga >> 4) - bstart;
                uint32_t bsd[kTileMaxD];
#pragma unroll
                for (int d = 1; d < (int)kTileMaxD; ++d) bsd[d] = (uint32_t)__builtin_amdgcn_readlane((int)bstart, d);
                for (uint32_t i = 0; i * 64u < NB; ++i) {
                    const uint32_t b = i * 64u + lane;
                    uint32_t q = 0;
#pragma unroll
                    for (int d = 1; d < (int)kTileMaxD; ++d) q += bsd[d] <= b ? 1u : 0u;
                    const uint64_t delta = __shfl((unsigned long long)dlt, (int)q, 64);
                    if (b < NB)
                        glds16(reinterpret_cast<const uint8_t*>((b + delta) << 4), s_in + kPkSlack + 1024u * i);
                }
            }
            // ---- the next tile's registers, in flight during the hash
            const uint64_t tn = t + gridDim.x;
            PkRegs N{};
            if (tn < ntiles) pk_load<OBF>(B, tn, lane, N);
            // ---- keys on quads: lane 4k+i holds word i of datagram k's key
            const uint32_t qk = lane >> 2, qi = lane & 3;
            const uint64_t salt = R.salt;
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
            if (tn < ntiles) pk_load_salt<OBF>(B, tn, lane, N);
            R = N;
            pk_wait_vm();   // the DMA has landed in LDS (and the next tile's registers are in)
        }
        hy_lds_barrier();   // staged input, keys and metadata visible to every wave

        // ---- every thread: the tile's output range on the global 16-byte grid
        const uint32_t nt = M.nt;
        const uint64_t base = M.base;
        const uint32_t tend = M.os[nt];
        const uint32_t head = (uint32_t)(base & 15);   // bytes of the first chunk before the tile
        const uint32_t nch = tend ? (head + tend + 15) >> 4 : 0u;
        uint8_t* __restrict__ ob = B.out + (base - head);
        // region starts in registers (lane d: datagram d, past nt: never reached)
        const int32_t osl = lane < nt ? (int32_t)M.os[lane] : 0x7fffffff;
        int32_t osd[kTileMaxD];
#pragma unroll
        for (int d = 1; d < (int)kTileMaxD; ++d) osd[d] = __builtin_amdgcn_readlane(osl, d);
        // sweep: the chunks inside one payload (every lane on the same path)
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
        // edges: a region's other chunks are its first, the one holding its last salt
        // byte (obfuscate) and its last.  Thread e takes candidate e % NC of datagram
        // e / NC; the first region touching a chunk merges every region touching it.
        constexpr uint32_t NC = OBF ? 3u : 2u;
        if (tend && tid < NC * nt) {
            const uint32_t v = tid / NC, w = tid % NC;
            const int32_t os = (int32_t)M.os[v], W = (int32_t)M.w[v];
            auto cand = [&](uint32_t i) -> int32_t {   // chunk index on the tile's grid
                const int32_t x = i == 0 ? os : (i == NC - 1 ? os + W - 1 : os + 7);
                return (x + (int32_t)head) >> 4;
            };
            const int32_t c = cand(w), a = 16 * c - (int32_t)head;
            bool skip = W == 0 || (w > 0 && cand(0) == c) || (w == 2 && cand(1) == c) ||
                        (os + (int32_t)SALT <= a && a + 16 <= os + W);   // inside the payload: the sweep's
            // an earlier region reaching into the chunk owns it (regions are back to
            // back: region u ends at or before os[u + 1])
            for (int32_t u = (int32_t)v - 1; !skip && u >= 0 && (int32_t)M.os[u + 1] > a; --u)
                skip = M.w[u] && (int32_t)(M.os[u] + M.w[u]) > a;
            if (!skip) {
                u128 r = 0;
                uint32_t cov = 0;
                for (uint32_t kk = v; kk < nt && (int32_t)M.os[kk] < a + 16; ++kk)
                    pk_contrib<OBF>(B, M, s_in, s_keyb, s_salt, kk, a, r, cov);
                if (cov == 0xFFFFu)
                    store16_global(ob + 16 * c, (uint64_t)r, (uint64_t)(r >> 64));
                else if (cov)
                    store_masked(ob + 16 * c, r, cov);
            }
        }
        hy_lds_barrier();   // every wave is done with this tile's LDS
    }
}

// The pipelined packed kernel (opt-in, HYOBFS_KERNEL=packed): every packed batch;
// the scan's tile prefix is in B.tile_prefix and each 16-datagram tile's offset
// inside its scan tile in B.sub_prefix.  Tile-local offsets are 32-bit: a tile's
// 16 regions span less than 2^31 bytes (kMaxDatagram = 16 MiB).
template <bool OBF, int SW>
void launch_packed_sw(const BatchParams& b, const KeyParams& k, hipStream_t s) {
    constexpr size_t shm = kPkSlack + HY_PK_LDS + kPkSlack;
    static int grid_max = 0;   // resident workgroups on the device (per instantiation)
    if (!grid_max) {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, salamander_packed_kernel<OBF, SW>, 256, shm);
        grid_max = std::max(1, cus) * std::max(1, per);
    }
    const uint64_t tiles = div_up(b.n, kTileMaxD);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(tiles, (uint64_t)grid_max);
    hipLaunchKernelGGL((salamander_packed_kernel<OBF, SW>), dim3(grid), dim3(256), shm, s, b, k);
}

}  // namespace hyobfs
