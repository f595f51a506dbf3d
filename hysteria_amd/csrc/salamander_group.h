// salamander_group.h -- the group kernel: CONTIGUOUS input into PACKED output
// (gfx950), BASELINE configs[2]'s layout, in the headline tile kernel's shape.
//
// Reference: extras/obfs/salamander.go:59-91 (Obfuscate, Deobfuscate, keyLocked).
//
// One-shot workgroups of four waves, each owning kGD consecutive datagrams: their
// output region [o_p0, o_p0 + sum W) and, with contiguous input, the one input window
// behind it.  Nothing waits on another launch's per-tile record: a workgroup knows its
// datagrams from blockIdx, so
//   * every wave loads the group's lengths (lane per datagram) and the lengths of the
//     scan tile's earlier datagrams (4 per lane) in one round trip and derives the
//     group's output and input offsets from the width / length scan (tile_sums_kernel,
//     scan_tiles_kernel, salamander.hip);
//   * wave 0 loads the salts at the same time (obfuscate) and hashes the kGD keys four
//     lanes per key (quad_key, salamander_tile.h) -- the hash starts after one round
//     trip, as in the tile kernel -- rotated to the output's 32-byte phase;
//   * waves 1-3 copy the input window into LDS by LDS-DMA (global_load_lds_dwordx4,
//     non-temporal, 1 KiB per wave instruction);
//   * after one barrier every thread composes 16-byte output chunks from LDS with the
//     flat kernel's chunk classes (flat_chunk, salamander_flat.h: inside one payload,
//     across one region edge, the general merge) and stores them non-temporal; the two
//     chunks a region shares with the neighbouring groups are byte-masked, so each
//     group writes exactly its own bytes.
// Deobfuscate reads the wire salts at the datagrams' input offsets (a second round
// trip before the hash).  Windows larger than the stage (datagrams over ~1.3 KB on
// average) read the bytes past it from global memory in the general merge: correct
// for every batch, slower.  Applies where the flat kernel does (flat_eligible,
// salamander.hip); HYOBFS_KERNEL=flat selects the flat kernel instead.
#pragma once
#include "salamander_flat.h"

namespace hyobfs {

constexpr uint32_t kGD = 15;   // datagrams per group: keys of 15 on one wave's 16 quads
constexpr int kGT = 16;        // table entries (o[kGT] the sentinel)
#ifndef HY_GROUP_STAGE
#define HY_GROUP_STAGE 20512   // staged input bytes: 15 x 1358 B wire datagrams + 16-byte rounding
#endif
constexpr uint32_t kGStage = HY_GROUP_STAGE;
static_assert(kGStage % 16 == 0, "whole 16-byte DMA chunks");
#ifndef HY_GROUP_MIN_WAVES
#define HY_GROUP_MIN_WAVES 7   // the LDS (~21.6 KB) allows 7 workgroups per CU
#endif

struct GroupLDS {
    uint8_t stage[kFGuard + kGStage + kFGuard];   // input window, byte 0 at stage[kFGuard]
    uint64_t key[kGT][4];     // key rotated to the output's 32-byte phase
    uint64_t salt[kGT];
    int32_t o[kGT + 1];       // output start relative to the group's first chunk ([nt..] = INT_MAX)
    int32_t dlt[kGT];         // stage index of the payload byte at relative output x: x + dlt
    uint32_t w[kGT];          // width (0: dropped) | kFlatOffWin | kFlatOffGrid
};

template <bool OBF, int SW>
__global__ __launch_bounds__(256, HY_GROUP_MIN_WAVES) void salamander_group_kernel(BatchParams B, KeyParams K,
                                                                                   uint64_t ntiles) {
    constexpr int32_t SALT = OBF ? 8 : 0;      // salt bytes in front of the output payload
    constexpr uint32_t SKIP = OBF ? 0u : 8u;   // salt bytes in front of the input payload
    __shared__ __attribute__((aligned(16))) GroupLDS S;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = uni32(tid >> 6);
    const uint8_t* __restrict__ in = B.in;
    const uint64_t p0 = (B.blk0 + blockIdx.x) * (uint64_t)kGD;
    if (p0 >= B.n) return;   // whole workgroup
    const uint32_t nt = (uint32_t)min<uint64_t>((uint64_t)kGD, B.n - p0);

    // ---- every wave: offsets of the group from the scan tile's prefix plus the widths
    // and lengths of the tile's earlier datagrams (at most 255: four per lane)
    const uint64_t tb = p0 / kTile;
    uint64_t pw = 0, pl = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t q = tb * kTile + 4ull * lane + k;
        if (q < p0) {
            const uint32_t Lq = B.in_len[q];
            pw += out_width<OBF>(Lq, B.pkt_cap);
            pl += Lq;
        }
    }
    const bool live = lane < nt;
    const uint32_t L = live ? B.in_len[p0 + lane] : 0u;
    uint64_t salt = OBF && live ? B.salts[p0 + lane] : 0ull;
    const uint64_t o_p0 = uni64(B.tile_prefix[tb] + wave_sum(pw));
    const uint64_t i_p0 = uni64(B.in_tile_prefix[tb] + wave_sum(pl));
    uint32_t W = live ? out_width<OBF>(L, B.pkt_cap) : 0u;
    const uint32_t iw = wave_incl_scan32(W, (int)lane), il = wave_incl_scan32(L, (int)lane);
    const uint64_t o = o_p0 + iw - W, i = i_p0 + il - L;
    if (W && o + W > B.out_cap) W = 0;   // does not fit: dropped (and every later one), offsets unchanged
    const uint64_t Xb = o_p0 & ~15ull;    // the group's first chunk
    // the group's bytes end at its last valid region's end; its input at the last datagram's end
    const uint64_t oend = uni64(wave_max_u64(W ? o + W : 0ull));
    const uint64_t iend = uni64(i_p0 + __shfl(il, 63, 64));
    const uint64_t ws = (i_p0 + SKIP) & ~15ull;
    const uint32_t wlen = (uint32_t)min<uint64_t>(kGStage, iend > ws ? iend - ws : 0ull);

    if (wid != 0) {
        // ---- waves 1-3: the input window into LDS, 1 KiB per instruction (a partial
        // last 16 bytes by single lanes)
        const uint32_t nfull = wlen >> 4;
        for (uint32_t c = wid - 1; c * 64u < nfull; c += 3) {
            const uint32_t ch = c * 64u + lane;
            if (ch < nfull) glds16(in + ws + 16ull * ch, S.stage + kFGuard + 1024u * c);
        }
        const uint32_t tail = wlen & 15u;
        if (tail && wid == 3 && lane < tail) S.stage[kFGuard + 16u * nfull + lane] = in[ws + 16ull * nfull + lane];
    } else {
        // ---- wave 0: keys, four lanes each, rotated to the output's 32-byte phase, and the table
        if (!OBF && W) salt = load8u(in + i);   // the wire's salt
        const uint32_t k = lane >> 2, qi = lane & 3u;
        const uint64_t sk = __shfl(salt, (int)k, 64);
        const uint32_t ok = (uint32_t)__shfl((uint32_t)o, (int)k, 64);
        const uint64_t kw = quad_key<SW>(K, sk, qi);
        const uint32_t rr = (ok + (uint32_t)SALT) & 31u;
        const uint32_t st = (8u * qi - rr) & 31u, w0 = st >> 3, sh = (st & 7u) * 8u;
        const uint64_t a = __shfl(kw, (int)((lane & ~3u) | w0), 64);
        const uint64_t b = __shfl(kw, (int)((lane & ~3u) | ((w0 + 1) & 3u)), 64);
        if (k < nt) S.key[k][qi] = sh ? (a >> sh) | (b << (64 - sh)) : a;
        const int32_t orel = (int32_t)((int64_t)o - (int64_t)Xb);
        const int32_t dlt = (int32_t)((int64_t)(i + SKIP) - (int64_t)ws) - (orel + SALT);
        uint32_t fl = 0;   // the payload inside the staged window, on the 8-byte grid
        if (W) {
            const int32_t ps = orel + SALT, pe = orel + (int32_t)W;
            if (ps < pe && (ps + dlt < 0 || pe + dlt > (int32_t)wlen)) fl |= kFlatOffWin;
            if (dlt & 7) fl |= kFlatOffGrid;
        }
        if (lane < (uint32_t)kGT) {
            S.o[lane] = live ? orel : 0x7FFFFFFF;
            S.w[lane] = W | fl;
            S.dlt[lane] = dlt;
            S.salt[lane] = salt;
        }
        if (lane == 0) S.o[kGT] = 0x7FFFFFFF;
        // the reference's return values
        if (live) {
            if (B.out_off) B.out_off[p0 + lane] = o;
            if (B.out_len) B.out_len[p0 + lane] = W;
        }
        if (B.out_total) {
            const uint64_t written = uni64(wave_sum(W));
            if (lane == 0 && written) atomicAdd(B.out_total, (unsigned long long)written);
        }
    }
    __syncthreads();   // the stage has landed (every wave's vmcnt(0)), the table and keys are published
    if (oend <= o_p0) return;   // nothing valid in this group

    // ---- compose: chunks [Xb, oend) relative to Xb; the first and last are shared with
    // the neighbouring groups and carry only this group's bytes (byte-masked stores)
    uint8_t* __restrict__ ob = B.out + Xb;
    const int32_t tl = (int32_t)(oend - Xb);
    const int32_t first = (int32_t)(o_p0 - Xb);   // 0..15: bytes of the previous group
    const uint32_t kh0 = (uint32_t)(Xb >> 4) & 1u;
    for (int32_t c0 = 0; c0 < tl; c0 += 16 * 256 * kFU) {
        u128 r[kFU];
        uint32_t gen = 0;   // bit u: chunk u takes the general merge
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
            const int32_t rel = c0 + 16 * (int32_t)(u * 256 + tid);
            r[u] = 0;
            if (rel >= tl) continue;
            const bool whole = rel >= first && rel + 16 <= tl;   // no other group's bytes
            if (!whole || !flat_chunk<OBF, kGT>(S, rel, 2u * ((((uint32_t)rel >> 4) + kh0) & 1u), nt, r[u]))
                gen |= 1u << u;
        }
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
            const int32_t rel = c0 + 16 * (int32_t)(u * 256 + tid);
            if (rel < tl && !((gen >> u) & 1u)) store16_stream(ob + rel, r[u]);
        }
        while (gen) {   // the general merge, byte-masked to this group's bytes
            const int u = __builtin_ctz(gen);
            gen &= gen - 1;
            const int32_t rel = c0 + 16 * (int32_t)(u * 256 + tid);
            uint32_t q = 0;
            for (uint32_t s = kGT / 2; s; s >>= 1) q = S.o[q + s] <= rel ? q + s : q;
            u128 v = 0;
            uint32_t cov = 0;
            for (uint32_t k = q; k < nt && S.o[k] < rel + 16; ++k)
                flat_contrib<OBF>(S, in, ws, wlen, k, rel, (((uint32_t)rel >> 4) + kh0) & 1u, v, cov);
            if (cov == 0xFFFFu)
                store16_stream(ob + rel, v);
            else if (cov)
                store_masked(ob + rel, v, cov);
        }
    }
}

template <bool OBF, int SW>
void launch_group_sw(const BatchParams& b, const KeyParams& k, uint64_t ntiles, hipStream_t s) {
    const uint64_t groups = div_up(b.n, kGD);
    BatchParams bp = b;
    bp.blk0 = 0;
    hipLaunchKernelGGL((salamander_group_kernel<OBF, SW>), dim3((uint32_t)groups), dim3(256), 0, s, bp, k, ntiles);
}

}  // namespace hyobfs
