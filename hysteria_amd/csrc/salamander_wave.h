// salamander_wave.h -- the wave-group Salamander kernel (gfx950).
//
// One wavefront owns a GROUP of 64 consecutive datagrams (lane l <-> datagram
// l) and does everything for it without workgroup barriers:
//   1. metadata: length, input offset, salt, output width and offset (packed
//      layout: wavefront scan on top of the tile prefix), drop rules
//      (salamander.go:60-62, :75-77);
//   2. key = BLAKE2b-256(PSK || salt) (salamander.go:88-91), all 12 (or 24)
//      rounds in registers, rotated to the output's 32-byte phase, into LDS;
//   3. boundary: lane l computes the chunks datagram l owns that are not
//      inside one payload (salt bytes, datagram and run edges) and parks the
//      complete ones in LDS, pre-XORed with its key half;
//   4. sweep: the group's output bytes are one contiguous range; the 64 lanes
//      walk it in 16-byte chunks, 1 KiB per wave instruction, kWU chunks per
//      lane in flight.  A chunk inside one payload is one unaligned 16 B load,
//      one LDS key read, four XORs and one aligned non-temporal 16 B store; a
//      parked chunk is an LDS read instead of the load, so every byte of a
//      128-byte line leaves in the same store instructions (no partial-line
//      write-backs);
//   5. late: the few boundary chunks that were not parked (partial chunks at
//      gaps and run edges, slot overflow) are stored with byte masks.
// The four waves of a workgroup are independent (their LDS slices are
// separate), so a CU holds up to 32 waves at different phases: the VALU-bound
// hash of one wave runs while the others stream.  The register budget (64
// VGPRs, 8 waves per SIMD) is what the design is for: the bytes in flight
// per CU come from wave count, not from a deep per-wave pipeline.
#pragma once
#include "salamander_device.h"

namespace hyobfs {

constexpr int kGroup = 64;           // datagrams per wave group (= lanes)
constexpr int kWavesPerBlock = 4;    // independent waves per workgroup
#ifndef HY_WU
#define HY_WU 6                      // 8 spills 12 B with the store order below; 4, 6, 8 run alike
#endif                               // (profiles/r04_ab_wave_store_waits.txt)
constexpr int kWU = HY_WU;           // chunks per lane per sweep iteration
#ifndef HY_RUN_LOG2
#define HY_RUN_LOG2 3
#endif
#ifndef HY_WAVE_MIN_WAVES
#define HY_WAVE_MIN_WAVES 8          // __launch_bounds__ min waves per SIMD (slotted layout)
#endif
#ifndef HY_PACKED_MIN_WAVES
#define HY_PACKED_MIN_WAVES (HY_PACKED_PARK_SLOTS > 64 ? 7 : 8)   // what the packed LDS (park slots) allows
#endif

#ifndef HY_PACKED_DPW
#define HY_PACKED_DPW 32             // packed runs of 64: datagrams per wave (lanes 0..DPW-1 own one)
#endif
#ifndef HY_PACKED_PARK_SLOTS
#define HY_PACKED_PARK_SLOTS 64      // park slots per group, packed layout: ragged mixes have up to ~2
                                     // boundary chunks per datagram, so 64 slots fit 32 datagrams per wave
                                     // (with 64 per wave they overflowed into byte-masked late stores and
                                     // 128 slots were needed, profiles/r02_ab_packed_park_slots.txt).
                                     // 32 per wave + 64 slots (4736 B of LDS per wave: 8 waves/SIMD) ran
                                     // 0.8-1.0 % faster than 64 + 128 (7 waves), 16 per wave 28 % slower
                                     // (profiles/r03_ab_packed_dpw.txt)
#endif
template <bool PACKED>
struct GroupBufT {                   // one wave's group, in LDS (4736 B with 64 slots: 8 workgroups per CU)
    static constexpr int kSlots = PACKED ? HY_PACKED_PARK_SLOTS : kGroup;
    uint2 ow[kGroup];                // output region start (virtual), width (0 = dropped)
    uint64_t io[kGroup];             // input payload start (absolute byte offset)
    uint64_t delta[kGroup];          // real output offset - virtual offset (the run's)
    uint4 key[2 * kGroup];           // key rotated to the output's 32-byte phase, 2 halves
    union {
        uint64_t salt[kGroup];       // salts (obfuscate), read while boundary chunks are built
        u128 bnd[kSlots];            // then: parked boundary chunks, XORed with the owner's key half
    };
    uint16_t park[kGroup];           // bits 0-2 parked (first, second, last chunk), 3-5 late, 8-15 first slot
};
static_assert(HY_PACKED_PARK_SLOTS >= kGroup && HY_PACKED_PARK_SLOTS <= 255, "park slot index is 8 bits");

// ---- BLAKE2b message words of the device block(s).  The message is
// PSK || salt, zero padded: every word after the salt's is a compile-time 0,
// the words before it are PSK words (wave-uniform, scalar), the salt's one or
// two words are per lane.  (KeyParams: hyobfs_api.cpp make_key_params.)
template <int SW, int BLK>
__device__ __forceinline__ uint64_t wmsg(const KeyParams& K, uint64_t lo, uint64_t hi, int idx) {
    if (BLK == 1) return idx == 0 ? hi : 0ull;   // second block: the salt's tail only
    if (idx < SW) return K.m[idx];
    if (idx == SW) return K.m[idx] | lo;
    if (idx == SW + 1) return hi;
    return 0ull;
}

template <int R, int SW, int BLK>
__device__ __forceinline__ void wround(uint64_t v[16], const KeyParams& K, uint64_t lo, uint64_t hi) {
#define HY_W(k) wmsg<SW, BLK>(K, lo, hi, kSigma[R][k])
    HY_G(v, 0, 4, 8, 12, HY_W(0), HY_W(1));
    HY_G(v, 1, 5, 9, 13, HY_W(2), HY_W(3));
    HY_G(v, 2, 6, 10, 14, HY_W(4), HY_W(5));
    HY_G(v, 3, 7, 11, 15, HY_W(6), HY_W(7));
    HY_G(v, 0, 5, 10, 15, HY_W(8), HY_W(9));
    HY_G(v, 1, 6, 11, 12, HY_W(10), HY_W(11));
    HY_G(v, 2, 7, 8, 13, HY_W(12), HY_W(13));
    HY_G(v, 3, 4, 9, 14, HY_W(14), HY_W(15));
#undef HY_W
}

template <int SW, int BLK>
__device__ __forceinline__ void wrounds(uint64_t v[16], const KeyParams& K, uint64_t lo, uint64_t hi) {
    wround<0, SW, BLK>(v, K, lo, hi);
    wround<1, SW, BLK>(v, K, lo, hi);
    wround<2, SW, BLK>(v, K, lo, hi);
    wround<3, SW, BLK>(v, K, lo, hi);
    wround<4, SW, BLK>(v, K, lo, hi);
    wround<5, SW, BLK>(v, K, lo, hi);
    wround<6, SW, BLK>(v, K, lo, hi);
    wround<7, SW, BLK>(v, K, lo, hi);
    wround<8, SW, BLK>(v, K, lo, hi);
    wround<9, SW, BLK>(v, K, lo, hi);
    wround<10, SW, BLK>(v, K, lo, hi);
    wround<11, SW, BLK>(v, K, lo, hi);
}

// keyLocked (salamander.go:88-91) for one lane's salt: BLAKE2b-256 of
// PSK || salt from the host's PSK-only prefix state (RFC 7693 F, unrolled).
template <int SW>
__device__ __forceinline__ void wave_key(const KeyParams& K, uint64_t salt, uint64_t key[4]) {
    const uint32_t sb = (K.salt_pos & 7) * 8;
    const uint64_t lo = salt << sb;
    const uint64_t hi = sb ? (salt >> (64 - sb)) : 0ull;
    uint64_t v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = K.h[i];
        v[i + 8] = kIV[i];
    }
    v[12] ^= K.t[0];
    v[14] = (K.nblk == 1) ? ~v[14] : v[14];
    wrounds<SW, 0>(v, K, lo, hi);
    if (SW == 15 && K.nblk == 2) {   // salt_pos 121..127: chain into the salt's second block
        uint64_t h1[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) h1[i] = K.h[i] ^ v[i] ^ v[i + 8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            v[i] = h1[i];
            v[i + 8] = kIV[i];
        }
        v[12] ^= K.t[1];
        v[14] = ~v[14];
        wrounds<SW, 1>(v, K, lo, hi);
#pragma unroll
        for (int i = 0; i < 4; ++i) key[i] = h1[i] ^ v[i] ^ v[i + 8];
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) key[i] = K.h[i] ^ v[i] ^ v[i + 8];
}

// All bytes datagram k of the group contributes to the 16-byte chunk at relative a.
template <bool OBF, class GroupBuf, class SaltOf>
__device__ __forceinline__ void group_contrib(const GroupBuf& G, const uint8_t* __restrict__ in, uint32_t k,
                                              uint32_t a, u128& r, uint32_t& cov, SaltOf salt_of) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;
    const uint2 owk = G.ow[k];
    const uint32_t oq = owk.x, wq = owk.y;
    if (wq == 0 || oq + wq <= a || oq >= a + 16) return;
    if (OBF) {   // salt bytes [oq, oq + 8)
        const uint32_t sb = max(oq, a), se = min(oq + 8u, a + 16u);
        if (sb < se) {
            u128 S = (u128)salt_of(k);
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
        const uint8_t* src = in + G.io[k];
        u128 X = 0;
        if (PL >= 16) {   // one 16-byte window inside the payload, shifted into place
            const int ws = min(max(base, 0), (int)PL - 16);
            const u128 V = load16u(src + ws);
            const int d = ws - base;
            X = d >= 0 ? (V << (8 * d)) : (V >> (8 * -d));
        } else {
            for (uint32_t j = ps - a; j < pe - a; ++j) X |= (u128)src[base + (int)j] << (8 * j);
        }
        const uint4 kk = G.key[2 * k + ((a >> 4) & 1)];
        u128 k128;
        __builtin_memcpy(&k128, &kk, 16);
        r |= (X ^ k128) & bytemask(ps - a, pe - a);
        cov |= ((1u << (pe - ps)) - 1u) << (ps - a);
    }
}

// Streamed input of the wave kernel: read once, non-temporal (measured faster
// here; the persistent kernel keeps HY_NT_LOADS).
#ifndef HY_WAVE_NT_LOADS
#define HY_WAVE_NT_LOADS 1
#endif
__device__ __forceinline__ u128 load16_nt(const uint8_t* p) {
#if defined(HYOBFS_EMULATE)
    return load16u(p);
#elif !HY_WAVE_NT_LOADS
    typedef uint32_t v4u __attribute__((ext_vector_type(4), aligned(4)));
    typedef const __attribute__((address_space(1))) v4u gv4u;
    const v4u v = *(gv4u*)(p);
    u128 r;
    __builtin_memcpy(&r, &v, 16);
    return r;
#else
    // explicitly global: a generic pointer lets the compiler merge this load
    // with the sweep's LDS read of a parked chunk into one (slow) flat load
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(1))) v4u gv4u;
    const v4u v = __builtin_nontemporal_load((gv4u*)(p));
    u128 r;
    __builtin_memcpy(&r, &v, 16);
    return r;
#endif
}

__device__ __forceinline__ uint64_t load8_nt(const uint8_t* p) {   // 8-aligned
#if defined(HYOBFS_EMULATE)
    return load8u(p);
#else
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    typedef const __attribute__((address_space(1))) v2u gv2u;
    const v2u v = __builtin_nontemporal_load((gv2u*)(p));
    return (uint64_t)v.y << 32 | v.x;
#endif
}

// Last datagram of the group whose region starts at or before virtual offset a.
template <class GroupBuf>
__device__ __forceinline__ uint32_t group_search(const GroupBuf& G, uint32_t a) {
    uint32_t qq = 0;   // last datagram whose region starts at or before a
#pragma unroll
    for (uint32_t step = kGroup / 2; step; step >>= 1) qq = (G.ow[qq + step].x <= a) ? qq + step : qq;
    return qq;
}

// Where the sweep looks for a parked chunk at virtual offset a: datagram qq
// (group_search(a), region owq) if its region reaches into the chunk, else
// datagram qq + 1.  Returns that datagram's region in owo (width 0: none).
template <class GroupBuf>
__device__ __forceinline__ uint32_t park_owner(const GroupBuf& G, uint32_t a, uint32_t qq, uint2 owq, uint2& owo) {
    if (owq.y != 0 && owq.x + owq.y > a) {
        owo = owq;
        return qq;
    }
    owo = qq + 1 < (uint32_t)kGroup ? G.ow[qq + 1] : make_uint2(0xFFFFFFFFu, 0u);
    return qq + 1;
}

// Index of chunk c among a region's boundary candidates: 0 first chunk, 1 the
// next one, 2 the last (when it is neither); 3: not a candidate.
__device__ __forceinline__ uint32_t park_index(uint2 ow, uint32_t c) {
    if (ow.y == 0) return 3u;
    const uint32_t cs = ow.x >> 4, ce = (ow.x + ow.y - 1) >> 4;
    return c == cs ? 0u : (c == cs + 1 && cs + 1 <= ce) ? 1u : (c == ce && ce > cs + 1) ? 2u : 3u;
}

template <bool OBF, bool PACKED, int SW>
__global__ __launch_bounds__(kGroup* kWavesPerBlock, PACKED ? HY_PACKED_MIN_WAVES : HY_WAVE_MIN_WAVES) void
salamander_wave_kernel(BatchParams B, KeyParams K) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;   // salt bytes in front of the output payload
    constexpr uint32_t SKIP = OBF ? 0u : 8u;   // salt bytes in front of the input payload
    constexpr int U = kWU;
    using GroupBuf = GroupBufT<PACKED>;
    __shared__ GroupBuf gbuf[kWavesPerBlock];

    const int lane = threadIdx.x & 63;
    const uint32_t wid = uni32(threadIdx.x >> 6);
    GroupBuf& G = gbuf[wid];
    const uint8_t* __restrict__ in = B.in;
    // Runs of RUN = 2^rl consecutive datagrams; wave w owns runs w, w + Wt,
    // w + 2 Wt, ... (64 / RUN of them), so the waves running at one time work
    // on neighbouring runs and the chip sweeps memory in address order.
    const uint32_t rl = B.run_log2, RUN = 1u << rl;
    const uint64_t Wt = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t w = (B.blk0 + blockIdx.x) * kWavesPerBlock + wid;   // (blk0 > 0 only for packed runs of 64)
    const uint32_t j = (uint32_t)lane >> rl, i = (uint32_t)lane & (RUN - 1);
    const uint64_t r = (uint64_t)j * Wt + w;   // this lane's run
    // packed runs of 64: a wave takes DPW consecutive datagrams (lanes 0..DPW-1)
    constexpr uint32_t DPW = PACKED ? HY_PACKED_DPW : kGroup;
    const bool one_run = PACKED && RUN == kGroup;
    const uint64_t p = one_run ? w * DPW + (uint64_t)lane : (r << rl) + i;   // this lane's datagram
    const bool live = p < B.n && (!one_run || (uint32_t)lane < DPW);
    const uint32_t cnt = uni32((uint32_t)wave_sum(live ? 1u : 0u));   // live lanes are a prefix
    if (cnt == 0) return;

    // ---- 1. metadata
    uint32_t L = 0;
    uint64_t ioff = 0, salt = 0;
    if (live) {
        L = pkt_len(B, p);
        ioff = pkt_in_off(B, p);
        if (OBF) salt = B.salts[p];
    }
    uint32_t W = live ? out_width<OBF>(L, B.pkt_cap) : 0u;
    uint64_t ooff, rfirst;   // output offset of the datagram / of its run's first datagram
    if (PACKED && RUN == kGroup) {   // tile prefix + widths of the tile's earlier datagrams + wave scan
        const uint64_t p0 = w * DPW;
        const uint64_t tb = p0 / kTile * kTile;
        uint64_t pre = 0, ipre = 0;   // widths and (contiguous input) lengths of the tile's earlier datagrams
        for (uint64_t q = tb + lane; q < p0; q += kGroup) {
            const uint32_t Lq = pkt_len(B, q);
            pre += out_width<OBF>(Lq, B.pkt_cap);
            ipre += Lq;
        }
        rfirst = uni64(B.tile_prefix[p0 / kTile] + wave_sum(pre));
        ooff = rfirst + wave_incl_scan(W, lane) - W;
        if (B.in_tile_prefix)   // contiguous input: offsets from the scan of the lengths
            ioff = uni64(B.in_tile_prefix[p0 / kTile] + wave_sum(ipre)) + wave_incl_scan((uint64_t)L, lane) - L;
    } else if (PACKED) {   // shorter runs: the same per run, over the run's RUN lanes
        const uint64_t s0 = r << rl;   // the run's first datagram
        const uint64_t tb = s0 / kTile * kTile;
        uint64_t pre = 0;
        if (s0 < B.n)
            for (uint64_t q = tb + i; q < s0; q += RUN) pre += out_width<OBF>(pkt_len(B, q), B.pkt_cap);
        uint64_t inc = W;   // run sum of `pre`, segmented inclusive scan of W inside the run
        for (uint32_t m = 1; m < RUN; m <<= 1) {
            pre += __shfl_xor(pre, (int)m, 64);
            const uint64_t y = __shfl_up(inc, m, 64);
            if (i >= m) inc += y;
        }
        rfirst = s0 < B.n ? B.tile_prefix[s0 / kTile] + pre : 0;
        ooff = rfirst + inc - W;
    } else {
        ooff = p * B.out_stride;
        rfirst = (r << rl) * B.out_stride;
    }
    if (W && ooff + W > B.out_cap) W = 0;   // does not fit: dropped, offsets unchanged
    if (live) {
        if (B.out_off) B.out_off[p] = ooff;
        if (B.out_len) B.out_len[p] = W;
    }
    if (B.out_total) {   // bytes this wave writes
        const uint64_t written = uni64(wave_sum(W));
        if (lane == 0 && written) atomicAdd(B.out_total, (unsigned long long)written);
    }
    if (!OBF && W) salt = load8u(in + ioff);   // the wire's salt

    // ---- virtual layout: the wave's runs one after another, each from its
    // 16-aligned real base; real address = virtual + delta.  Each run starts at
    // the virtual offset that makes delta a multiple of 128 (up to 7 unused
    // chunks in front of it), so every 1 KiB store instruction of the sweep
    // covers whole 128-byte lines of the output.
    const uint64_t rb = rfirst & ~15ull;
    uint64_t rend = W ? ooff + W : rb;   // end of the run's written bytes
    for (uint32_t m = 1; m < RUN; m <<= 1) rend = max(rend, (uint64_t)__shfl_xor(rend, (int)m, 64));
    const uint32_t nch = live ? (uint32_t)((rend - rb + 15) >> 4) : 0u;   // the run's chunks
#ifndef HY_LINE_ALIGN
#define HY_LINE_ALIGN 1
#endif
    const uint32_t ph = HY_LINE_ALIGN ? (uint32_t)(rb >> 4) & 7u : 0u;   // the run base's chunk within its line
    const uint32_t slots = HY_LINE_ALIGN ? (ph + nch + 7u) >> 3 : nch;   // virtual lines (or chunks) the run takes
    const uint32_t vp = (uint32_t)wave_incl_scan(i == 0 ? slots : 0u, lane) - (i == 0 ? slots : 0u);
    const uint32_t vrun = (HY_LINE_ALIGN ? (__shfl(vp, (int)(lane & ~(RUN - 1)), 64) << 3) + ph
                                         : __shfl(vp, (int)(lane & ~(RUN - 1)), 64))
                          << 4;   // run's virtual start
    const uint32_t rel = live ? vrun + (uint32_t)min<uint64_t>(ooff - rb, (uint64_t)nch << 4) : 0xFFFFFFFFu;
    const uint32_t end = W ? rel + W : 0u;
    uint32_t incm = end;   // inclusive max-scan of region ends (chunk ownership)
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incm, d, 64);
        if (lane >= d) incm = max(incm, y);
    }
    const uint32_t totm = uni32(__shfl(incm, 63, 64));
    // metadata to LDS first: only salt and rel stay live through the hash
    G.ow[lane] = make_uint2(rel, W);
    G.io[lane] = ioff + SKIP;
    G.delta[lane] = rb - vrun;
    if (OBF) G.salt[lane] = salt;

    // ---- 2. key, rotated to the output phase
    {
        uint64_t key[4], kr[4];
        wave_key<SW>(K, salt, key);
        rotl_key_bytes(key, (rel + SALT) & 31u, kr);
        G.key[2 * lane] = make_uint4((uint32_t)kr[0], (uint32_t)(kr[0] >> 32), (uint32_t)kr[1],
                                     (uint32_t)(kr[1] >> 32));
        G.key[2 * lane + 1] = make_uint4((uint32_t)kr[2], (uint32_t)(kr[2] >> 32), (uint32_t)kr[3],
                                         (uint32_t)(kr[3] >> 32));
    }
    hy_wave_sync();

    // ---- 3. boundary chunks datagram `lane` owns (the first datagram touching a
    // chunk owns it: exclusive max-scan of region ends) that are not inside one
    // payload.  A complete one that the sweep's lookup (park_owner/park_index)
    // maps back to this lane is parked; the rest are stored late (step 5).
    // (Merging these bytes inside the sweep instead measured slower: the
    // divergent byte merging cost more than the partial lines it saved.)
    {
        uint32_t parkm = 0, want = 0;
        u128 bv[3] = {0, 0, 0};
        const uint32_t pe0 = __shfl_up(incm, 1, 64);   // max region end over earlier datagrams
        const uint32_t pe = lane ? pe0 : 0u;
        if (W) {
            const uint32_t st = rel, en = rel + W;
            const uint32_t cs = st >> 4, ce = (en - 1) >> 4;
            const uint32_t cand[3] = {cs, cs + 1, ce};
            const bool use[3] = {pe <= (cs << 4), cs + 1 <= ce, ce > cs + 1};
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const uint32_t a = cand[t] << 4;
                if (!use[t] || (st + SALT <= a && a + 16 <= en)) continue;   // inside the payload: swept
                want |= 1u << t;
                u128 rr = 0;
                uint32_t cov = 0;
                for (uint32_t k = lane; k < cnt && G.ow[k].x < a + 16; ++k)
                    group_contrib<OBF>(G, in, k, a, rr, cov, [&](uint32_t kk) { return G.salt[kk]; });
                const uint32_t qq = group_search(G, a);
                uint2 owo;
                const uint32_t o = park_owner(G, a, qq, G.ow[qq], owo);
                if (cov == 0xFFFFu && o == (uint32_t)lane && park_index(owo, cand[t]) == (uint32_t)t) {
                    const uint4 kk = G.key[2 * lane + ((a >> 4) & 1)];
                    u128 k128;
                    __builtin_memcpy(&k128, &kk, 16);
                    bv[t] = rr ^ k128;   // the sweep XORs the owner's key half back in
                    parkm |= 1u << t;
                }
            }
        }
        const uint32_t np = (uint32_t)__builtin_popcount(parkm);
        const uint32_t base = (uint32_t)wave_incl_scan(np, lane) - np;
        if (base + np > (uint32_t)GroupBuf::kSlots) parkm = 0;   // out of slots: store late
        hy_wave_sync();   // every lane has read the salts the slots overwrite
        uint32_t sl = base;
#pragma unroll
        for (int t = 0; t < 3; ++t)
            if ((parkm >> t) & 1u) G.bnd[sl++] = bv[t];
        G.park[lane] = (uint16_t)(parkm | ((want & ~parkm) << 3) | (base << 8));
    }
    hy_wave_sync();

    // ---- 4. sweep: virtual chunks inside one payload, and parked chunks
    const uint32_t nchunks = (totm + 15u) >> 4;
    struct Sweep {   // one iteration's loads in flight
        u128 v[U];
        uint32_t q[U];
        bool fast[U];
    };
    auto issue = [&](uint32_t c0, Sweep& R) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * kGroup + lane;
            const uint32_t a = c << 4;
            const uint32_t qq = group_search(G, a);
            R.q[u] = qq;
            const uint2 owq = G.ow[qq];
            R.fast[u] = (c < nchunks) && owq.y != 0 && owq.x + SALT <= a && a + 16 <= owq.x + owq.y;
            R.v[u] = 0;
            if (R.fast[u]) {
                R.v[u] = load16_nt(in + G.io[qq] + (a - owq.x - SALT));
            }
            else if (c < nchunks) {   // parked boundary chunk?
                uint2 owo;
                const uint32_t o = park_owner(G, a, qq, owq, owo);
                const uint32_t t = park_index(owo, c);
                if (t < 3) {
                    const uint32_t pk = G.park[o];
                    if ((pk >> t) & 1u) {
                        R.fast[u] = true;
                        R.q[u] = o;
                        R.v[u] = G.bnd[(pk >> 8) + (uint32_t)__builtin_popcount(pk & ((1u << t) - 1u))];
                    }
                }
            }
        }
    };
    // Every chunk's value is finished before the first store: the stores then leave
    // from distinct registers.  (Computing each value into the registers the
    // previous store read made the compiler wait for that store to complete,
    // vmcnt(0), before every store of the iteration.)
    auto retire = [&](uint32_t c0, Sweep& R) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t a = (c0 + u * kGroup + lane) << 4;
            const uint4 kk = G.key[2 * R.q[u] + ((a >> 4) & 1)];
            u128 k128;
            __builtin_memcpy(&k128, &kk, 16);
            R.v[u] ^= k128;
#ifndef HYOBFS_EMULATE
            // keep each value in its own registers (no instruction): otherwise the
            // compiler sinks the XOR into the conditional store below, into the
            // registers the previous store read
            uint64_t lo = (uint64_t)R.v[u], hi = (uint64_t)(R.v[u] >> 64);
            __asm__ volatile("" : "+v"(lo), "+v"(hi));
            R.v[u] = (u128)hi << 64 | lo;
#endif
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!R.fast[u]) continue;
            const uint32_t a = (c0 + u * kGroup + lane) << 4;
            store16_stream(B.out + (G.delta[R.q[u]] + a), R.v[u]);
        }
    };
    constexpr uint32_t STEP = kGroup * U;
    for (uint32_t c0 = 0; c0 < nchunks; c0 += STEP) {
        Sweep R;
        issue(c0, R);
        retire(c0, R);
    }

    // ---- 5. late boundary chunks (not parked): byte-masked stores.  The salt
    // slots now hold parked chunks, so salts come from the batch.
    const uint32_t late = (uint32_t)(G.park[lane] >> 3) & 7u;
    if (late) {
        const uint2 own = G.ow[lane];
        const uint32_t st = own.x, en = own.x + own.y;
        const uint32_t cs = st >> 4, ce = (en - 1) >> 4;
        const uint32_t cand[3] = {cs, cs + 1, ce};
        uint8_t* outb = B.out + G.delta[lane];   // a chunk's contributors share its run
        auto salt_of = [&](uint32_t k) {   // datagram index of lane k: its run, then its place in the run
            return B.salts[one_run ? w * DPW + k : ((((uint64_t)(k >> rl)) * Wt + w) << rl) + (k & (RUN - 1))];
        };
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            if (!((late >> t) & 1u)) continue;
            const uint32_t a = cand[t] << 4;
            u128 rr = 0;
            uint32_t cov = 0;
            for (uint32_t k = lane; k < cnt && G.ow[k].x < a + 16; ++k) group_contrib<OBF>(G, in, k, a, rr, cov, salt_of);
            if (cov) store_masked(outb + a, rr, cov);
        }
    }
}

// Datagrams per run for slotted batches (HYOBFS_RUN_LOG2 overrides).  3 = runs
// of 8 datagrams, ~9.6 KB at 1200 B: small enough that the waves in flight
// sweep a ~80 MB window in address order (whole 64-datagram groups leave a
// ~630 MB window, tools/region_copy.hip), large enough that few 128-byte
// lines are shared between runs of different waves.
#ifndef HY_PACKED_RUN_LOG2
#define HY_PACKED_RUN_LOG2 6
#endif
// Environment knobs are read once per process, thread-safely (function-local statics).
inline uint32_t env_run_log2(const char* name, int dflt) {
    const char* e = std::getenv(name);
    const int v = e ? std::atoi(e) : dflt;
    return (uint32_t)(v < 0 ? 0 : v > 6 ? 6 : v);
}
inline uint32_t wave_packed_run_log2() {   // packed layout: datagrams per run (HYOBFS_PACKED_RUN_LOG2)
    static const uint32_t v = env_run_log2("HYOBFS_PACKED_RUN_LOG2", HY_PACKED_RUN_LOG2);
    return v;
}
inline uint32_t wave_run_log2() {
    static const uint32_t v = env_run_log2("HYOBFS_RUN_LOG2", HY_RUN_LOG2);
    return v;
}

// Workgroups per launch for packed runs of 64 (their waves are independent of the
// grid size; the slotted runs interleave over the whole grid and stay one launch):
// HYOBFS_WAVE_LAUNCH_BLOCKS overrides, 0 = one launch (the default: every split measured
// slower on configs[2], 1.51-1.88 against 1.47 ms, profiles/r03_ab_wave_launch_split.txt;
// unlike the tile kernel's, these waves live long enough that each launch pays a tail).
#ifndef HY_WAVE_LAUNCH_BLOCKS
#define HY_WAVE_LAUNCH_BLOCKS 0
#endif
inline uint64_t wave_launch_blocks() {
    static const uint64_t v = [] {
        const char* e = std::getenv("HYOBFS_WAVE_LAUNCH_BLOCKS");
        const long long x = e ? std::atoll(e) : HY_WAVE_LAUNCH_BLOCKS;
        return (uint64_t)(x < 0 ? 0 : x);
    }();
    return v;
}

template <bool OBF, bool PACKED, int SW>
void launch_wave_sw(const BatchParams& bp, const KeyParams& k, hipStream_t s) {
    BatchParams b = bp;
    b.run_log2 = PACKED ? wave_packed_run_log2() : wave_run_log2();
    const bool one_run = PACKED && b.run_log2 == 6;
    const uint64_t ngroups = div_up(bp.n, one_run ? (uint64_t)HY_PACKED_DPW : (uint64_t)kGroup);
    const uint64_t blocks = div_up(ngroups, kWavesPerBlock);
    const uint64_t per = one_run && wave_launch_blocks() ? wave_launch_blocks() : blocks;
    for (uint64_t b0 = 0; b0 < blocks; b0 += per) {
        b.blk0 = b0;
        hipLaunchKernelGGL((salamander_wave_kernel<OBF, PACKED, SW>), dim3((uint32_t)min(per, blocks - b0)),
                           dim3(kGroup * kWavesPerBlock), 0, s, b, k);
    }
}

}  // namespace hyobfs
