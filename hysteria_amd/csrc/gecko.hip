// gecko.hip -- Gecko framing kernels (include/hyobfs_gecko.h).
//
// Encode: one wavefront per group of 64 frames.  The wire datagram of frame f is
//     salt(8) || (hdr(5) || pad || chunk) ^ key_f[i % 32]
// (gecko_frame.go:39-61 encodeFrame, then salamander.go:59-72 Obfuscate).  Lane l
// loads frame l's record, offsets and salt and hashes its key in registers (BLAKE2b-256,
// wave_key<SW> of salamander_wave.h: one instantiation per salt word), so the hash
// overlaps other waves' sweeps (a separate keys_kernel pass via the workspace was 15 %
// slower).  Then, when the group's frames lie in ascending wire order (what
// plan_fragments / writeFragmented produce), the aligned path:
//   1. per frame, the key rotated to the wire's 32-byte phase, the salt and a 16-byte
//      record (wire start, lengths, chunk offset) into LDS; the keystream columns of the
//      edge chunks that hold padding, a column per lane;
//   2. lane l stores frame l's edge chunks (salt and header, the padding/chunk seam,
//      the end), merging every frame that touches such a chunk under byte masks;
//   3. the 64 lanes sweep the group's wire range in aligned 16-byte chunks, two
//      iterations of loads in flight, each lane walking its frame record forward: a chunk
//      inside the padding is one column of a ChaCha8 keystream block (keyed per batch;
//      four lanes per block, gk_ks_quad), one inside the message bytes one unaligned
//      load; each leaves XORed with the key as one 16-byte non-temporal store.
// Otherwise the per-frame window path sweeps 16-byte plaintext windows of each frame
// (numbered by a wave scan) and finishes the edge windows after the sweep.
//
// Parse: one thread per deobfuscated datagram, the checks of ReadFrom
// (gecko.go:170-193) and decodeFrame (gecko_frame.go:65-86) in their order.
#include "kernels.h"
#include "salamander_device.h"
#include "salamander_wave.h"   // wave_key<SW>: the key unrolled per salt word
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

#ifndef HY_GK_U
#define HY_GK_U 3   // 4 spills at the 5-wave register cap
#endif
constexpr int kGkU = HY_GK_U;   // windows per lane in flight

struct GeckoGroup {             // one wave's 64 frames, in LDS
    union {
        struct {                // plaintext-window path
            uint64_t out_off[64];   // wire datagram start
            uint32_t wstart[65];    // first plaintext window of the frame (exclusive scan), [64] = total
        };
        uint4 rec[65];          // aligned path: {rs, hp_plain, chunk_off lo, hi}, [64] = sentinel
    };
    uint64_t chunk_off[64];
    uint16_t hid[64];           // msg_id | idx_total << 8 (the header's varying bytes besides pad_len; gk_hdr)
    uint32_t hp_plain[64];      // chunk start (low 16 bits) | plaintext length (high 16 bits)
    uint64_t salt[64];          // aligned path: the salts (merged into the edge chunks)
    gk_u128 key[128];           // the frame's key, two halves (aligned path: rotated to the wire phase)
    gk_u128 eks[128];           // aligned path: keystream of frame k's edge chunks holding padding
                                // ([2k] the pad's first chunk, [2k + 1] its last)
};

// The 5 header bytes of frame k, little-endian in the low bytes (encodeFrame,
// gecko_frame.go:39-61): flag, msg_id, idx << 4 | total, pad_len big-endian.
__device__ __forceinline__ uint64_t gk_hdr(const GeckoGroup& G, uint32_t k) {
    const uint32_t id = G.hid[k], pad = (G.hp_plain[k] & 0xffff) - HYOBFS_GECKO_HEADER_LEN;
    return (uint64_t)HYOBFS_GECKO_FLAG_FRAGMENT | (uint64_t)(id & 0xff) << 8 | (uint64_t)(id >> 8) << 16 |
           (uint64_t)(pad >> 8) << 24 | (uint64_t)(pad & 0xff) << 32;
}

// ---- padding keystream (include/hyobfs_gecko.h): ChaCha, 8 rounds, RFC 8439 block
// (constants, 8 key words, 32-bit counter, 3 nonce words), each 64-byte block's
// bytes in column order: keystream bytes 64 blk + 16 c .. + 15 are state words c,
// c + 4, c + 8, c + 12.  Pad byte j of frame i is keystream byte out_off[i] + 13 + j.
// The block index is 64-bit: its low word is the counter, its high word is XORed
// into nonce word 0, so offsets past 256 GiB never repeat a block.
// Column order lets four lanes compute one block, a column each, with no transpose.
constexpr int kGkPadRounds = 8;   // ChaCha8: part of the wire format (include/hyobfs_gecko.h)
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
__device__ __forceinline__ gk_u128 gk_ks_quad(const GkPad& P, uint64_t blk, uint32_t qi) {
    const uint32_t a0 = gk_sel4(kChaC0, kChaC1, kChaC2, kChaC3, qi);
    const uint32_t b0 = gk_sel4(P.k[0], P.k[1], P.k[2], P.k[3], qi);
    const uint32_t c0 = gk_sel4(P.k[4], P.k[5], P.k[6], P.k[7], qi);
    const uint32_t d0 = gk_sel4((uint32_t)blk, P.n[0] ^ (uint32_t)(blk >> 32), P.n[1], P.n[2], qi);
    uint32_t a = a0, b = b0, c = c0, d = d0;
#pragma unroll
    for (int r = 0; r < kGkPadRounds / 2; ++r) {
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
__device__ __forceinline__ gk_u128 gk_ks_single(const GkPad& P, uint64_t blk, uint32_t col) {
    uint32_t x[16] = {kChaC0, kChaC1, kChaC2, kChaC3, P.k[0], P.k[1], P.k[2], P.k[3],
                      P.k[4], P.k[5], P.k[6], P.k[7], (uint32_t)blk, P.n[0] ^ (uint32_t)(blk >> 32), P.n[1], P.n[2]};
    uint32_t s[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = x[i];
#pragma unroll
    for (int r = 0; r < kGkPadRounds / 2; ++r) {
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
    const gk_u128 x0 = gk_ks_single(P, c0 >> 6, (uint32_t)(c0 >> 4) & 3u);
    if (!sh) return x0;
    const gk_u128 x1 = gk_ks_single(P, (c0 + 16) >> 6, (uint32_t)((c0 + 16) >> 4) & 3u);
    return (x0 >> (8 * sh)) | (x1 << (8 * (16 - sh)));
}

#ifndef HY_GK_FORCE_WINDOWS
#define HY_GK_FORCE_WINDOWS 0   // A/B and tests: 1 = always the plaintext-window path
#endif

// Frame k's bytes in the 16-byte wire chunk at rel (group-relative, 16-aligned)
// address a: salt, then header / padding / chunk XOR the frame's key.
__device__ __forceinline__ void gk_contrib(const hyobfs_gecko_batch& B, const GkPad& P, const GeckoGroup& G, uint64_t base,
                                           uint32_t k, uint32_t a, gk_u128& r, uint32_t& cov) {
    const uint32_t hpl = G.hp_plain[k];
    if (!hpl) return;
    const int32_t hp = (int32_t)(hpl & 0xffff), plain = (int32_t)(hpl >> 16);
    const uint32_t rs = G.rec[k].x;
    const int32_t p0 = (int32_t)a - (int32_t)rs - HYOBFS_SALT_LEN;   // plaintext index of chunk byte 0
    const int32_t xlo = max(p0, 0), xhi = min(p0 + 16, plain);
    if (xlo < xhi) {
        gk_u128 X = 0;
        const int32_t hhi = min(p0 + 16, (int32_t)HYOBFS_GECKO_HEADER_LEN);
        if (xlo < hhi) {   // header
            const gk_u128 H = (gk_u128)gk_hdr(G, k);
            X |= (p0 <= 0 ? H << (8 * -p0) : H >> (8 * p0)) & gk_mask(xlo - p0, hhi - p0);
        }
        const int32_t plo = max(p0, (int32_t)HYOBFS_GECKO_HEADER_LEN), phi = min(p0 + 16, hp);
        if (plo < phi) {   // the 16-aligned wire chunk at base + a is one keystream column
            // an edge chunk holding padding is the pad's first or last chunk (precomputed)
            const uint32_t c0 = (rs + HYOBFS_SALT_LEN + HYOBFS_GECKO_HEADER_LEN) >> 4;
            X |= G.eks[2 * k + ((a >> 4) == c0 ? 0u : 1u)] & gk_mask(plo - p0, phi - p0);
        }
        const int32_t clo = max(p0, hp);
        if (clo < xhi) {   // chunk bytes
            const uint8_t* __restrict__ ch = B.msg + G.chunk_off[k];
            const int32_t clen = plain - hp, cb = p0 - hp;
            gk_u128 Xc = 0;
            if (clen >= 16) {   // one in-bounds 16-byte load, shifted into place
                const int32_t ws = min(max(cb, 0), clen - 16), d = ws - cb;
                const gk_u128 V = gk_load16u(ch + ws);
                Xc = d >= 0 ? V << (8 * d) : V >> (8 * -d);
            } else {
                for (int32_t j = clo; j < xhi; ++j) Xc |= (gk_u128)ch[j - hp] << (8 * (j - p0));
            }
            X |= Xc & gk_mask(clo - p0, xhi - p0);
        }
        r |= (X ^ G.key[2 * k + ((a >> 4) & 1)]) & gk_mask(xlo - p0, xhi - p0);
        cov |= ((1u << (xhi - xlo)) - 1u) << (xlo - p0);
    }
    const uint32_t slo = max(rs, a), shi = min(rs + HYOBFS_SALT_LEN, a + 16);
    if (slo < shi) {   // salt
        const gk_u128 S = (gk_u128)G.salt[k];
        r |= (rs >= a ? S << (8 * (rs - a)) : S >> (8 * (a - rs))) & gk_mask(slo - a, shi - a);
        cov |= ((1u << (shi - slo)) - 1u) << (slo - a);
    }
}

// The aligned sweep of one wave's group (see the kernel comment).
__device__ __forceinline__ void gecko_encode_aligned(const KeyParams& K, const hyobfs_gecko_batch& B, GeckoGroup& G,
                                                  uint64_t f0, uint32_t lane, bool valid, uint64_t oo,
                                                  uint64_t prevE, uint64_t maxE, unsigned long long vmask,
                                                  uint32_t plain, uint64_t salt, gk_u128 k0, gk_u128 k1) {
    (void)K;
    const GkPad P = gk_pad_params(B);
    // 256-aligned: each wave store instruction (64 lanes x 16 B) covers whole 128-B lines,
    // and the quads of a store instruction hold whole 64-byte keystream blocks
    const uint64_t base = uni64(__shfl(oo, (int)__builtin_ctzll(vmask), 64)) & ~255ull;
    const uint32_t rs = valid ? (uint32_t)(oo - base) : (prevE > base ? (uint32_t)(prevE - base) : 0u);
    const uint32_t rend = (uint32_t)(maxE - base);
    if (!valid) G.hp_plain[lane] = 0;
    {   // (out_off, which this overlays, is not read on the aligned path)
        const uint64_t co = valid ? G.chunk_off[lane] : 0ull;
        G.rec[lane] = make_uint4(rs, valid ? G.hp_plain[lane] : 0u, (uint32_t)co, (uint32_t)(co >> 32));
        if (lane == 0) G.rec[64] = make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);   // stops every walk
    }
    if (valid) {   // the key rotated so that rel address (a + b) mod 32 indexes it
        const uint64_t kw[4] = {(uint64_t)k0, (uint64_t)(k0 >> 64), (uint64_t)k1, (uint64_t)(k1 >> 64)};
        uint64_t kr[4];
        rotl_key_bytes(kw, (rs + HYOBFS_SALT_LEN) & 31u, kr);
        G.key[2 * lane] = (gk_u128)kr[1] << 64 | kr[0];
        G.key[2 * lane + 1] = (gk_u128)kr[3] << 64 | kr[2];
        G.salt[lane] = salt;
    }
    // ---- the keystream columns of the edge chunks that hold padding: frame l's pad
    // runs over wire [rs + 13, rs + 8 + hp); its first and last chunk are edges unless
    // wholly padding (then the sweep covers them).  One column per lane, 64 per pass
    // (gk_ks_single: a whole block, one column kept); lane quads that keep one column
    // of four ran 2.3 % slower (profiles/r05_abg_gecko_sweep_records.txt).
    {
        uint32_t need0 = ~0u, need1 = ~0u;   // group-relative chunk indices
        if (valid) {
            const uint32_t hp = G.hp_plain[lane] & 0xffff;
            const uint32_t ps = rs + HYOBFS_SALT_LEN + HYOBFS_GECKO_HEADER_LEN, pe = rs + HYOBFS_SALT_LEN + hp;
            if (pe > ps) {
                const uint32_t c0 = ps >> 4, c1 = (pe - 1) >> 4;
                if ((ps & 15u) || 16u * c0 + 16u > pe) need0 = c0;
                if (c1 != c0 && (pe & 15u)) need1 = c1;
            }
        }
        const unsigned long long any = __ballot(need0 != ~0u || need1 != ~0u);
        const uint32_t last = any ? 63u - (uint32_t)__builtin_clzll(any) : 0u;   // last frame with a need
        for (uint32_t j = 0; any && j * 32u <= last; ++j) {   // pass j: needs 64 j .. 64 j + 63 (frames 32 j ..)
            const uint32_t n = j * 64u + lane, fr = n >> 1;
            const uint32_t n0 = __shfl(need0, (int)fr, 64), n1 = __shfl(need1, (int)fr, 64);
            const uint32_t c = (n & 1u) ? n1 : n0;
            if (c != ~0u) G.eks[n] = gk_ks_single(P, (base + 16ull * c) >> 6, c & 3u);
        }
    }
    hy_wave_sync();
    uint8_t* __restrict__ ob = B.out + base;
    const uint32_t tc = (rend + 15) >> 4;   // chunks of the group's wire range
    // a chunk is interior when it lies inside one frame's padding or chunk bytes
    auto interior = [&](uint32_t q, uint32_t a, int32_t& p, int32_t& hp) {
        const uint32_t hpl = G.hp_plain[q];
        hp = (int32_t)(hpl & 0xffff);
        const int32_t pl = (int32_t)(hpl >> 16);
        p = (int32_t)a - (int32_t)G.rec[q].x - HYOBFS_SALT_LEN;
        return hpl != 0 && ((p >= (int32_t)HYOBFS_GECKO_HEADER_LEN && p + 16 <= hp) || (p >= hp && p + 16 <= pl));
    };
    // ---- first, the edge chunks of frame `lane` (plain stores, so each such line is
    // still in the L2 when the sweep's streaming stores complete it): the first two (salt, header), the one holding
    // the padding/chunk seam, the last; a chunk an earlier frame reaches into is that
    // frame's, and its owner merges every frame that touches it
    if (valid) {
        const uint32_t hp = G.hp_plain[lane] & 0xffff;
        const uint32_t cs = rs >> 4, ce = (rs + HYOBFS_SALT_LEN + plain - 1) >> 4;
        const uint32_t seam = (rs + HYOBFS_SALT_LEN + hp - 1) >> 4;
        const uint32_t prel = prevE > base ? (uint32_t)(prevE - base) : 0u;
        auto cand = [&](int i) { return i == 0 ? cs : i == 1 ? cs + 1 : i == 2 ? seam : ce; };
        uint32_t m = 0;   // distinct candidates this lane owns
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bool dup = cand(i) > ce || (i == 0 && prel > 16 * cs);
#pragma unroll
            for (int d = 0; d < i; ++d) dup = dup || cand(d) == cand(i);
            if (!dup) m |= 1u << i;
        }
#pragma unroll 1
        while (m) {
            const uint32_t c = cand(__builtin_ctz(m)), a = 16 * c;
            m &= m - 1;
            int32_t p, php;
            if (interior(lane, a, p, php)) continue;
            gk_u128 r = 0;
            uint32_t cov = 0;
            for (uint32_t k = lane; k < 64 && G.rec[k].x < a + 16; ++k) gk_contrib(B, P, G, base, k, a, r, cov);
            if (cov == 0xFFFFu) gk_store16u(ob + a, r);   // a plain store: the line stays in L2 for the sweep's part
            else if (cov) store_masked(ob + a, r, cov);
        }
    }
    // ---- sweep: lane windows move forward by 64 chunks, so the frame walk does too.
    // Per iteration: every lane issues its kGkU loads unconditionally (a chunk that
    // is not message bytes reads the 16-byte hy_safe_line), then the padding chunks
    // are computed and stored, then the message chunks.  With the loads under a
    // branch the compiler waited for vmcnt(0) before every store, i.e. for the
    // previous store's completion; this way each message store waits only for its
    // own load, and the keystream work runs while the loads are in flight.
    struct Step {   // one iteration: kGkU chunks per lane
        gk_u128 v[kGkU];
        uint32_t kq[kGkU];
        uint8_t kind[kGkU];   // 0 nothing, 1 padding, 2 message bytes
    };
    uint32_t q = 0;
    // the lane's frame record and the next one's stay in registers: a window moves
    // forward by 64 chunks, so the walk reads one record per frame passed (the sentinel
    // rec[64] stops it) and the classification needs no further LDS read
    uint4 rq = G.rec[0];
    uint32_t rnx = G.rec[1].x;   // the next frame's wire start
    const uint8_t* const safe = hy_safe_line();
    auto issue = [&](uint32_t T, Step& S) {
#pragma unroll
        for (int u = 0; u < kGkU; ++u) {
            const uint32_t c = T + lane + 64 * u, a = 16 * c;
            while (rnx <= a) {
                ++q;
                rq = G.rec[q];
                rnx = G.rec[q + 1].x;
            }
            const int32_t hp = (int32_t)(rq.y & 0xffff), pl = (int32_t)(rq.y >> 16);
            const int32_t p = (int32_t)a - (int32_t)rq.x - HYOBFS_SALT_LEN;
            const bool in = c < tc && rq.y != 0;
            const bool pad = in && p >= (int32_t)HYOBFS_GECKO_HEADER_LEN && p + 16 <= hp;
            const bool msg = in && p >= hp && p + 16 <= pl;
            S.kind[u] = pad ? 1 : msg ? 2 : 0;
            const uint64_t co = (uint64_t)rq.w << 32 | rq.z;
            S.kq[u] = q;
            S.v[u] = gk_load16u(msg ? B.msg + co + (uint32_t)(p - hp) : safe);
        }
    };
    auto retire = [&](uint32_t T, Step& S) {
#pragma unroll
        for (int u = 0; u < kGkU; ++u) {
            if (__ballot(S.kind[u] == 1)) {   // the whole wave: a quad computes one 64-byte block
                const uint32_t c = T + lane + 64 * u;
                const gk_u128 ks = gk_ks_quad(P, (base + 16ull * c) >> 6, lane & 3u);
                S.v[u] = S.kind[u] == 1 ? ks : S.v[u];
            }
        }
#pragma unroll
        for (int u = 0; u < kGkU; ++u) {
            const uint32_t c = T + lane + 64 * u;
            if (S.kind[u]) store16_stream(ob + 16 * c, S.v[u] ^ G.key[2 * S.kq[u] + (c & 1)]);
        }
    };
    constexpr uint32_t STEP = 64 * kGkU;
    // Software pipelined: iteration i+1's loads are issued before iteration i's
    // stores, so waiting for them never waits for those stores (vmcnt counts loads
    // and stores in issue order); past the range end issue() reads only the safe line.
    {
        Step S0, S1;
        issue(0, S0);
        for (uint32_t T = 0; T < tc; T += 2 * STEP) {
            issue(T + STEP, S1);
            retire(T, S0);
            if (T + STEP >= tc) break;
            issue(T + 2 * STEP, S0);
            retire(T + STEP, S1);
        }
    }
}

// Register cap: 5 waves/SIMD with the pipelined sweep (two iterations' registers):
// 0.536-0.539 ms against 0.545 at 6 waves and 0.551 unpipelined at 6
// (profiles/r03_ab_gecko_pipe.txt).  Unpipelined, 6 waves measured fastest with the
// per-salt-word key: 0.561 ms against 0.567 at 5 waves (94 VGPRs), 0.623 for the
// generic key at 4 waves (97 VGPRs) and 0.734 at 8 waves (heavy spills),
// profiles/r03_ab_gecko_occupancy.txt.
#ifndef HY_GK_WPE
#define HY_GK_WPE 5
#endif
#ifdef HYOBFS_EMULATE
#define HY_GK_ATTR
#else
#define HY_GK_ATTR __attribute__((amdgpu_waves_per_eu(HY_GK_WPE)))
#endif
template <int SW>
__global__ __launch_bounds__(256) HY_GK_ATTR void gecko_encode_kernel(KeyParams K, hyobfs_gecko_batch B) {
    __shared__ GeckoGroup gg[4];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    GeckoGroup& G = gg[wid];
    const uint64_t f0 = ((uint64_t)blockIdx.x * 4 + wid) * 64;
    if (f0 >= B.n) return;
    // ---- 1. lane l: frame f0 + l's record, offsets, salt and key into LDS
    const uint64_t f = f0 + lane;
    uint32_t nwin = 0, plain = 0;
    uint64_t oo = 0, salt = 0;
    gk_u128 k0 = 0, k1 = 0;
    if (f < B.n) {
        const hyobfs_gecko_frame fr = B.frames[f];
        const uint32_t total = fr.idx_total & 0x0f, idx = fr.idx_total >> 4;
        const uint32_t hp = HYOBFS_GECKO_HEADER_LEN + fr.pad_len;
        const uint64_t plain64 = (uint64_t)hp + fr.chunk_len;   // 64-bit: a hostile chunk_len must not wrap
        if (total >= HYOBFS_GECKO_MIN_CHUNKS && total <= HYOBFS_GECKO_MAX_CHUNKS && idx < total &&
            HYOBFS_SALT_LEN + plain64 <= HYOBFS_GECKO_BUFFER_SIZE) {   // else: skipped, nothing written
            plain = (uint32_t)plain64;
            nwin = (plain + 15) >> 4;
            oo = B.out_off[f];
            G.out_off[lane] = oo;
            G.chunk_off[lane] = fr.chunk_off;
            G.hid[lane] = (uint16_t)(fr.msg_id | fr.idx_total << 8);
            G.hp_plain[lane] = hp | plain << 16;
            salt = B.salts[f];
            // keyLocked (salamander.go:88-91) in registers; the hash overlaps other waves' sweeps
            uint64_t kw[4];
            wave_key<SW>(K, salt, kw);
            k0 = (gk_u128)kw[1] << 64 | kw[0];
            k1 = (gk_u128)kw[3] << 64 | kw[2];
        }
    }
    // Aligned path when the group's valid frames are in ascending, non-overlapping
    // wire order (what plan_fragments / writeFragmented produce): sweep the
    // group's wire range in aligned 16-byte chunks, so every interior line leaves
    // whole; otherwise the plaintext-window path below.
    const bool valid = nwin != 0;
    const uint64_t wend = oo + HYOBFS_SALT_LEN + plain;
    uint64_t incE = valid ? wend : 0;   // inclusive max-scan of wire ends
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(incE, d, 64);
        if (lane >= (uint32_t)d) incE = max(incE, y);
    }
    uint64_t prevE = __shfl_up(incE, 1, 64);
    if (lane == 0) prevE = 0;
    const uint64_t maxE = uni64(__shfl(incE, 63, 64));
    const unsigned long long vmask = __ballot(valid);
    const bool aligned = !HY_GK_FORCE_WINDOWS && vmask != 0 && !__ballot(valid && oo < prevE) &&
                         maxE - (uni64(__shfl(oo, (int)__builtin_ctzll(vmask), 64)) & ~255ull) < (1ull << 31);
    if (aligned) {
        gecko_encode_aligned(K, B, G, f0, lane, valid, oo, prevE, maxE, vmask, plain, salt, k0, k1);
        return;
    }
    if (valid) {
        G.key[2 * lane] = k0;
        G.key[2 * lane + 1] = k1;
        __builtin_memcpy(B.out + oo, &salt, HYOBFS_SALT_LEN);
    }
    uint32_t inc = nwin;   // inclusive scan of window counts
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
    }
    G.wstart[lane] = inc - nwin;
    if (lane == 63) G.wstart[64] = inc;
    hy_wave_sync();
    const uint32_t tw = __builtin_amdgcn_readfirstlane(G.wstart[64]);
    // A window is interior when it lies inside the padding or inside the chunk; the
    // sweep does only those (no divergent byte merging), lane l then finishes frame
    // l's few edge windows (header, padding/chunk seam, the frame's end).
    auto interior = [](uint32_t p, uint32_t hp, uint32_t plain) {
        return (p >= hp && p + 16 <= plain) || (p >= HYOBFS_GECKO_HEADER_LEN && p + 16 <= hp);
    };
    const GkPad P = gk_pad_params(B);
    auto pad16 = [&](uint32_t k, uint32_t p) -> gk_u128 {   // keystream at plaintext [p, p+16) of frame f0+k
        return gk_ks_at(P, G.out_off[k] + HYOBFS_SALT_LEN + p);
    };
    auto store = [&](uint32_t k, uint32_t p, uint32_t plain, gk_u128 v) {
        uint8_t* __restrict__ po = B.out + G.out_off[k] + HYOBFS_SALT_LEN;
        if (p + 16 <= plain) {
            gk_store16u(po + p, v);
        } else {   // the frame's last partial window
            for (uint32_t j = p; j < plain; ++j) po[j] = (uint8_t)(v >> (8 * (j - p)));
        }
    };
    // ---- edge windows of frame `lane`: header window, the window holding the
    // padding/chunk seam and the next one (short chunks), and the last window
    const uint32_t ehpl = nwin ? G.hp_plain[lane] : 0u, ehp = ehpl & 0xffff, eplain = ehpl >> 16;
    auto cand = [&](uint32_t c) { return c == 0 ? 0u : c == 3 ? nwin - 1 : (ehp >> 4) + c - 1; };
    uint32_t emask = 0;   // candidates that are edge windows (not interior, not repeated)
    if (nwin) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            bool dup = cand(c) >= nwin;
#pragma unroll
            for (int d = 0; d < c; ++d) dup = dup || cand(d) == cand(c);
            if (!dup && !interior(16 * cand(c), ehp, eplain)) emask |= 1u << c;
        }
    }
    auto edge = [&](uint32_t wi) {
        const uint32_t k = lane, hp = ehp, plain = eplain;
        const uint8_t* __restrict__ chunk = B.msg + G.chunk_off[k];
        const uint32_t p = 16 * wi;
        const uint32_t e = min(p + 16, plain);
        gk_u128 v = 0;
        if (p == 0) v = (gk_u128)gk_hdr(G, k) & gk_mask(0, min(e, (uint32_t)HYOBFS_GECKO_HEADER_LEN));
        const uint32_t plo = max(p, (uint32_t)HYOBFS_GECKO_HEADER_LEN), phi = min(e, hp);
        if (plo < phi) v |= pad16(k, p) & gk_mask(plo - p, phi - p);
        const uint32_t clo = max(p, hp);
        if (clo < e) {   // chunk bytes
            const uint32_t clen = plain - hp;
            gk_u128 X = 0;
            if (p >= hp && p + 16 <= plain) {
                X = gk_load16u(chunk + (p - hp));
            } else if (clen >= 16) {   // first or last window of the chunk: one in-bounds load, shifted
                X = p < hp ? gk_load16u(chunk) << (8 * (hp - p)) : gk_load16u(chunk + (clen - 16)) >> (8 * (p + 16 - plain));
            } else {
                for (uint32_t j = clo; j < e; ++j) X |= (gk_u128)chunk[j - hp] << (8 * (j - p));
            }
            v |= X & gk_mask(clo - p, e - p);
        }
        store(k, p, plain, v ^ G.key[2 * k + (wi & 1)]);
    };
    auto edges = [&](uint32_t m) {   // one copy of the edge code (registers: 5 waves/SIMD)
#pragma unroll 1
        while (m) {
            const uint32_t c = __builtin_ctz(m);
            m &= m - 1;
            edge(cand(c));
        }
    };
    // ---- 2. sweep: window t belongs to the last frame whose first window is <= t.
    // A lane's windows only move forward (t0 + 64 u), so its frame index q does too:
    // it steps over the frames started since its previous window (one or two LDS
    // reads for frames of >= 32 windows) instead of a fresh 6-step search.  Edge
    // windows come after the sweep: storing each inside the iteration whose range
    // holds it (an A/B build, since removed, meant to let lines split between a frame's
    // interior and its edges leave the L2 whole) made the sweep divergent, 0.616 ->
    // 0.826 ms (profiles/r01_ab_gecko/).
    uint32_t q = 0;
    for (uint32_t T = 0; T < tw; T += 64 * kGkU) {
        const uint32_t t0 = T + lane;
        gk_u128 v[kGkU];
        uint32_t kk[kGkU], pp[kGkU];
        bool ok[kGkU];
#pragma unroll
        for (int u = 0; u < kGkU; ++u) {   // all windows' loads first
            const uint32_t t = t0 + 64 * u;
            if (t < tw)   // wstart[64] = tw > t stops the walk at frame 63
                while (G.wstart[q + 1] <= t) ++q;
            const uint32_t wi = t - G.wstart[q], p = 16 * wi;
            const uint32_t hpl = G.hp_plain[q], hp = hpl & 0xffff, plain = hpl >> 16;
            kk[u] = q;
            pp[u] = p;
            ok[u] = t < tw && interior(p, hp, plain);
            v[u] = 0;
            if (ok[u]) {
                v[u] = p >= hp ? gk_load16u(B.msg + G.chunk_off[q] + (p - hp)) : pad16(q, p);
                v[u] ^= G.key[2 * q + (wi & 1)];
            }
        }
#pragma unroll
        for (int u = 0; u < kGkU; ++u)
            if (ok[u]) store(kk[u], pp[u], 0xFFFFFFFFu, v[u]);
    }
    edges(emask);   // ---- 3. all edge windows after the sweep
}

__global__ __launch_bounds__(256) void gecko_parse_kernel(const uint8_t* in, const uint64_t* in_off,
                                                          const uint32_t* in_len, uint64_t n,
                                                          hyobfs_gecko_parsed* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    hyobfs_gecko_parsed r{};
    const uint32_t len = in_len[i];
    const uint8_t* d = in + in_off[i];
    if (len == 0) {
        r.status = HYOBFS_GECKO_EMPTY;                       // n <= 0: continue
    } else if (!(d[0] & HYOBFS_GECKO_FLAG_FRAGMENT)) {
        r.status = HYOBFS_GECKO_PASS;                        // short header / garbage: passed through
        r.payload_len = len;
    } else if (len < HYOBFS_GECKO_HEADER_LEN) {
        r.status = HYOBFS_GECKO_ERR_TRUNCATED;
    } else {
        const uint32_t it = d[2], total = it & 0x0f, idx = it >> 4;
        const uint32_t pad = ((uint32_t)d[3] << 8) | d[4];
        if (total < HYOBFS_GECKO_MIN_CHUNKS || total > HYOBFS_GECKO_MAX_CHUNKS || idx >= total) {
            r.status = HYOBFS_GECKO_ERR_INVALID;
        } else if (HYOBFS_GECKO_HEADER_LEN + pad > len) {
            r.status = HYOBFS_GECKO_ERR_TRUNCATED;
        } else {
            r.status = HYOBFS_GECKO_FRAGMENT;
            r.msg_id = d[1];
            r.idx_total = (uint8_t)it;
            r.pad_len = (uint16_t)pad;
            r.payload_off = HYOBFS_GECKO_HEADER_LEN + pad;
            r.payload_len = len - r.payload_off;
        }
    }
    out[i] = r;
}

hipError_t launch_gecko_encode(const KeyParams& k, const hyobfs_gecko_batch& b, hipStream_t s) {
    if (b.n == 0) return hipSuccess;
    // instantiated per salt word (salamander_inst.hip's rule): the PSK's message words
    // stay scalar, only the salt's one or two words are per lane
    const dim3 grid((uint32_t)((b.n + 255) / 256)), block(256);
    switch (k.salt_pos >> 3) {
#define HY_CASE(n) \
    case n: hipLaunchKernelGGL(gecko_encode_kernel<n>, grid, block, 0, s, k, b); break;
        HY_CASE(0) HY_CASE(1) HY_CASE(2) HY_CASE(3) HY_CASE(4) HY_CASE(5) HY_CASE(6) HY_CASE(7)
        HY_CASE(8) HY_CASE(9) HY_CASE(10) HY_CASE(11) HY_CASE(12) HY_CASE(13) HY_CASE(14) HY_CASE(15)
#undef HY_CASE
    }
    return hipGetLastError();
}

hipError_t launch_gecko_parse(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint64_t n,
                              hyobfs_gecko_parsed* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gecko_parse_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, in, in_off, in_len,
                       n, out);
    return hipGetLastError();
}

}  // namespace hyobfs
