// gecko_tile.h -- the Gecko encode tile kernel (gfx950).
//
// Reference: extras/obfs/gecko_frame.go:39-61 (encodeFrame) under
// extras/obfs/salamander.go:59-72 (Obfuscate); the wire datagram of frame f is
//     salt(8) || (hdr(5) || pad || chunk) ^ key_f[i % 32],  key_f = BLAKE2b-256(PSK || salt)
// with the padding taken from the batch's keystream (include/hyobfs_gecko.h).
//
// The salamander_tile.h shape for frames.  A workgroup of four waves owns a tile
// of 16 consecutive frames and exits when done:
//   1. wave 0 loads the 16 frame records, offsets and salts in one round trip,
//      hashes the 16 keys on quads (quad_key: four lanes per key) and publishes
//      the valid frames' metadata, compacted in wire order, and the keys into LDS;
//   2. after one barrier, all four waves sweep the tile's wire range on the
//      global 16-byte grid from a 64-byte aligned base, so the four lanes of a
//      quad hold the four columns of one keystream block and compute it together
//      (gk_ks_quad).  The sweep takes the chunks inside one frame's padding (its
//      keystream column XOR 16 key bytes: an unaligned LDS read of the key stored
//      twice in a row) or inside its message bytes (one unaligned 16-byte load of
//      the message XOR the key): every lane on the same path;
//   3. then each frame's at most five other chunks (salt, header, the
//      padding/message seam, the frame's end) are merged by one thread each,
//      every frame touching the chunk under byte masks.  Chunks shared with the
//      neighbouring tiles: masked stores.  (Merging those inside the sweep made
//      every wave instruction run the merge for a few lanes: 2x slower.)
// A tile whose valid frames are not in ascending, non-overlapping wire order, or
// whose wire range has long gaps (more than kGtMaxRange bytes from the first
// frame's start to the last frame's end), sweeps each frame's own range instead.
#pragma once
#include "gecko_device.h"
#include "salamander_tile.h"

namespace hyobfs {

#ifndef HY_GT_U
#define HY_GT_U 2                 // chunks per thread and sweep pass (256 x 2 x 16 B = 8 KiB; 4: 78 VGPRs)
#endif
#ifndef HY_GT_MIN_WAVES
#define HY_GT_MIN_WAVES 8
#endif
// the merged sweep's longest tile range: 16 datagrams of the largest size, no gaps
constexpr uint32_t kGtMaxRange = kTileMaxD * HYOBFS_GECKO_BUFFER_SIZE + 64;

struct GtMeta {                      // the tile's valid frames in tile order (v = 0 .. nv-1)
    uint32_t rs[kTileMaxD + 1];      // merged: wire start relative to base; [nv] = end of the last
    uint32_t hpl[kTileMaxD];         // plaintext chunk start hp (low 16 bits) | plaintext length (high 16)
    uint32_t kix[kTileMaxD];         // the frame's place in the tile (its key in s_key)
    uint64_t hdr[kTileMaxD];         // the 5 header bytes, little-endian
    uint64_t coff[kTileMaxD];        // chunk offset in msg
    uint64_t salt[kTileMaxD];
    uint64_t oo[kTileMaxD];          // wire start (absolute offset in out)
    uint64_t base;                   // merged: 64-aligned absolute offset the sweep starts at
    uint32_t nv;
    uint32_t merged;
};

// Frame v's bytes in the 16-byte chunk whose byte 0 is at offset a, the frame's
// wire start being at rs (both relative to the same 64-aligned origin): salt,
// then header / padding (ks(): the chunk's keystream column) / chunk bytes, XOR the key.
template <class KS>
__device__ __forceinline__ void gt_contrib(const hyobfs_gecko_batch& B, const GtMeta& M, const uint8_t* s_keyb,
                                           uint32_t v, int32_t rs, int32_t a, KS&& ks, gk_u128& r,
                                           uint32_t& cov) {
    const uint32_t hpl = M.hpl[v];
    const int32_t hp = (int32_t)(hpl & 0xffff), plain = (int32_t)(hpl >> 16);
    const int32_t p0 = a - rs - (int32_t)HYOBFS_SALT_LEN;   // plaintext index of chunk byte 0
    const int32_t xlo = max(p0, 0), xhi = min(p0 + 16, plain);
    if (xlo < xhi) {
        gk_u128 X = 0;
        const int32_t hhi = min(p0 + 16, (int32_t)HYOBFS_GECKO_HEADER_LEN);
        if (xlo < hhi) {   // header
            const gk_u128 H = (gk_u128)M.hdr[v];
            X |= (p0 <= 0 ? H << (8 * -p0) : H >> (8 * p0)) & gk_mask(xlo - p0, hhi - p0);
        }
        const int32_t plo = max(p0, (int32_t)HYOBFS_GECKO_HEADER_LEN), phi = min(p0 + 16, hp);
        if (plo < phi) X |= ks() & gk_mask(plo - p0, phi - p0);   // padding
        const int32_t clo = max(p0, hp);
        if (clo < xhi) {   // chunk bytes
            const uint8_t* __restrict__ ch = B.msg + M.coff[v];
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
        gk_u128 Kb;   // key bytes for plaintext indices p0 .. p0 + 15
        __builtin_memcpy(&Kb, s_keyb + 64 * M.kix[v] + (uint32_t)(p0 & 31), 16);
        r |= (X ^ Kb) & gk_mask(xlo - p0, xhi - p0);
        cov |= ((1u << (xhi - xlo)) - 1u) << (xlo - p0);
    }
    const int32_t slo = max(rs, a), shi = min(rs + (int32_t)HYOBFS_SALT_LEN, a + 16);
    if (slo < shi) {   // salt
        const gk_u128 S = (gk_u128)M.salt[v];
        r |= (rs >= a ? S << (8 * (rs - a)) : S >> (8 * (a - rs))) & gk_mask(slo - a, shi - a);
        cov |= ((1u << (shi - slo)) - 1u) << (slo - a);
    }
}

template <int SW>
__global__ __launch_bounds__(256, HY_GT_MIN_WAVES) void gecko_tile_kernel(KeyParams K, hyobfs_gecko_batch B) {
    __shared__ uint64_t s_key[kTileMaxD * 8];   // frame k's key twice in a row: any 16 key bytes are contiguous
    __shared__ GtMeta M;
    constexpr int U = HY_GT_U;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = uni32(tid >> 6);
    const uint64_t f0 = (uint64_t)blockIdx.x * kTileMaxD;
    const uint32_t nt = (uint32_t)min<uint64_t>((uint64_t)kTileMaxD, B.n - f0);

    if (wid == 0) {
        // ---- one round trip: lane k < nt the frame record and offset, quad k the salt
        const uint32_t qk = lane >> 2, qi = lane & 3;
        hyobfs_gecko_frame fr{};
        uint64_t oo = 0;
        if (lane < nt) {
            fr = B.frames[f0 + lane];
            oo = B.out_off[f0 + lane];
        }
        const uint64_t salt = qk < nt ? B.salts[f0 + qk] : 0ull;
#if defined(HY_X_NOHASH) || defined(HY_X_TILE_NOHASH)   // ablation builds only (wrong output)
        const uint64_t kw = salt * (qi + 3);
#else
        const uint64_t kw = quad_key<SW>(K, salt, qi);   // keyLocked, salamander.go:88-91
#endif
        if (qk < nt) {
            s_key[qk * 8 + qi] = kw;
            s_key[qk * 8 + 4 + qi] = kw;
        }
        // ---- the frame rules of gecko_encode_kernel (a frame the reference could not
        // have produced is skipped, its bytes untouched)
        const uint32_t total = fr.idx_total & 0x0f, idx = fr.idx_total >> 4;
        const uint32_t hp = HYOBFS_GECKO_HEADER_LEN + fr.pad_len;
        const uint64_t plain64 = (uint64_t)hp + fr.chunk_len;   // 64-bit: a hostile chunk_len must not wrap
        const bool valid = lane < nt && total >= HYOBFS_GECKO_MIN_CHUNKS && total <= HYOBFS_GECKO_MAX_CHUNKS &&
                           idx < total && HYOBFS_SALT_LEN + plain64 <= HYOBFS_GECKO_BUFFER_SIZE;
        const uint32_t plain = valid ? (uint32_t)plain64 : 0u;
        const unsigned long long vm = __ballot(valid);
        const uint32_t nv = (uint32_t)__builtin_popcountll(vm);
        const uint32_t v = (uint32_t)__builtin_popcountll(vm & ((1ull << lane) - 1ull));   // compact index
        // merged sweep: valid frames ascending and non-overlapping, range bounded
        const uint64_t E = valid ? oo + HYOBFS_SALT_LEN + plain : 0ull;
        uint64_t incE = E;   // inclusive max-scan of wire ends
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint64_t y = __shfl_up(incE, d, 64);
            if (lane >= (uint32_t)d) incE = max(incE, y);
        }
        uint64_t prevE = __shfl_up(incE, 1, 64);
        if (lane == 0) prevE = 0;
        const uint64_t maxE = uni64(__shfl(incE, 15, 64));
        const uint64_t first = vm ? uni64(__shfl(oo, (int)__builtin_ctzll(vm), 64)) : 0ull;
        const uint64_t base = first & ~63ull;
        const bool merged = vm != 0 && !__ballot(valid && oo < prevE) && maxE - base <= kGtMaxRange;
        const uint64_t slt = __shfl(salt, (int)(4 * (lane & 15)), 64);
        if (valid) {
            M.rs[v] = (uint32_t)(oo - base);
            M.hpl[v] = hp | plain << 16;
            M.kix[v] = lane;
            M.hdr[v] = (uint64_t)HYOBFS_GECKO_FLAG_FRAGMENT | (uint64_t)fr.msg_id << 8 | (uint64_t)fr.idx_total << 16 |
                       (uint64_t)(fr.pad_len >> 8) << 24 | (uint64_t)(fr.pad_len & 0xff) << 32;
            M.coff[v] = fr.chunk_off;
            M.salt[v] = slt;
            M.oo[v] = oo;
        }
        if (lane == 0) {
            M.rs[nv] = (uint32_t)(maxE - base);
            M.base = base;
            M.nv = nv;
            M.merged = merged ? 1u : 0u;
        }
    }
    __syncthreads();   // keys and metadata published

    const uint32_t nv = M.nv;
    if (nv == 0) return;
    const GkPad P = gk_pad_params(B);
    const uint8_t* s_keyb = reinterpret_cast<const uint8_t*>(s_key);
    if (M.merged) {
        const uint64_t base = M.base;
        const uint32_t nch = (M.rs[nv] + 15) >> 4;
        uint8_t* __restrict__ ob = B.out + base;
        // frame starts in registers (lane d: frame d, past nv: never reached)
        const int32_t rsl = lane < nv ? (int32_t)M.rs[lane] : 0x7fffffff;
        int32_t rsd[kTileMaxD];
#pragma unroll
        for (int d = 1; d < (int)kTileMaxD; ++d) rsd[d] = __builtin_amdgcn_readlane(rsl, d);
        // ---- sweep: the chunks inside one frame's padding or message bytes
        for (uint32_t c0 = 0; c0 < nch; c0 += 256u * U) {
            gk_u128 r[U];
            bool ok[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = c0 + (uint32_t)u * 256u + tid;
                const int32_t a = (int32_t)(16u * c);
                const bool in = c < nch;
                uint32_t k = 0;   // the last frame starting at or before a
#pragma unroll
                for (int d = 1; d < (int)kTileMaxD; ++d) k += rsd[d] <= a ? 1u : 0u;
                const int32_t rs = (int32_t)M.rs[k];
                const uint32_t hpl = M.hpl[k];
                const int32_t hp = (int32_t)(hpl & 0xffff), plain = (int32_t)(hpl >> 16);
                const int32_t p = a - rs - (int32_t)HYOBFS_SALT_LEN;
                const bool ichunk = in && p >= hp && p + 16 <= plain;
                const bool ipad = in && p >= (int32_t)HYOBFS_GECKO_HEADER_LEN && p + 16 <= hp;
                gk_u128 ks = 0;
                if (__ballot(ipad))   // the whole wave: a quad computes one 64-byte block
#ifdef HY_X_NOPAD   // ablation builds only (timing experiments; wrong output)
                    ks = (gk_u128)(base + 16ull * c);
#else
                    ks = gk_ks_quad(P, (uint32_t)((base + 16ull * c) >> 6), lane & 3u);
#endif
                ok[u] = ichunk || ipad;
                r[u] = 0;
                if (ok[u]) {
                    const gk_u128 X = ichunk ? gk_load16u(B.msg + M.coff[k] + (uint32_t)(p - hp)) : ks;
                    gk_u128 Kb;
                    __builtin_memcpy(&Kb, s_keyb + 64 * M.kix[k] + (uint32_t)(p & 31), 16);
                    r[u] = X ^ Kb;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (ok[u]) store16_stream(ob + 16u * (c0 + (uint32_t)u * 256u + tid), r[u]);
        }
        // ---- edges: a frame's other chunks are among five (salt and header: 13 bytes,
        // at most two chunks; the last chunk holding padding or header and the first
        // holding message bytes; the last).  Thread e takes candidate e % 5 of frame
        // e / 5; the first frame touching a chunk merges every frame touching it.
        if (tid < 5u * nv) {
            const uint32_t v = tid / 5u, w = tid % 5u;
            const int32_t rs = (int32_t)M.rs[v];
            const uint32_t hpl = M.hpl[v];
            const int32_t hp = (int32_t)(hpl & 0xffff), plain = (int32_t)(hpl >> 16);
            const int32_t E = rs + (int32_t)HYOBFS_SALT_LEN + plain;
            auto cand = [&](uint32_t i) -> int32_t {
                const int32_t x = i == 0 ? rs : i == 1 ? rs + 12 : i == 2 ? rs + 7 + hp : i == 3 ? rs + 8 + hp : E - 1;
                return x >> 4;
            };
            const int32_t c = cand(w), a = 16 * c;
            bool skip = a >= E;   // no message bytes: candidate 3 may lie past the frame
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) skip = skip || (i < w && cand(i) == c);
            const int32_t p = a - rs - (int32_t)HYOBFS_SALT_LEN;
            skip = skip || (p >= hp && p + 16 <= plain) || (p >= (int32_t)HYOBFS_GECKO_HEADER_LEN && p + 16 <= hp);
            // frames are ascending: only the previous one can reach into the chunk
            skip = skip || (v > 0 && (int32_t)(M.rs[v - 1] + HYOBFS_SALT_LEN + (M.hpl[v - 1] >> 16)) > a);
            if (!skip) {
                gk_u128 r = 0, ksv = 0;
                uint32_t cov = 0;
                bool have = false;
                auto ks = [&]() -> gk_u128 {   // this chunk's keystream column, one lane alone
                    if (!have) {
                        const uint64_t g = base + (uint64_t)a;
                        ksv = gk_ks_single(P, (uint32_t)(g >> 6), (uint32_t)(g >> 4) & 3u);
                        have = true;
                    }
                    return ksv;
                };
                for (uint32_t kk = v; kk < nv && (int32_t)M.rs[kk] < a + 16; ++kk)
                    gt_contrib(B, M, s_keyb, kk, (int32_t)M.rs[kk], a, ks, r, cov);
                if (cov == 0xFFFFu)
                    store16_stream(ob + a, r);
                else if (cov)
                    store_masked(ob + a, r, cov);
            }
        }
        return;
    }
    // ---- each frame's own range, one wave per frame, from its 64-aligned origin
    for (uint32_t v = wid; v < nv; v += 4) {
        const uint64_t oo = M.oo[v];
        const uint64_t A0 = oo & ~63ull;
        const int32_t rs = (int32_t)(oo - A0);
        const uint32_t n = (uint32_t)((rs + HYOBFS_SALT_LEN + (M.hpl[v] >> 16) + 15) >> 4);
        for (uint32_t j0 = 0; j0 < n; j0 += 64) {
            const uint32_t j = j0 + lane;
            const gk_u128 ks = gk_ks_quad(P, (uint32_t)((A0 + 16ull * j) >> 6), lane & 3u);
            if (j < n) {
                gk_u128 r = 0;
                uint32_t cov = 0;
                gt_contrib(B, M, s_keyb, v, rs, (int32_t)(16u * j), [&] { return ks; }, r, cov);
                if (cov == 0xFFFFu)
                    store16_stream(B.out + A0 + 16u * j, r);
                else if (cov)
                    store_masked(B.out + A0 + 16u * j, r, cov);
            }
        }
    }
}

template <int SW>
void launch_gecko_tile_sw(const KeyParams& k, const hyobfs_gecko_batch& b, hipStream_t s) {
    const uint64_t blocks = div_up(b.n, kTileMaxD);
    hipLaunchKernelGGL((gecko_tile_kernel<SW>), dim3((uint32_t)blocks), dim3(256), 0, s, k, b);
}

}  // namespace hyobfs
