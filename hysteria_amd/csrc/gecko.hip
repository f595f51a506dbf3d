// gecko.hip -- Gecko framing kernels (include/hyobfs_gecko.h).
//
// Encode: one wavefront per group of 64 frames.  The wire datagram of frame f is
//     salt(8) || (hdr(5) || pad || chunk) ^ key_f[i % 32]
// (gecko_frame.go:39-61 encodeFrame, then salamander.go:59-72 Obfuscate).  Lane l
// loads frame l's record, offsets, salt and key once into LDS (and writes the
// salt); a wave scan numbers the group's 16-byte plaintext windows, and the 64
// lanes sweep the interior ones, several per lane in flight (loads first, then
// stores), each lane walking its window's frame forward through the LDS scan: a window
// inside the chunk is one unaligned 16-byte load, one inside the padding is two
// SplitMix64 words (pad byte at plaintext position q is stream byte f*2048 + q),
// each leaves as one 16-byte store.  Then lane l merges frame l's few edge windows
// (header, padding/chunk seam, frame end) under byte masks; keeping them out of
// the sweep keeps its lanes on the same path.  Lane l hashes frame l's key
// (BLAKE2b-256, salamander_device.h) in registers in step 1, so the hash overlaps
// other waves' sweeps (a separate keys_kernel pass via the workspace was 15 % slower).
//
// Parse: one thread per deobfuscated datagram, the checks of ReadFrom
// (gecko.go:170-193) and decodeFrame (gecko_frame.go:65-86) in their order.
#include "kernels.h"
#include "salamander_device.h"
#include "../../include/hyobfs_gecko.h"

namespace hyobfs {

__device__ __forceinline__ uint64_t gk_mix64(uint64_t z) {   // SplitMix64 finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

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
#define HY_GK_U 4
#endif
constexpr int kGkU = HY_GK_U;   // windows per lane in flight

struct GeckoGroup {             // one wave's 64 frames, in LDS
    uint64_t out_off[64];       // wire datagram start
    uint64_t chunk_off[64];
    uint64_t hdr[64];           // the 5 header bytes, little-endian in the low bytes
    uint32_t wstart[65];        // first plaintext window of the frame (exclusive scan), [64] = total
    uint32_t hp_plain[64];      // chunk start (low 16 bits) | plaintext length (high 16 bits)
    gk_u128 key[128];           // the frame's key, two halves
};

#ifdef HY_GK_WPE   // A/B builds only: register cap for the fused hash
#define HY_GK_ATTR __attribute__((amdgpu_waves_per_eu(HY_GK_WPE)))
#else
#define HY_GK_ATTR
#endif
__global__ __launch_bounds__(256) HY_GK_ATTR void gecko_encode_kernel(KeyParams K, hyobfs_gecko_batch B) {
    __shared__ GeckoGroup gg[4];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    GeckoGroup& G = gg[wid];
    const uint64_t f0 = ((uint64_t)blockIdx.x * 4 + wid) * 64;
    if (f0 >= B.n) return;
    // ---- 1. lane l: frame f0 + l's record, offsets, salt and key into LDS
    const uint64_t f = f0 + lane;
    uint32_t nwin = 0;
    if (f < B.n) {
        const hyobfs_gecko_frame fr = B.frames[f];
        const uint32_t total = fr.idx_total & 0x0f, idx = fr.idx_total >> 4;
        const uint32_t hp = HYOBFS_GECKO_HEADER_LEN + fr.pad_len;
        const uint64_t plain64 = (uint64_t)hp + fr.chunk_len;   // 64-bit: a hostile chunk_len must not wrap
        const uint32_t plain = (uint32_t)plain64;
        if (total >= HYOBFS_GECKO_MIN_CHUNKS && total <= HYOBFS_GECKO_MAX_CHUNKS && idx < total &&
            HYOBFS_SALT_LEN + plain64 <= HYOBFS_GECKO_BUFFER_SIZE) {   // else: skipped, nothing written
            nwin = (plain + 15) >> 4;
            const uint64_t oo = B.out_off[f];
            G.out_off[lane] = oo;
            G.chunk_off[lane] = fr.chunk_off;
            G.hdr[lane] = (uint64_t)HYOBFS_GECKO_FLAG_FRAGMENT | (uint64_t)fr.msg_id << 8 |
                          (uint64_t)fr.idx_total << 16 | (uint64_t)(fr.pad_len >> 8) << 24 |
                          (uint64_t)(fr.pad_len & 0xff) << 32;
            G.hp_plain[lane] = hp | plain << 16;
            const uint64_t salt = B.salts[f];
#ifdef HY_GK_KEYS_KERNEL   // A/B builds only: keys from keys_kernel via the workspace
            const uint8_t* kp = static_cast<const uint8_t*>(B.workspace) + 32 * f;
            gk_u128 k0, k1;
            __builtin_memcpy(&k0, kp, 16);
            __builtin_memcpy(&k1, kp + 16, 16);
#else   // keyLocked (salamander.go:88-91) in registers; the hash overlaps other waves' sweeps
            uint64_t kw[4];
            salamander_key(K, salt, kw);
            const gk_u128 k0 = (gk_u128)kw[1] << 64 | kw[0], k1 = (gk_u128)kw[3] << 64 | kw[2];
#endif
            G.key[2 * lane] = k0;
            G.key[2 * lane + 1] = k1;
            __builtin_memcpy(B.out + oo, &salt, HYOBFS_SALT_LEN);
        }
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
    auto pad16 = [&](uint32_t k, uint32_t p) -> gk_u128 {   // pad stream at plaintext [p, p+16) of frame f0+k
#ifdef HY_X_NOPAD   // ablation builds only (timing experiments; wrong output)
        return (gk_u128)(f0 + k + p);
#else
        const uint64_t w = ((f0 + k) * HYOBFS_GECKO_BUFFER_SIZE + p) >> 3;
        const uint64_t z0 = B.pad_seed + (w + 1) * 0x9e3779b97f4a7c15ull;   // SplitMix64 outputs w and w + 1
        return (gk_u128)gk_mix64(z0 + 0x9e3779b97f4a7c15ull) << 64 | gk_mix64(z0);
#endif
    };
    auto store = [&](uint32_t k, uint32_t p, uint32_t plain, gk_u128 v) {
        uint8_t* __restrict__ po = B.out + G.out_off[k] + HYOBFS_SALT_LEN;
        if (p + 16 <= plain) {
#ifdef HY_X_ALIGNST   // ablation builds only (timing experiments; wrong output)
            gk_store16u((uint8_t*)((uintptr_t)(po + p) & ~(uintptr_t)15), v);
#else
            gk_store16u(po + p, v);
#endif
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
        if (p == 0) v = (gk_u128)G.hdr[k] & gk_mask(0, min(e, (uint32_t)HYOBFS_GECKO_HEADER_LEN));
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
    // holds it (HY_GK_EDGES_INLINE, meant to let lines split between a frame's
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
#ifdef HY_GK_BSEARCH   // A/B builds only: the per-window binary search
            q = 0;
            if (t < tw) {
#pragma unroll
                for (uint32_t step = 32; step; step >>= 1) q = (G.wstart[q + step] <= t) ? q + step : q;
            }
#else
            if (t < tw)   // wstart[64] = tw > t stops the walk at frame 63
                while (G.wstart[q + 1] <= t) ++q;
#endif
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
#ifdef HY_GK_EDGES_INLINE   // A/B builds only: edges stored inside the sweep iteration
        if (emask) {
            const uint32_t ws = G.wstart[lane];
            uint32_t m = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if ((emask >> c & 1) && ws + cand(c) - T < 64u * kGkU) m |= 1u << c;
            edges(m);
        }
#endif
    }
#ifndef HY_GK_EDGES_INLINE   // ---- 3. all edge windows after the sweep
    edges(emask);
#endif
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
#ifdef HY_GK_KEYS_KERNEL
    hipError_t e = launch_keys(k, b.salts, static_cast<uint8_t*>(b.workspace), b.n, s);
    if (e != hipSuccess) return e;
#endif
    // (Instantiating per salt word as the wave kernel does cuts 96 -> 60 VGPRs, 5 -> 8
    // waves/SIMD, and measured 4 % slower: profiles/r01_ab_gecko/.)
    static const uint32_t lds_pad = [] {   // A/B only: unused dynamic LDS to cap workgroups per CU
        const char* e = std::getenv("HYOBFS_GK_LDS_PAD");
        return e ? (uint32_t)std::atoi(e) : 0u;
    }();
    hipLaunchKernelGGL(gecko_encode_kernel, dim3((uint32_t)((b.n + 255) / 256)), dim3(256), lds_pad, s, k, b);
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
