// salamander.hip -- gfx950 kernels for Hysteria's Salamander obfuscation.
//
// Reference semantics (apernet/hysteria): extras/obfs/salamander.go:59-91.
//   Obfuscate:   out = salt(8) || in[i] ^ key[i % 32]        (:59-72)
//   Deobfuscate: out[i] = in[8 + i] ^ key[i % 32], reject len <= 8  (:74-86)
//   key = BLAKE2b-256(PSK || salt)                              (:88-91)
//
// Kernel shape ("Kernels"): one 256-thread workgroup per tile of
// 256 datagrams.
//   Phase A: lane t owns datagram t of the tile.  It derives the output width
//            and offset (packed layout: wavefront scan of the widths plus the
//            tile's prefix), hashes PSK||salt with BLAKE2b in registers, and
//            stores the key -- pre-rotated to the output's 32-byte phase --
//            and the datagram's metadata in LDS.
//   Phase B: the tile's output bytes form one contiguous range.  All 256
//            lanes sweep it in 16-byte chunks, 64 consecutive chunks (1 KiB)
//            per wave instruction.  A chunk that lies inside one datagram's
//            payload is one unaligned 16-byte load, one LDS key read, four
//            XORs and one aligned 16-byte store.  Chunks at datagram edges
//            (salt bytes, two datagrams, tile edges) take the general path.
// No MFMA: there is no contraction; the kernel is HBM-bound (2L+16 bytes per
// obfuscated datagram).
#include "kernels.h"

namespace hyobfs {

// ------------------------------------------------------------------ BLAKE2b
// RFC 7693; golang.org/x/crypto@v0.54.0 blake2b.Sum256 is the reference's
// implementation (extras/go.mod:18).
__device__ constexpr uint64_t kIV[8] = {
    0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
    0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
    0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

__device__ constexpr uint8_t kSigma[12][16] = {
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

__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) {
    return (x >> n) | (x << (64 - n));
}

#define HY_G(a, b, c, d, x, y)           \
    do {                                 \
        v[a] = v[a] + v[b] + (x);        \
        v[d] = rotr64(v[d] ^ v[a], 32);  \
        v[c] = v[c] + v[d];              \
        v[b] = rotr64(v[b] ^ v[c], 24);  \
        v[a] = v[a] + v[b] + (y);        \
        v[d] = rotr64(v[d] ^ v[a], 16);  \
        v[c] = v[c] + v[d];              \
        v[b] = rotr64(v[b] ^ v[c], 63);  \
    } while (0)

// RFC 7693 section 3.2 F(h, m, t, f).  Fully unrolled: the message schedule
// folds to register indices, 96 G functions of 64-bit add/xor/rotate on the
// 32-bit VALU (v_add_co/v_addc, v_xor, v_alignbit).
__device__ __forceinline__ void b2b_compress(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                             bool last) {
    uint64_t v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = h[i];
        v[i + 8] = kIV[i];
    }
    v[12] ^= t;
    v[14] = last ? ~v[14] : v[14];
#pragma unroll
    for (int r = 0; r < 12; ++r) {
        HY_G(0, 4, 8, 12, m[kSigma[r][0]], m[kSigma[r][1]]);
        HY_G(1, 5, 9, 13, m[kSigma[r][2]], m[kSigma[r][3]]);
        HY_G(2, 6, 10, 14, m[kSigma[r][4]], m[kSigma[r][5]]);
        HY_G(3, 7, 11, 15, m[kSigma[r][6]], m[kSigma[r][7]]);
        HY_G(0, 5, 10, 15, m[kSigma[r][8]], m[kSigma[r][9]]);
        HY_G(1, 6, 11, 12, m[kSigma[r][10]], m[kSigma[r][11]]);
        HY_G(2, 7, 8, 13, m[kSigma[r][12]], m[kSigma[r][13]]);
        HY_G(3, 4, 9, 14, m[kSigma[r][14]], m[kSigma[r][15]]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}
#undef HY_G

// keyLocked (salamander.go:88-91): BLAKE2b-256(PSK || salt) from the host's
// PSK-only prefix state.  Returns the 4 little-endian key words.
__device__ __forceinline__ void salamander_key(const KeyParams& K, uint64_t salt, uint64_t key[4]) {
    const uint32_t sw = K.salt_pos >> 3;
    const uint32_t sb = (K.salt_pos & 7) * 8;
    const uint64_t lo = salt << sb;
    const uint64_t hi = sb ? (salt >> (64 - sb)) : 0ull;
    uint64_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = K.h[i];
    for (uint32_t b = 0; b < K.nblk; ++b) {
        uint64_t m[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t idx = 16 * b + j;
            uint64_t w = K.m[idx];
            w |= (idx == sw) ? lo : 0ull;
            w |= (idx == sw + 1) ? hi : 0ull;
            m[j] = w;
        }
        b2b_compress(h, m, K.t[b], b + 1 == K.nblk);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) key[i] = h[i];
}

// 256-bit rotate left by 8*r bits (r = 0..31): byte j of the result is byte
// (j - r) mod 32 of the key, so the result indexed by an output address
// modulo 32 gives the key byte of that address.
__device__ __forceinline__ void rotl_key_bytes(const uint64_t k[4], uint32_t r, uint64_t o[4]) {
    const uint32_t wr = r >> 3;
    const uint32_t s = (r & 7) * 8;
    uint64_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t a0 = k[i], a1 = k[(i + 3) & 3], a2 = k[(i + 2) & 3], a3 = k[(i + 1) & 3];
        w[i] = wr == 0 ? a0 : wr == 1 ? a1 : wr == 2 ? a2 : a3;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        o[i] = s ? ((w[i] << s) | (w[(i + 3) & 3] >> (64 - s))) : w[i];
}

// ------------------------------------------------------------------ helpers
typedef unsigned __int128 u128;

__device__ __forceinline__ u128 load16u(const uint8_t* p) {   // any alignment
    u128 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ uint64_t load8u(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
__device__ __forceinline__ u128 bytemask(uint32_t lo, uint32_t hi) {  // bytes [lo, hi), hi <= 16
    const uint32_t nb = hi - lo;
    const u128 ones = ~(u128)0;
    const u128 m = nb >= 16 ? ones : (((u128)1 << (8 * nb)) - 1);
    return m << (8 * lo);
}

template <bool OBF>
__device__ __forceinline__ uint32_t out_width(uint32_t L, uint32_t cap) {
    if (L > kMaxDatagram) return 0;
    if (OBF) {
        const uint32_t W = L + 8;                       // salamander.go:60
        return (cap == 0 || W <= cap) ? W : 0u;          // :61-62
    } else {
        if (L <= 8) return 0;                           // :75-76, outLen <= 0
        const uint32_t W = L - 8;
        return (cap == 0 || W <= cap) ? W : 0u;          // :76-77
    }
}

__device__ __forceinline__ uint32_t pkt_len(const BatchParams& B, uint64_t p) {
    return B.in_len ? B.in_len[p] : B.len_uniform;
}
__device__ __forceinline__ uint64_t pkt_in_off(const BatchParams& B, uint64_t p) {
    return B.in_off ? B.in_off[p] : p * B.in_stride;
}

// wavefront-inclusive scan (64 lanes)
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x = max(x, (uint32_t)__shfl_xor(x, d, 64));
    return x;
}

// ------------------------------------------------------ packed-layout scan
// Tile sums of the output widths; the main kernel adds a wavefront scan.
template <bool OBF>
__global__ __launch_bounds__(kTile) void tile_sums_kernel(BatchParams B) {
    __shared__ uint64_t s_w[kTile / 64];
    const uint64_t p = (uint64_t)blockIdx.x * kTile + threadIdx.x;
    uint32_t W = 0;
    if (p < B.n) W = out_width<OBF>(pkt_len(B, p), B.pkt_cap);
    const uint64_t ws = wave_sum(W);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = ws;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
#pragma unroll
        for (int i = 0; i < kTile / 64; ++i) s += s_w[i];
        B.tile_sums[blockIdx.x] = s;
    }
}

// Exclusive scan of ntiles values in place, one workgroup of 1024 threads;
// writes the total at [ntiles].
__global__ __launch_bounds__(1024) void scan_tiles_kernel(uint64_t* v, uint64_t ntiles) {
    __shared__ uint64_t s_w[16];
    __shared__ uint64_t s_carry;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    if (t == 0) s_carry = 0;
    __syncthreads();
    for (uint64_t base = 0; base < ntiles; base += 1024) {
        const uint64_t i = base + t;
        const uint64_t x = i < ntiles ? v[i] : 0;
        const uint64_t inc = wave_incl_scan(x, lane);
        if (lane == 63) s_w[wid] = inc;
        __syncthreads();
        uint64_t wpre = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            const uint64_t sw = s_w[w];
            wpre += (w < wid) ? sw : 0;
            tot += sw;
        }
        const uint64_t carry = s_carry;
        if (i < ntiles) v[i] = carry + wpre + inc - x;
        __syncthreads();
        if (t == 0) s_carry = carry + tot;
        __syncthreads();
    }
    if (t == 0) v[ntiles] = s_carry;
}

// --------------------------------------------------------------- main kernel
template <bool OBF, bool PACKED>
__global__ __launch_bounds__(kTile) void salamander_kernel(BatchParams B, KeyParams K) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;   // bytes of salt in front of the output payload
    constexpr uint32_t SKIP = OBF ? 0u : 8u;   // bytes of salt in front of the input payload
    constexpr int U = 4;                        // chunks in flight per lane

    __shared__ uint32_t s_ooff[kTile];    // output region start, tile-relative
    __shared__ uint32_t s_wlen[kTile];    // output region width (0 = dropped)
    __shared__ uint64_t s_ioff[kTile];    // input payload start (absolute byte offset)
    __shared__ uint64_t s_salt[kTile];    // salt (obfuscate)
    __shared__ uint4 s_key[2 * kTile];    // key rotated to the output phase, 2 halves
    __shared__ uint64_t s_red[kTile / 64];
    __shared__ uint32_t s_redm[kTile / 64];

    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const uint64_t tile = blockIdx.x;
    const uint64_t p0 = tile * kTile;
    const uint32_t cnt = (uint32_t)min<uint64_t>((uint64_t)kTile, B.n - p0);
    const uint64_t p = p0 + t;
    const bool live = (uint32_t)t < cnt;

    // ---------------- phase A: widths, offsets, keys
    uint32_t L = 0, W = 0;
    uint64_t ioff = 0;
    if (live) {
        L = pkt_len(B, p);
        ioff = pkt_in_off(B, p);
        W = out_width<OBF>(L, B.pkt_cap);
    }
    uint64_t ooff, first_off;
    if (PACKED) {
        const uint64_t inc = wave_incl_scan(W, lane);
        if (lane == 63) s_red[wid] = inc;
        __syncthreads();
        uint64_t wpre = 0;
#pragma unroll
        for (int w = 0; w < kTile / 64; ++w) wpre += (w < wid) ? s_red[w] : 0;
        first_off = B.tile_prefix[tile];
        ooff = first_off + wpre + inc - W;
        __syncthreads();   // s_red reused below
    } else {
        ooff = p * B.out_stride;
        first_off = p0 * B.out_stride;
    }
    if (W && ooff + W > B.out_cap) W = 0;   // does not fit: dropped, offsets unchanged
    if (live) {
        if (B.out_off) B.out_off[p] = ooff;
        if (B.out_len) B.out_len[p] = W;
    }
    const uint64_t tile_base = first_off & ~15ull;
    const uint32_t rel = live ? (uint32_t)(ooff - tile_base) : 0xFFFFFFFFu;

    uint64_t salt = 0;
    if (W) salt = OBF ? B.salts[p] : load8u(B.in + ioff);
    uint64_t kr[4] = {0, 0, 0, 0};
    if (W) {
        uint64_t key[4];
        salamander_key(K, salt, key);
        rotl_key_bytes(key, (rel + SALT) & 31u, kr);
    }
    s_ooff[t] = rel;
    s_wlen[t] = W;
    s_ioff[t] = ioff + SKIP;
    s_salt[t] = salt;
    s_key[2 * t] = make_uint4((uint32_t)kr[0], (uint32_t)(kr[0] >> 32), (uint32_t)kr[1],
                              (uint32_t)(kr[1] >> 32));
    s_key[2 * t + 1] = make_uint4((uint32_t)kr[2], (uint32_t)(kr[2] >> 32), (uint32_t)kr[3],
                                  (uint32_t)(kr[3] >> 32));
    // tile extent and bytes written
    const uint32_t endm = wave_max(W ? rel + W : 0u);
    const uint64_t wsum = wave_sum(W);
    if (lane == 0) {
        s_redm[wid] = endm;
        s_red[wid] = wsum;
    }
    __syncthreads();
    uint32_t tile_end = 0;
    uint64_t tile_written = 0;
#pragma unroll
    for (int w = 0; w < kTile / 64; ++w) {
        tile_end = max(tile_end, s_redm[w]);
        tile_written += s_red[w];
    }
    if (t == 0 && B.out_total && tile_written) atomicAdd(B.out_total, (unsigned long long)tile_written);

    // ---------------- phase B: sweep the tile's output in 16-byte chunks
    const uint32_t nchunks = (tile_end + 15u) >> 4;
    const uint32_t d0 = (uint32_t)(first_off - tile_base);
    uint8_t* __restrict__ outb = B.out + tile_base;
    const uint8_t* __restrict__ in = B.in;

    for (uint32_t c0 = 0; c0 < nchunks; c0 += kTile * U) {
        uint32_t qv[U];
        bool fast[U];
        u128 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * kTile + t;
            const uint32_t a = c << 4;
            uint32_t q;
            if (PACKED) {   // last datagram whose region starts at or before a
                q = 0;
#pragma unroll
                for (uint32_t step = kTile / 2; step; step >>= 1)
                    q = (s_ooff[q + step] <= a) ? q + step : q;
            } else {
                uint32_t x = a >= d0 ? a - d0 : 0u;
                q = (uint32_t)((double)x * B.inv_stride);
                const uint64_t st = B.out_stride;
                if ((uint64_t)(q + 1) * st <= x) ++q;
                if ((uint64_t)q * st > x) --q;
                q = min(q, cnt - 1);
            }
            qv[u] = q;
            const uint32_t oq = s_ooff[q], wq = s_wlen[q];
            const uint32_t op = oq + SALT;
            fast[u] = (c < nchunks) && wq != 0 && op <= a && a + 16 <= oq + wq;
            v[u] = 0;
            if (fast[u]) v[u] = load16u(in + s_ioff[q] + (a - op));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * kTile + t;
            if (c >= nchunks) continue;
            const uint32_t a = c << 4;
            uint32_t q = qv[u];
            if (fast[u]) {
                const uint4 kk = s_key[2 * q + ((a >> 4) & 1)];
                u128 k128;
                __builtin_memcpy(&k128, &kk, 16);
                const u128 r = v[u] ^ k128;
                __builtin_memcpy(outb + a, &r, 16);   // 16-byte aligned
                continue;
            }
            // general path: salt bytes, several datagrams, tile edges, tiny datagrams
            u128 r = 0;
            uint32_t cov = 0;
            for (; q < cnt; ++q) {
                const uint32_t oq = s_ooff[q];
                if (oq >= a + 16) break;
                const uint32_t wq = s_wlen[q];
                if (wq == 0 || oq + wq <= a) continue;
                if (OBF) {   // salt bytes [oq, oq+8)
                    const uint32_t sb = max(oq, a), se = min(oq + 8u, a + 16u);
                    if (sb < se) {
                        u128 S = (u128)s_salt[q];
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
                    const uint8_t* src = in + s_ioff[q];
                    u128 X = 0;
                    if (PL >= 16) {
                        const int ws = min(max(base, 0), (int)PL - 16);
                        const u128 V = load16u(src + ws);
                        const int d = ws - base;
                        X = d >= 0 ? (V << (8 * d)) : (V >> (8 * -d));
                    } else {
                        for (uint32_t j = ps - a; j < pe - a; ++j)
                            X |= (u128)src[base + (int)j] << (8 * j);
                    }
                    const uint4 kk = s_key[2 * q + ((a >> 4) & 1)];
                    u128 k128;
                    __builtin_memcpy(&k128, &kk, 16);
                    r |= (X ^ k128) & bytemask(ps - a, pe - a);
                    cov |= ((1u << (pe - ps)) - 1u) << (ps - a);
                }
            }
            if (cov == 0xFFFFu) {
                __builtin_memcpy(outb + a, &r, 16);
            } else if (cov) {   // bytes owned by a neighbouring tile or a gap stay untouched
#pragma unroll
                for (int dw = 0; dw < 4; ++dw) {
                    const uint32_t m4 = (cov >> (4 * dw)) & 0xFu;
                    const uint32_t word = (uint32_t)(r >> (32 * dw));
                    if (m4 == 0xFu) {
                        *reinterpret_cast<uint32_t*>(outb + a + 4 * dw) = word;
                    } else if (m4) {
                        for (int b = 0; b < 4; ++b)
                            if (m4 & (1u << b)) outb[a + 4 * dw + b] = (uint8_t)(word >> (8 * b));
                    }
                }
            }
        }
    }
}

// keys only (hyobfs_salamander_key): key[i] = BLAKE2b-256(PSK || salts[i])
__global__ __launch_bounds__(256) void keys_kernel(KeyParams K, const uint64_t* salts, uint8_t* keys,
                                                   uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k[4];
    salamander_key(K, salts[i], k);
#pragma unroll
    for (int w = 0; w < 4; ++w) __builtin_memcpy(keys + 32 * i + 8 * w, &k[w], 8);
}

// ------------------------------------------------------- synthetic inputs
__device__ __forceinline__ uint64_t sm64_at(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// dst[b] = byte (start + b) of the little-endian SplitMix64(seed) stream.
// dst is 16-byte aligned; each thread writes 16 bytes.
__global__ void synth_stream_kernel(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t start) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t b0 = 16 * i;
    if (b0 >= nbytes) return;
    const uint64_t g = start + b0;
    const uint64_t w = g >> 3;
    const uint32_t s = (uint32_t)(g & 7) * 8;
    const uint64_t x0 = sm64_at(seed, w), x1 = sm64_at(seed, w + 1), x2 = sm64_at(seed, w + 2);
    const uint64_t lo = s ? (x0 >> s) | (x1 << (64 - s)) : x0;
    const uint64_t hi = s ? (x1 >> s) | (x2 << (64 - s)) : x1;
    if (b0 + 16 <= nbytes) {
        *reinterpret_cast<uint64_t*>(dst + b0) = lo;
        *reinterpret_cast<uint64_t*>(dst + b0 + 8) = hi;
    } else {
        for (uint64_t j = 0; b0 + j < nbytes; ++j)
            dst[b0 + j] = (uint8_t)((j < 8 ? lo >> (8 * j) : hi >> (8 * (j - 8))));
    }
}

__global__ void synth_u64_kernel(uint64_t* dst, uint64_t n, uint64_t seed, uint64_t first) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = sm64_at(seed, first + i);
}

__global__ void synth_bimodal_kernel(uint32_t* dst, uint64_t n, uint64_t seed, uint64_t first) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = (sm64_at(seed, first + i) % 5) < 2 ? 64u : 1350u;
}

// ------------------------------------------------------------------ launchers
static inline uint64_t div_up(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

hipError_t launch_salamander(bool obf, const BatchParams& b, const KeyParams& k, hipStream_t s) {
    if (b.n == 0) return hipSuccess;
    const uint64_t ntiles = div_up(b.n, kTile);
    if (ntiles > 0x7fffffffull) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)ntiles), block(kTile);
    BatchParams bp = b;
    if (b.out_stride == 0) {
        if (obf)
            hipLaunchKernelGGL(tile_sums_kernel<true>, grid, block, 0, s, bp);
        else
            hipLaunchKernelGGL(tile_sums_kernel<false>, grid, block, 0, s, bp);
        hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(1024), 0, s, bp.tile_sums, ntiles);
        bp.tile_prefix = bp.tile_sums;
        if (obf)
            hipLaunchKernelGGL((salamander_kernel<true, true>), grid, block, 0, s, bp, k);
        else
            hipLaunchKernelGGL((salamander_kernel<false, true>), grid, block, 0, s, bp, k);
    } else {
        bp.inv_stride = 1.0 / (double)b.out_stride;
        if (obf)
            hipLaunchKernelGGL((salamander_kernel<true, false>), grid, block, 0, s, bp, k);
        else
            hipLaunchKernelGGL((salamander_kernel<false, false>), grid, block, 0, s, bp, k);
    }
    return hipGetLastError();
}

hipError_t launch_keys(const KeyParams& k, const uint64_t* salts, uint8_t* keys, uint64_t n,
                       hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(keys_kernel, dim3((uint32_t)div_up(n, 256)), dim3(256), 0, s, k, salts, keys, n);
    return hipGetLastError();
}

hipError_t launch_synth_stream(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t start,
                               hipStream_t s) {
    if (nbytes == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_stream_kernel, dim3((uint32_t)div_up(div_up(nbytes, 16), 256)), dim3(256),
                       0, s, dst, nbytes, seed, start);
    return hipGetLastError();
}

hipError_t launch_synth_u64(uint64_t* dst, uint64_t n, uint64_t seed, uint64_t first, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_u64_kernel, dim3((uint32_t)div_up(n, 256)), dim3(256), 0, s, dst, n, seed,
                       first);
    return hipGetLastError();
}

hipError_t launch_synth_bimodal(uint32_t* dst, uint64_t n, uint64_t seed, uint64_t first,
                                hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_bimodal_kernel, dim3((uint32_t)div_up(n, 256)), dim3(256), 0, s, dst, n,
                       seed, first);
    return hipGetLastError();
}

}  // namespace hyobfs
