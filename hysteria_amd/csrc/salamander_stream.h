// salamander_stream.h -- the stream kernel: a CONTIGUOUS packed input (datagram i
// at in + in_len[0] + ... + in_len[i-1], include/hyobfs.h) to packed output
// (gfx950).  The layout of BASELINE configs[2] and of any batch that arrives
// back to back (GRO-style receive buffers, a sender's queue copied into one
// buffer).
//
// Reference: extras/obfs/salamander.go:59-91 (Obfuscate, Deobfuscate, keyLocked).
//
// Because the input is contiguous, the input bytes behind any contiguous range of
// output bytes are one contiguous range too.  The output is cut into tiles of kST
// bytes (16 KiB, 128-byte aligned: every output line is written whole, by one
// workgroup, in one store instruction):
//   1. prepass (three launches): block sums of lengths and widths, their scan,
//      then per datagram its input and output offset (out_off / out_len) and,
//      for the datagram holding each tile's first output byte, the tile's
//      descriptor (that datagram, its offsets, the tile's first input byte);
//   2. stream kernel: one workgroup of four waves per tile.  Waves 2-3 copy the
//      tile's input range into LDS by LDS-DMA (one contiguous range, known from
//      the descriptors alone, 1 KiB per wave instruction, non-temporal) while
//      waves 0-1 load the lengths and salts of the tile's datagrams, scan them and
//      hash the keys, four lanes per key (quad_key, salamander_tile.h), rotated to
//      the output's 32-byte phase; after one barrier the chunks that hold a salt or
//      a datagram edge are assembled and parked in LDS, and all 256 threads sweep
//      the tile's output in 16-byte chunks (payload bytes from LDS, key XOR, one
//      aligned non-temporal 16-byte store each).  The workgroup exits with its
//      stores in flight.  (A persistent loop over tiles measured 2.39 ms against
//      1.48 ms for the wave kernel on configs[2]: each tile's chain started by
//      waiting for the previous tile's stores, profiles/r04a_ab_bimodal_*.txt.)
// A tile with more than 64 datagrams runs in passes of 64; a tile whose input
// span does not fit the LDS stage (long dropped datagrams between its valid
// ones) reads its payload bytes straight from global memory.  Both are correct
// and slower; neither occurs for input without drops and datagrams of >= 256 B
// on average.
#pragma once
#include "salamander_tile.h"

namespace hyobfs {

#ifndef HY_STREAM_T
#define HY_STREAM_T 16384
#endif
constexpr uint32_t kST = HY_STREAM_T;          // output bytes per tile (multiple of 128)
static_assert(kST % 128 == 0, "tiles must be whole 128-byte lines");
constexpr int kSD = 64;                        // datagrams per pass
constexpr uint32_t kSIn = kST + 1024;          // staged input bytes (deobfuscate: + the tile's salts)
constexpr uint32_t kSGuard = 16;               // LDS bytes before the stage (funnel reads at pos >= -16)
constexpr int kSBlk = 1024;                    // datagrams per prepass block (256 threads x 4)
#ifndef HY_STREAM_U
#define HY_STREAM_U 2
#endif
constexpr int kSU = HY_STREAM_U;               // sweep chunks per thread in flight

struct StreamDesc {      // one output tile (or the tail record)
    uint64_t d;          // the datagram holding the tile's first output byte (tail: end of the valid ones)
    uint64_t s;          // its input start
    uint64_t o;          // its output start (tail: end of the valid output)
    uint64_t in0;        // input position of the tile's first payload byte (tail: input end)
};

struct StreamParams {
    StreamDesc* desc;          // ntiles_max + 1 (the tail record at [ntiles_max])
    uint64_t* bsum;            // 2 x (nblocks + 1): per block sum of lengths, of widths; then their scan
    uint64_t* in_off_out;      // optional: input offsets (for the wave kernel fallback)
    uint64_t ntiles_max;       // ceil(out_cap / kST)
    uint64_t nblocks;
    int write_out;             // the prepass writes out_off / out_len (the stream kernel runs next)
};

// ------------------------------------------------------------------ prepass
// 1. per block of 1024 datagrams: sum of lengths and of widths
template <bool OBF>
__global__ __launch_bounds__(256) void stream_sums_kernel(BatchParams B, StreamParams S) {
    __shared__ uint64_t s_l[4], s_w[4];
    const uint32_t tid = threadIdx.x;
    const uint64_t p0 = (uint64_t)blockIdx.x * kSBlk + 4ull * tid;
    uint64_t sl = 0, sw = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (p0 + k < B.n) {
            const uint32_t L = B.in_len[p0 + k];
            sl += L;
            sw += out_width<OBF>(L, B.pkt_cap);
        }
    }
    sl = wave_sum(sl);
    sw = wave_sum(sw);
    if ((tid & 63) == 0) {
        s_l[tid >> 6] = sl;
        s_w[tid >> 6] = sw;
    }
    __syncthreads();
    if (tid == 0) {
        S.bsum[2 * blockIdx.x] = s_l[0] + s_l[1] + s_l[2] + s_l[3];
        S.bsum[2 * blockIdx.x + 1] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    }
}

// 2. exclusive scan of the (length, width) block sums in place, one workgroup;
// the totals go to [nblocks] and into the default tail record (no datagram cut
// by out_cap; stream_locate_kernel overwrites it when one is)
template <bool OBF>   // (a template: this header is compiled into several translation units)
__global__ __launch_bounds__(1024) void stream_scan_kernel(BatchParams B, StreamParams S) {
    constexpr int PER = 8;
    __shared__ uint64_t s_w[2][16];
    __shared__ uint64_t s_carry[2];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    if (t < 2) s_carry[t] = 0;
    __syncthreads();
    for (uint64_t base = 0; base < S.nblocks; base += 1024 * PER) {
        const uint64_t i0 = base + (uint64_t)t * PER;
        uint64_t xl[PER], xw[PER], suml = 0, sumw = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const bool in = i0 + k < S.nblocks;
            xl[k] = in ? S.bsum[2 * (i0 + k)] : 0;
            xw[k] = in ? S.bsum[2 * (i0 + k) + 1] : 0;
            suml += xl[k];
            sumw += xw[k];
        }
        const uint64_t incl = wave_incl_scan(suml, lane), incw = wave_incl_scan(sumw, lane);
        if (lane == 63) {
            s_w[0][wid] = incl;
            s_w[1][wid] = incw;
        }
        __syncthreads();
        uint64_t pl = 0, pw = 0, tl = 0, tw = 0;
        for (int w = 0; w < 16; ++w) {
            pl += (w < wid) ? s_w[0][w] : 0;
            pw += (w < wid) ? s_w[1][w] : 0;
            tl += s_w[0][w];
            tw += s_w[1][w];
        }
        uint64_t rl = s_carry[0] + pl + incl - suml, rw = s_carry[1] + pw + incw - sumw;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            if (i0 + k < S.nblocks) {
                S.bsum[2 * (i0 + k)] = rl;
                S.bsum[2 * (i0 + k) + 1] = rw;
            }
            rl += xl[k];
            rw += xw[k];
        }
        __syncthreads();
        if (t == 0) {
            s_carry[0] += tl;
            s_carry[1] += tw;
        }
        __syncthreads();
    }
    if (t == 0) {
        S.bsum[2 * S.nblocks] = s_carry[0];
        S.bsum[2 * S.nblocks + 1] = s_carry[1];
    }
    if (t == 0 && S.desc) {
        StreamDesc tail;
        tail.d = B.n;
        tail.s = s_carry[0];
        tail.o = s_carry[1];
        tail.in0 = s_carry[0];
        S.desc[S.ntiles_max] = tail;
    }
}

// 3. per datagram: input and output offsets (the reference's return values into
// out_off / out_len), and the descriptor of every tile whose first output byte it
// holds.  Valid = width > 0 and the region ends inside out_cap; the first
// datagram that does not fit ends the valid output (packed: offsets never move,
// every later one is dropped too) and writes the tail record.
template <bool OBF>
__global__ __launch_bounds__(256) void stream_locate_kernel(BatchParams B, StreamParams S) {
    constexpr uint32_t SALT = OBF ? 8u : 0u;
    __shared__ uint64_t s_l[4], s_w[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t p0 = (uint64_t)blockIdx.x * kSBlk + 4ull * tid;
    uint32_t L[4], W[4];
    uint64_t sl = 0, sw = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        L[k] = p0 + k < B.n ? B.in_len[p0 + k] : 0u;
        W[k] = p0 + k < B.n ? out_width<OBF>(L[k], B.pkt_cap) : 0u;
        sl += L[k];
        sw += W[k];
    }
    const uint64_t il = wave_incl_scan(sl, (int)lane), iw = wave_incl_scan(sw, (int)lane);
    if (lane == 63) {
        s_l[wid] = il;
        s_w[wid] = iw;
    }
    __syncthreads();
    uint64_t s = S.bsum[2 * blockIdx.x] + il - sl, o = S.bsum[2 * blockIdx.x + 1] + iw - sw;
    for (uint32_t w = 0; w < wid; ++w) {
        s += s_l[w];
        o += s_w[w];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t p = p0 + k;
        if (p < B.n) {
            const bool fits = W[k] && o + W[k] <= B.out_cap;
            if (S.write_out && B.out_off) B.out_off[p] = o;
            if (S.write_out && B.out_len) B.out_len[p] = fits ? W[k] : 0u;
            if (S.in_off_out) S.in_off_out[p] = s;
            if (fits && S.desc) {   // tiles whose first byte lies in [o, o + W)
                for (uint64_t t = (o + kST - 1) / kST; t * kST < o + W[k]; ++t) {
                    const uint64_t tT = t * kST;
                    StreamDesc d;
                    d.d = p;
                    d.s = s;
                    d.o = o;
                    d.in0 = OBF ? s + (tT > o + SALT ? tT - o - SALT : 0) : s + 8 + (tT - o);
                    S.desc[t] = d;
                }
            } else if (W[k] && o <= B.out_cap && S.desc) {   // the first datagram past out_cap: the valid output ends at o
                StreamDesc d;
                d.d = p;
                d.s = s;
                d.o = o;
                d.in0 = s;
                S.desc[S.ntiles_max] = d;
            }
        }
        s += L[k];
        o += W[k];
    }
}

// ------------------------------------------------------------- stream kernel
struct StreamLDS {
    uint8_t in[kSGuard + kSIn + 32];   // the tile's staged input, stage byte 0 at in[kSGuard]
    uint64_t key[kSD * 4];             // keys rotated to the output's 32-byte phase
    uint64_t salt[kSD];
    int64_t src[kSD];                  // stage position of payload byte 0 (staged) / absolute input position
    int32_t o[kSD + 1];                // output start relative to the tile; [mp..] = INT_MAX (searches)
    uint32_t w[kSD];                   // width (0: dropped)
    u128 park[3 * kSD];                // assembled boundary chunks: datagram k's candidate t at 3k + t
    uint8_t parked[3 * kSD];
};

// 16 bytes of the stage at position pos (>= -16) from two aligned ds_read_b128
__device__ __forceinline__ u128 stage16(const StreamLDS& S, int32_t pos) {
    const int32_t q = pos + (int32_t)kSGuard;
    const int32_t a = q & ~15;
    const uint32_t sh = (uint32_t)(q & 15);
    const u128 A = *reinterpret_cast<const u128*>(S.in + a);
    if (!sh) return A;
    const u128 Bv = *reinterpret_cast<const u128*>(S.in + a + 16);
    return (A >> (8 * sh)) | (Bv << (128 - 8 * sh));
}

__device__ __forceinline__ u128 key16(const StreamLDS& S, uint32_t k, int32_t x) {
    const uint32_t i = 4 * k + 2 * (((uint32_t)x >> 4) & 1u);
    return (u128)S.key[i + 1] << 64 | S.key[i];
}

// Payload bytes of datagram k for the 16-byte chunk whose chunk byte 0 is payload
// index base (any sign; bytes outside the payload are garbage, masked by the caller).
template <bool OBF>
__device__ __forceinline__ u128 payload16(const StreamLDS& S, const uint8_t* __restrict__ in, bool staged, uint32_t k,
                                          int32_t base) {
    if (staged) return stage16(S, (int32_t)S.src[k] + base);
    constexpr uint32_t SALT = OBF ? 8u : 0u;
    const int32_t PL = (int32_t)(S.w[k] - SALT);
    const uint8_t* src = in + S.src[k];
    if (PL >= 16) {   // one in-bounds window, shifted into place
        const int32_t ws = min(max(base, 0), PL - 16);
        const u128 V = load16u(src + ws);
        const int32_t d = ws - base;
        return d >= 0 ? (V << (8 * d)) : (V >> (8 * -d));
    }
    u128 X = 0;
    for (int32_t j = max(base, 0); j < min(base + 16, PL); ++j) X |= (u128)src[j] << (8 * (j - base));
    return X;
}

// All bytes datagram k contributes to the chunk at tile-relative x.
template <bool OBF>
__device__ __forceinline__ void stream_contrib(const StreamLDS& S, const uint8_t* __restrict__ in, bool staged,
                                               uint32_t k, int32_t x, u128& r, uint32_t& cov) {
    constexpr int32_t SALT = OBF ? 8 : 0;
    const uint32_t W = S.w[k];
    const int32_t o = S.o[k];
    if (W == 0 || o >= x + 16 || o + (int32_t)W <= x) return;
    if (OBF) {   // salt bytes [o, o + 8)
        const int32_t sb = max(o, x), se = min(o + 8, x + 16);
        if (sb < se) {
            u128 Sv = (u128)S.salt[k];
            Sv = o >= x ? (Sv << (8 * (o - x))) : (Sv >> (8 * (x - o)));
            r |= Sv & bytemask((uint32_t)(sb - x), (uint32_t)(se - x));
            cov |= ((1u << (se - sb)) - 1u) << (sb - x);
        }
    }
    const int32_t ps = max(o + SALT, x), pe = min(o + (int32_t)W, x + 16);
    if (ps < pe) {
        const u128 X = payload16<OBF>(S, in, staged, k, x - (o + SALT));
        r |= (X ^ key16(S, k, x)) & bytemask((uint32_t)(ps - x), (uint32_t)(pe - x));
        cov |= ((1u << (pe - ps)) - 1u) << (ps - x);
    }
}

// Boundary candidates of datagram k (chunk indices relative to the tile): the
// chunk of its first byte, of its first payload byte, of its last byte.
__device__ __forceinline__ int32_t stream_cand(int32_t o, uint32_t W, int32_t salt, int t) {
    return t == 0 ? (o >> 4) : t == 1 ? ((o + salt) >> 4) : ((o + (int32_t)W - 1) >> 4);
}

#ifndef HY_STREAM_WAVES
#define HY_STREAM_WAVES 5   // min waves per SIMD (the LDS allows 6 workgroups of 24 KB per CU)
#endif
#ifndef HY_STREAM_LAUNCH_TILES
#define HY_STREAM_LAUNCH_TILES 65536   // tiles per launch (1 GiB of output): the XCDs stay close in the address space
#endif
// One workgroup per output tile (tile t0 + blockIdx.x).  The chain per tile is the
// uniform tile kernel's: the descriptors, then at once waves 2-3 issue the input
// window's LDS-DMA while waves 0-1 load lengths and salts, scan and hash the keys;
// one barrier; boundary chunks; one barrier; the sweep, and the workgroup exits with
// its stores in flight (no wave ever waits for its own stores).
template <bool OBF, int SW>
__global__ __launch_bounds__(256, HY_STREAM_WAVES) void salamander_stream_kernel(BatchParams B, KeyParams K,
                                                                                  StreamParams SP, uint64_t t0) {
    constexpr int32_t SALT = OBF ? 8 : 0;   // salt bytes in front of the output payload
    constexpr int64_t SKIP = OBF ? 0 : 8;   // salt bytes in front of the input payload
    __shared__ __attribute__((aligned(16))) StreamLDS S;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = uni32(tid >> 6);
    const uint8_t* __restrict__ in = B.in;

    // the tail record: end of the valid output (and of the datagrams and input)
    const StreamDesc* __restrict__ D = SP.desc;
    const uint64_t E = D[SP.ntiles_max].o;
    const uint64_t ntiles = (E + kST - 1) / kST;
    const uint64_t t = t0 + blockIdx.x;
    if (t == 0 && tid == 0 && B.out_total) *B.out_total = E;
    if (t >= ntiles) return;
    // this tile's descriptor and the next one's (or the tail)
    const StreamDesc* __restrict__ pc = &D[t];
    const StreamDesc* __restrict__ pn = &D[t + 1 < ntiles ? t + 1 : SP.ntiles_max];
    const uint64_t d0 = pc->d, s0 = pc->s, o0 = pc->o, in_lo = pc->in0;
    const uint64_t nd = pn->d, no = pn->o, in_hi = pn->in0;
    const uint64_t tT = t * kST;
    const bool last = t + 1 == ntiles;
    // the tile's datagrams [d0, dend): the next tile's first datagram belongs here
    // too when it starts inside this tile
    const uint64_t dend = last ? nd : nd + (no < tT + kST ? 1 : 0);
    const uint32_t tile_len = (uint32_t)(last ? E - tT : kST);
    const uint64_t base16 = in_lo & ~15ull;
    const uint64_t span = ((in_hi + 15) & ~15ull) - base16;
    const bool staged = span <= kSIn;

    // ---- waves 2-3: the tile's input range into LDS (LDS-DMA, 1 KiB per instruction)
    if (wid >= 2 && staged) {
        const uint32_t nch = (uint32_t)(span >> 4);
        for (uint32_t i = wid - 2; i * 64u < nch; i += 2) {
            const uint32_t ch = i * 64u + lane;
            if (ch < nch) glds16(in + base16 + 16u * ch, S.in + kSGuard + 1024u * i);
        }
    }
    uint64_t sfirst = s0, ofirst = o0;   // offsets of the pass's first datagram
    for (uint64_t g0 = d0; g0 < dend; g0 += kSD) {
        const uint32_t mp = (uint32_t)min<uint64_t>((uint64_t)kSD, dend - g0);
        // ---- every wave: lengths, widths and offsets of the pass's datagrams (lane k:
        // datagram g0 + k); wave 0 publishes them
        const uint64_t j = g0 + lane;
        const bool live = lane < mp;
        // this wave's key slice: datagram 16 wid + lane / 4 (its salt loads with the lengths)
        const uint32_t k = 16u * wid + (lane >> 2), qi = lane & 3u;
        const uint32_t kk = k < mp ? k : 16u * wid;
        uint64_t salt = 0;
        if (OBF && 16u * wid < mp) salt = B.salts[g0 + kk];
        const uint32_t L = live ? B.in_len[j] : 0u;
        const uint32_t W = live ? out_width<OBF>(L, B.pkt_cap) : 0u;
        const uint64_t il = wave_incl_scan((uint64_t)L, (int)lane), iw = wave_incl_scan((uint64_t)W, (int)lane);
        const uint64_t s = sfirst + il - L, o = ofirst + iw - W;
        sfirst += uni64(__shfl(il, 63, 64));
        ofirst += uni64(__shfl(iw, 63, 64));
        if (wid == 0) {
            S.o[lane] = live ? (int32_t)((int64_t)o - (int64_t)tT) : 0x7FFFFFFF;
            if (lane == 0) S.o[kSD] = 0x7FFFFFFF;
            S.w[lane] = W;
            S.src[lane] = staged ? (int64_t)(s + SKIP) - (int64_t)base16 : (int64_t)(s + SKIP);
        }
        // ---- keys: wave w hashes datagrams 16w .. 16w + 15, four lanes each, rotated
        // to the output phase (key byte of output byte x at x mod 32)
        if (16u * wid < mp) {
            if (!OBF) {   // the wire's salt
                const uint64_t sk = __shfl(s, (int)kk, 64);
                const uint32_t Wk = __shfl(W, (int)kk, 64);
                salt = Wk ? load8u(in + sk) : 0;
            }
            const uint64_t okk = __shfl(o, (int)kk, 64);
            const uint64_t kw = quad_key<SW>(K, salt, qi);
            const uint32_t r = ((uint32_t)okk + (uint32_t)SALT) & 31u;
            const uint32_t st = (8u * qi - r) & 31u, w0 = st >> 3, sh = (st & 7u) * 8u;
            const uint64_t a = __shfl(kw, (int)((lane & ~3u) | w0), 64);
            const uint64_t b = __shfl(kw, (int)((lane & ~3u) | ((w0 + 1) & 3u)), 64);
            if (k < mp) {
                S.key[4 * k + qi] = sh ? (a >> sh) | (b << (64 - sh)) : a;
                if (qi == 0) S.salt[k] = salt;
            }
        }
        __syncthreads();   // the stage has landed (vmcnt(0) of the DMA waves), keys and metadata are published

        // ---- the pass's output range [ps, pe) (tile-relative); a multi-pass tile
        // splits at datagram edges, whose partial chunks are stored masked
        const int32_t ps = g0 == d0 ? 0 : max(S.o[0], 0);
        int32_t pe = (int32_t)tile_len;
        if (g0 + mp < dend) pe = S.o[mp - 1] + (int32_t)S.w[mp - 1];
        const int32_t cA = (ps + 15) >> 4, cB = pe >> 4;   // full chunks [cA, cB)
        // ---- boundary chunks: wave t (0..2) assembles candidate t of datagram
        // `lane`, parked when that datagram is the first one touching it
        if (wid < 3 && lane < mp) {
            const uint32_t k = lane, Wb = S.w[k];
            const int32_t ob = S.o[k];
            uint8_t pk = 0;
            if (Wb) {
                const int32_t c = stream_cand(ob, Wb, SALT, (int)wid);
                bool dup = false;
                for (int u = 0; u < (int)wid; ++u) dup = dup || stream_cand(ob, Wb, SALT, u) == c;
                const int32_t x = 16 * c;
                const bool fast = ob + SALT <= x && x + 16 <= ob + (int32_t)Wb;
                // the output is contiguous: the previous valid datagram ends at ob, so it
                // reaches into the chunk unless the chunk starts at or after ob
                const bool mine = k == 0 || ob <= x;
                if (!dup && !fast && c >= cA && c < cB && mine) {
                    u128 rr = 0;
                    uint32_t cov = 0;
                    for (uint32_t q = k; q < mp && S.o[q] < x + 16; ++q) stream_contrib<OBF>(S, in, staged, q, x, rr, cov);
                    if (cov == 0xFFFFu) {
                        S.park[3 * k + wid] = rr;
                        pk = 1;
                    } else if (cov) {
                        store_masked(B.out + tT + x, rr, cov);
                    }
                }
            }
            S.parked[3 * k + wid] = pk;
        } else if (wid == 3 && lane < 2) {
            // partial chunks at the pass's ends (multi-pass tiles, the batch's end)
            const int32_t e0 = (ps & 15) ? (ps >> 4) : -1;
            int32_t e1 = (pe & 15) ? (pe >> 4) : -1;
            if (e1 == e0) e1 = -1;
            const int32_t c = lane == 0 ? e0 : e1;
            if (c >= 0) {
                const int32_t x = 16 * c;
                u128 rr = 0;
                uint32_t cov = 0;
                for (uint32_t q = 0; q < mp; ++q)
                    if (S.o[q] < x + 16) stream_contrib<OBF>(S, in, staged, q, x, rr, cov);
                const int32_t lo = max(x, ps), hi = min(x + 16, pe);
                cov &= lo < hi ? ((1u << (hi - lo)) - 1u) << (lo - x) : 0u;
                if (cov) store_masked(B.out + tT + x, rr, cov);
            }
        }
        hy_lds_barrier();

        // ---- sweep: every full chunk, from LDS (payload XOR key) or from the park
        uint8_t* __restrict__ ob = B.out + tT;
        for (int32_t c0 = cA; c0 < cB; c0 += 256 * kSU) {
            u128 v[kSU];
            bool ok[kSU];
#pragma unroll
            for (int u = 0; u < kSU; ++u) {
                const int32_t c = c0 + u * 256 + (int32_t)tid, x = 16 * c;
                ok[u] = false;
                v[u] = 0;
                if (c >= cB) continue;
                uint32_t q = 0;   // last datagram whose output starts at or before x
#pragma unroll
                for (uint32_t step = kSD / 2; step; step >>= 1) q = S.o[q + step] <= x ? q + step : q;
                const int32_t oq = S.o[q];
                const uint32_t Wq = S.w[q];
                if (Wq && oq + SALT <= x && x + 16 <= oq + (int32_t)Wq) {
                    v[u] = payload16<OBF>(S, in, staged, q, x - (oq + SALT)) ^ key16(S, q, x);
                    ok[u] = true;
                } else {
                    // the first datagram touching the chunk owns it
                    uint32_t own = q;
                    if (!(Wq && oq + (int32_t)Wq > x)) {
                        own = q + 1;
                        while (own < mp && S.w[own] == 0) ++own;
                    }
                    if (own < mp) {
                        const int32_t oo = S.o[own];
                        const uint32_t Wo = S.w[own];
#pragma unroll
                        for (int tt = 0; tt < 3; ++tt) {
                            if (!ok[u] && stream_cand(oo, Wo, SALT, tt) == c && S.parked[3 * own + tt]) {
                                v[u] = S.park[3 * own + tt];
                                ok[u] = true;
                            }
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < kSU; ++u) {
                const int32_t x = 16 * (c0 + u * 256 + (int32_t)tid);
                if (ok[u]) store16_stream(ob + x, v[u]);
            }
        }
        // a further pass overwrites metadata, keys and parked chunks: only the LDS
        // reads must be done (no wait for the stores)
        if (g0 + kSD < dend) hy_lds_barrier();
    }
}

inline uint64_t stream_ntiles_max(uint64_t out_cap) { return (out_cap + kST - 1) / kST; }
inline uint64_t stream_nblocks(uint64_t n) { return (n + kSBlk - 1) / kSBlk; }
// scratch bytes of the prepass: block sums (16 B per block + totals), descriptors
// (32 B per tile + the tail) when the stream kernel runs, input offsets when
// another kernel runs on them
inline uint64_t stream_workspace_bytes(uint64_t n, uint64_t out_cap, bool tiles, bool in_offsets) {
    return 16 * (stream_nblocks(n) + 1) + (tiles ? sizeof(StreamDesc) * (stream_ntiles_max(out_cap) + 1) : 0) +
           (in_offsets ? 8 * n : 0);
}

// The prepass (three launches); fills S from the scratch at ws: the block sums, then
// the descriptors (tiles: the stream kernel runs next), then the input offsets
// (in_offsets: another kernel runs next and reads them).
template <bool OBF>
void launch_stream_prepass(const BatchParams& b, StreamParams& S, void* ws, bool tiles, bool in_offsets,
                           hipStream_t s) {
    S.nblocks = stream_nblocks(b.n);
    S.ntiles_max = tiles ? stream_ntiles_max(b.out_cap) : 0;
    S.bsum = static_cast<uint64_t*>(ws);
    S.desc = tiles ? reinterpret_cast<StreamDesc*>(S.bsum + 2 * (S.nblocks + 1)) : nullptr;
    uint8_t* after = reinterpret_cast<uint8_t*>(S.bsum + 2 * (S.nblocks + 1)) +
                     (tiles ? sizeof(StreamDesc) * (S.ntiles_max + 1) : 0);
    S.in_off_out = in_offsets ? reinterpret_cast<uint64_t*>(after) : nullptr;
    S.write_out = tiles ? 1 : 0;
    hipLaunchKernelGGL(stream_sums_kernel<OBF>, dim3((uint32_t)S.nblocks), dim3(256), 0, s, b, S);
    hipLaunchKernelGGL(stream_scan_kernel<OBF>, dim3(1), dim3(1024), 0, s, b, S);
    hipLaunchKernelGGL(stream_locate_kernel<OBF>, dim3((uint32_t)S.nblocks), dim3(256), 0, s, b, S);
}

template <bool OBF, int SW>
void launch_stream_sw(const BatchParams& b, const KeyParams& k, const StreamParams& S, hipStream_t s) {
    // one workgroup per tile that out_cap allows (tiles past the valid output exit at
    // once); at least one, which writes out_total
    const uint64_t nt = S.ntiles_max < 1 ? 1 : S.ntiles_max;
    for (uint64_t t0 = 0; t0 < nt; t0 += HY_STREAM_LAUNCH_TILES) {
        const uint64_t g = nt - t0 < (uint64_t)HY_STREAM_LAUNCH_TILES ? nt - t0 : (uint64_t)HY_STREAM_LAUNCH_TILES;
        hipLaunchKernelGGL((salamander_stream_kernel<OBF, SW>), dim3((uint32_t)g), dim3(256), 0, s, b, k, S, t0);
    }
}

}  // namespace hyobfs
