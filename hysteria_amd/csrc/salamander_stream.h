// salamander_stream.h -- pipelined two-pass Salamander for uniform batches (gfx950).
//
// Same batch shape as salamander_uniform.h (equal lengths, a multiple of 8,
// dense 16-aligned slots).  The batch is cut into a few chunks of whole runs
// (a run = two neighbouring datagrams, whose input and output are whole 16-byte
// chunks).  Launch 0 derives the keys of chunk 0; launch i (i = 1..M) sweeps
// chunk i-1 and derives the keys of chunk i in the same grid:
//   * key blocks: one lane per datagram, key = BLAKE2b-256(PSK || salt)
//     (salamander.go:88-91), 4 words into the key buffer, plus the datagram's
//     out_off / out_len / out_total.  VALU-bound; they run beside the sweep's
//     memory-bound waves.
//   * sweep blocks: one-shot waves, each sweeping one contiguous region of
//     64 x kSU OUTPUT chunks (4 KiB): aligned 16-byte input chunks, the left
//     neighbour's chunk by a DPP wavefront shift (as in the uniform kernel),
//     key words from the buffer (written by the previous launch).
// The sweep's access shape is the one-shot 4 KiB region copy, the fastest copy
// shape measured on MI355X (tools/region_copy.hip, 6.0-6.1 TB/s); a kernel
// that hashes 64 keys per wave cannot have it (one wave's keys cover 77 KB of
// output).  Chunk sizes grow geometrically so that each launch's key work
// hides under its sweep; only chunk 0's keys (a small chunk) are exposed.
#pragma once
#include "salamander_uniform.h"

namespace hyobfs {

#ifndef HY_STREAM_U
#define HY_STREAM_U 4                // chunks per lane: a region of 64 x U chunks per wave
#endif
constexpr int kSU = HY_STREAM_U;

struct StreamParams {
    uint32_t D;          // payload words per datagram
    uint32_t CC;         // chunks swept per run: obfuscate D + 1 (output), deobfuscate D (output)
    double inv_cc;       // 1.0 / CC
    uint64_t run_in, run_out;
    uint64_t LI;         // input bytes per datagram
    uint32_t W;          // output bytes per datagram
    uint32_t nkb;        // key blocks of this launch: grid positions 0, kstride, 2 kstride, ...
    uint32_t kstride;    // (spread through the grid so the hashing overlaps the sweep)
    uint64_t run0;       // first run of the chunk swept by this launch
    uint64_t nch;        // output chunks swept by this launch
    uint64_t kp0, kp1;   // datagrams keyed by this launch
};

// Key block: datagrams [kp0, kp1), one per lane: key words to B.keys[4p .. 4p+3]
template <bool OBF, int SW>
__device__ __forceinline__ void stream_keys(const BatchParams& B, const KeyParams& K, const StreamParams& P,
                                            uint64_t blk) {
    const uint64_t p = P.kp0 + blk * 256 + threadIdx.x;
    const bool live = p < P.kp1;
    uint64_t salt = 0;
    if (live) {
        salt = OBF ? B.salts[p] : load8u(B.in + p * P.LI);   // the wire's salt
        if (B.out_off) B.out_off[p] = p * P.W;
        if (B.out_len) B.out_len[p] = P.W;
    }
    if (B.out_total) {
        const uint64_t wr = uni64(wave_sum(live ? P.W : 0u));
        if ((threadIdx.x & 63) == 0 && wr) atomicAdd(B.out_total, (unsigned long long)wr);
    }
    if (!live) return;
    uint64_t key[4];
#ifdef HY_X_NOHASH   // ablation builds only (timing experiments; wrong output)
    key[0] = salt; key[1] = salt * 3; key[2] = salt ^ 7; key[3] = salt + 1;
#else
    wave_key<SW>(K, salt, key);
#endif
    store16a_nt(reinterpret_cast<uint64_t>(B.keys + 4 * p), key[0], key[1]);
    store16a_nt(reinterpret_cast<uint64_t>(B.keys + 4 * p + 2), key[2], key[3]);
}

__device__ __forceinline__ uint64_t load8_global(uint64_t addr) {
#ifdef HYOBFS_EMULATE
    uint64_t v;
    std::memcpy(&v, reinterpret_cast<const void*>(addr), 8);
    return v;
#else
    return *(const __attribute__((address_space(1))) uint64_t*)addr;
#endif
}

// Sweep block: output chunks [64 kSU w, 64 kSU (w+1)) of the launch's chunk.
template <bool OBF>
__device__ __forceinline__ void stream_sweep(const BatchParams& B, const StreamParams& P, uint64_t blk) {
    constexpr int U = kSU;
    const int lane = threadIdx.x & 63;
    const uint64_t w = blk * kWavesPerBlock + uni32(threadIdx.x >> 6);
    const uint64_t c0 = w * (kGroup * U);   // first output chunk of this wave (in the launch's chunk)
    if (c0 >= P.nch) return;                // wave-uniform
    const uint32_t D = P.D, CC = P.CC;
    const uint64_t inb = reinterpret_cast<uint64_t>(B.in) + P.run0 * P.run_in;
    const uint64_t outb = reinterpret_cast<uint64_t>(B.out) + P.run0 * P.run_out;
    const uint64_t keyb = reinterpret_cast<uint64_t>(B.keys) + P.run0 * 64;
    const uint64_t saltb = reinterpret_cast<uint64_t>(B.salts) + P.run0 * 16;
    auto divcc = [&](uint64_t c, uint64_t& j, uint32_t& k) {   // c / CC, c % CC
        uint64_t q = (uint64_t)((double)c * P.inv_cc);
        if (q * CC > c) --q;
        else if ((q + 1) * CC <= c) ++q;
        j = q;
        k = (uint32_t)(c - q * CC);
    };
    struct Pos {
        uint64_t c, j;
        uint32_t k;
    };
    auto advance = [&](Pos& q) {   // CC > 64: at most one run boundary per step
        q.c += kGroup;
        q.k += kGroup;
        const bool wrap = q.k >= CC;
        q.k = wrap ? q.k - CC : q.k;
        q.j += wrap ? 1u : 0u;
    };
    // input chunk a lane at (run j, output chunk k) holds: obfuscate input chunk
    // k (none for k == D), deobfuscate input chunk k + 1 (the wire's salt0 sits in
    // chunk 0, so output chunk k starts in input chunk k)
    auto in_addr = [&](uint64_t j, uint32_t k) { return inb + j * P.run_in + 16ull * (OBF ? k : k + 1); };
    // the chunk the previous region ended with: lane 0's left neighbour (wave-uniform)
    uint32_t cy0 = 0, cy1 = 0, cy2 = 0, cy3 = 0;
    if (c0) {
        uint64_t jj;
        uint32_t kk;
        divcc(c0 - 1, jj, kk);
        if (!OBF || kk < D) {
            const u128 x = load16a_nt(in_addr(jj, kk));
            cy0 = (uint32_t)x;
            cy1 = (uint32_t)(x >> 32);
            cy2 = (uint32_t)(x >> 64);
            cy3 = (uint32_t)(x >> 96);
        }
    }
    Pos s0;
    s0.c = c0 + lane;
    divcc(s0.c, s0.j, s0.k);
    u128 v[U];
    uint64_t x0[OBF ? 1 : U];   // deobfuscate: input chunk 0's high word for a run's first output chunk
    Pos q = s0;
#pragma unroll
    for (int u = 0; u < U; ++u) {   // issue every load first
        v[u] = 0;
        if (q.c < P.nch && (!OBF || q.k < D)) v[u] = load16a_nt(in_addr(q.j, q.k));
        if (!OBF) {
            x0[u] = 0;
            if (q.c < P.nch && q.k == 0) x0[u] = load8_global(inb + q.j * P.run_in + 8);
        }
        advance(q);
    }
    q = s0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t o0 = (uint32_t)v[u], o1 = (uint32_t)(v[u] >> 32);
        const uint32_t o2 = (uint32_t)(v[u] >> 64), o3 = (uint32_t)(v[u] >> 96);
        // left neighbour (all lanes active: the shift reads every lane)
        const uint32_t p0 = OBF ? wave_prev32(o0, cy0) : 0u, p1 = OBF ? wave_prev32(o1, cy1) : 0u;
        const uint32_t p2 = wave_prev32(o2, cy2), p3 = wave_prev32(o3, cy3);
        if (OBF) {
            cy0 = lane63(o0);
            cy1 = lane63(o1);
        }
        cy2 = lane63(o2);
        cy3 = lane63(o3);
        const uint32_t k = q.k;
        if (q.c < P.nch) {
            const uint64_t own_lo = (uint64_t)o1 << 32 | o0, own_hi = (uint64_t)o3 << 32 | o2;
            const uint64_t prev_lo = (uint64_t)p1 << 32 | p0;
            uint64_t prev_hi = (uint64_t)p3 << 32 | p2;
            const uint64_t kb = keyb + 64 * q.j;   // the run's two keys, 4 words each
            const uint32_t e = 2 * k;              // output word of the chunk's low half
            uint64_t lo, hi;
            if (OBF) {
                // output words of the run: salt0 | payload0 (input words 0..D-1) |
                // salt1 | payload1 (input words D..2D-1)
                const bool d1l = e > D, d1h = e + 1 > D;
                const uint64_t kl = load8_global(kb + 32 * d1l + 8 * ((d1l ? e - D - 2 : e - 1) & 3));
                const uint64_t kh = load8_global(kb + 32 * d1h + 8 * ((d1h ? e - D - 1 : e) & 3));
                lo = pick(prev_hi, prev_lo, d1l) ^ kl;
                hi = pick(own_lo, prev_hi, d1h) ^ kh;
                if (e == 0 || e == D || e == D + 1) {   // the salt words (two chunks per run)
                    const uint64_t sb = saltb + 16 * q.j;
                    if (e == 0) lo = load8_global(sb);
                    if (e == D + 1) lo = load8_global(sb + 8);
                    if (e == D) hi = load8_global(sb + 8);
                }
            } else {
                // input words of the run: salt0 | payload0 | salt1 | payload1;
                // output words: payload0 (input words 1..D) | payload1 (D+2..2D+1)
                if (k == 0) prev_hi = x0[u];
                const bool d1l = e >= D, d1h = e + 1 >= D;
                const uint64_t kl = load8_global(kb + 32 * d1l + 8 * ((d1l ? e - D : e) & 3));
                const uint64_t kh = load8_global(kb + 32 * d1h + 8 * ((d1h ? e + 1 - D : e + 1) & 3));
                lo = pick(prev_hi, own_lo, d1l) ^ kl;
                hi = pick(own_lo, own_hi, d1h) ^ kh;
            }
            store16a_nt(outb + q.j * P.run_out + 16ull * k, lo, hi);
        }
        advance(q);
    }
}

template <bool OBF, int SW>
__global__ __launch_bounds__(256) void salamander_stream_kernel(BatchParams B, KeyParams K, StreamParams P) {
    const uint32_t b = blockIdx.x, kb = b / P.kstride;
    if (b % P.kstride == 0 && kb < P.nkb)
        stream_keys<OBF, SW>(B, K, P, kb);
    else   // key blocks at positions <= b: min(nkb, kb + 1)
        stream_sweep<OBF>(B, P, b - min(P.nkb, kb + 1));
}

// Key pass alone (HYOBFS_KERNEL_PIPE): a small grid, grid-stride over the
// launch's key blocks, on the side lane's stream.  Its few waves hash beside
// the memory-bound sweep of the previous chunk instead of sharing that grid:
// in one grid the late key blocks held the launch open after its sweep waves
// had drained.
template <bool OBF, int SW>
__global__ __launch_bounds__(256) void salamander_stream_keys_kernel(BatchParams B, KeyParams K, StreamParams P) {
    for (uint64_t kb = blockIdx.x; kb < P.nkb; kb += gridDim.x) stream_keys<OBF, SW>(B, K, P, kb);
}

template <bool OBF>
inline bool stream_params(const BatchParams& b, StreamParams& P) {
    UniformParams U;
    if (!b.keys || !uniform_params<OBF>(b, U)) return false;
    P = StreamParams{};
    P.D = U.D;
    P.CC = OBF ? U.D + 1 : U.D;   // output chunks per run
    if (P.CC <= (uint32_t)kGroup) return false;
    P.inv_cc = 1.0 / (double)P.CC;
    P.run_in = U.run_in;
    P.run_out = U.run_out;
    P.LI = U.LI;
    P.W = U.W;
    return true;
}

// Chunk boundaries (in runs): the first chunk small, each next one up to
// kGrow times the previous, so a launch's keys (for the next chunk) take less
// time than its sweep.
#ifndef HY_STREAM_FIRST_RUNS
#define HY_STREAM_FIRST_RUNS 8192    // 16K datagrams: ~1 us of exposed keys
#endif
#ifndef HY_STREAM_GROW
#define HY_STREAM_GROW 4
#endif

inline uint64_t stream_env(const char* name, uint64_t dflt) {   // A/B knobs, read once per name
    const char* e = std::getenv(name);
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? (uint64_t)v : dflt;
}

// Side-lane schedule (HYOBFS_KERNEL_PIPE) defaults: chunk 0 of 2048 runs
// (4K datagrams) keyed by a full grid, then chunks up to 4x the previous one,
// each keyed by at most 256 workgroups (one wave per SIMD) while the caller's
// stream sweeps the chunk before it.
#ifndef HY_PIPE_FIRST_RUNS
#define HY_PIPE_FIRST_RUNS 2048
#endif
#ifndef HY_PIPE_GROW
#define HY_PIPE_GROW 4
#endif
#ifndef HY_PIPE_KEY_BLOCKS
#define HY_PIPE_KEY_BLOCKS 256
#endif

template <bool OBF, int SW>
void launch_stream_sw(const BatchParams& bp, const KeyParams& k, const StreamParams& base, uint64_t nruns,
                      uint64_t nkeys, hipStream_t s, const SideLane* side) {
    static const uint64_t s_first = stream_env("HYOBFS_STREAM_FIRST_RUNS", HY_STREAM_FIRST_RUNS);
    static const uint64_t s_grow = std::max<uint64_t>(2, stream_env("HYOBFS_STREAM_GROW", HY_STREAM_GROW));
    // the side-lane knobs are read per call (in-process A/B of schedules)
    const uint64_t first = side ? stream_env("HYOBFS_PIPE_FIRST_RUNS", HY_PIPE_FIRST_RUNS) : s_first;
    const uint64_t grow = side ? std::max<uint64_t>(2, stream_env("HYOBFS_PIPE_GROW", HY_PIPE_GROW)) : s_grow;
    // chunk i = runs [r[i], r[i+1])
    uint64_t r[64];
    int m = 0;
    r[0] = 0;
    uint64_t len = first;
    while (r[m] < nruns && m < 62) {
        r[m + 1] = std::min<uint64_t>(nruns, r[m] + len);
        ++m;
        len *= grow;
    }
    if (r[m] < nruns) r[m] = nruns;   // (not reached: 62 growing chunks)
    auto key_range = [&](int i, StreamParams& P) {   // keys of chunk i (the odd tail with the last)
        P.kp0 = 2 * r[i];
        P.kp1 = (i + 1 == m) ? nkeys : 2 * r[i + 1];
        P.nkb = (uint32_t)div_up(P.kp1 - P.kp0, 256);
    };
    if (side) {
        // side stream: after the caller's earlier work (the inputs), the keys of
        // chunk 0, 1, ... back to back, event i+1 after chunk i's; caller's
        // stream: sweep chunk i once event i+1 has fired.  Keys run ahead of the
        // sweeps (a throttled grid still hashes ~8x faster than the sweep moves
        // bytes), so only chunk 0's keys are exposed.
        const uint64_t kblocks = stream_env("HYOBFS_PIPE_KEY_BLOCKS", HY_PIPE_KEY_BLOCKS);
        if (hipEventRecord(side->ev[0], s) != hipSuccess) return;
        if (hipStreamWaitEvent(side->s, side->ev[0], 0) != hipSuccess) return;
        for (int i = 0; i < m; ++i) {
            StreamParams P = base;
            key_range(i, P);
            const uint64_t grid = i == 0 ? P.nkb : std::min<uint64_t>(P.nkb, kblocks);
            hipLaunchKernelGGL((salamander_stream_keys_kernel<OBF, SW>), dim3((uint32_t)grid),
                               dim3(kGroup * kWavesPerBlock), 0, side->s, bp, k, P);
            if (hipEventRecord(side->ev[i + 1], side->s) != hipSuccess) return;
        }
        for (int i = 0; i < m; ++i) {
            StreamParams P = base;   // nkb = 0: every block sweeps
            P.kstride = 1;
            P.run0 = r[i];
            P.nch = (r[i + 1] - r[i]) * P.CC;
            const uint64_t blocks = div_up(div_up(P.nch, (uint64_t)kGroup * kSU), kWavesPerBlock);
            if (hipStreamWaitEvent(s, side->ev[i + 1], 0) != hipSuccess) return;
            hipLaunchKernelGGL((salamander_stream_kernel<OBF, SW>), dim3((uint32_t)blocks),
                               dim3(kGroup * kWavesPerBlock), 0, s, bp, k, P);
        }
        return;
    }
    for (int i = 0; i <= m; ++i) {   // launch i: keys of chunk i, sweep of chunk i - 1
        StreamParams P = base;
        if (i < m) key_range(i, P);
        uint64_t sweep_blocks = 0;
        if (i > 0) {
            P.run0 = r[i - 1];
            P.nch = (r[i] - r[i - 1]) * P.CC;
            sweep_blocks = div_up(div_up(P.nch, (uint64_t)kGroup * kSU), kWavesPerBlock);
        }
        const uint64_t blocks = P.nkb + sweep_blocks;
        P.kstride = P.nkb ? (uint32_t)std::max<uint64_t>(1, blocks / P.nkb) : 1;
        hipLaunchKernelGGL((salamander_stream_kernel<OBF, SW>), dim3((uint32_t)blocks), dim3(kGroup * kWavesPerBlock),
                           0, s, bp, k, P);
    }
}

}  // namespace hyobfs
