// salamander.hip -- gfx950 batch kernels for Hysteria's Salamander obfuscation:
// launch dispatch, the packed layout's tile scan, the keys-only kernel and the
// synthetic-input kernels.
//
// Reference semantics (apernet/hysteria): extras/obfs/salamander.go:59-91.
//   Obfuscate:   out = salt(8) || in[i] ^ key[i % 32]        (:59-72)
//   Deobfuscate: out[i] = in[8 + i] ^ key[i % 32], reject len <= 8  (:74-86)
//   key = BLAKE2b-256(PSK || salt)                              (:88-91)
//
// Three batch kernels ("Kernels"), all HBM-bound byte work, no MFMA:
//   * salamander_tile_kernel (salamander_tile.h): slotted batches whose region
//     edges are all multiples of 8 -- the uniform 1200-byte headline batch.
//     One-shot workgroups of 16 datagrams: a key wave beside three data waves.
//   * salamander_flat_kernel (salamander_flat.h): contiguous input into packed
//     output (configs[2]).  One-shot workgroups per 16 KiB of output.
//   * salamander_wave_kernel (salamander_wave.h): every other layout (packed
//     output, ragged lengths, any alignment).  One wave per 64-datagram group.
#include <unistd.h>

#include <atomic>
#include <chrono>

#include "salamander_flat.h"

namespace hyobfs {

// The kernels' instantiations live in salamander_inst.hip (one TU per salt word).
#define HY_EXTERN_SW(n)                                                                                   \
    extern template void launch_wave_sw<true, true, n>(const BatchParams&, const KeyParams&, hipStream_t);  \
    extern template void launch_wave_sw<true, false, n>(const BatchParams&, const KeyParams&, hipStream_t); \
    extern template void launch_wave_sw<false, true, n>(const BatchParams&, const KeyParams&, hipStream_t); \
    extern template void launch_wave_sw<false, false, n>(const BatchParams&, const KeyParams&, hipStream_t); \
    extern template void launch_tile_sw<true, n>(const BatchParams&, const KeyParams&, const TileParams&,   \
                                                 hipStream_t);                                              \
    extern template void launch_tile_sw<false, n>(const BatchParams&, const KeyParams&, const TileParams&,  \
                                                  hipStream_t);                                             \
    extern template void launch_flat_sw<true, n>(const BatchParams&, const KeyParams&, const FlatParams&,   \
                                                 hipStream_t);                                              \
    extern template void launch_flat_sw<false, n>(const BatchParams&, const KeyParams&, const FlatParams&,  \
                                                  hipStream_t);
HY_EXTERN_SW(0) HY_EXTERN_SW(1) HY_EXTERN_SW(2) HY_EXTERN_SW(3) HY_EXTERN_SW(4) HY_EXTERN_SW(5)
HY_EXTERN_SW(6) HY_EXTERN_SW(7) HY_EXTERN_SW(8) HY_EXTERN_SW(9) HY_EXTERN_SW(10) HY_EXTERN_SW(11)
HY_EXTERN_SW(12) HY_EXTERN_SW(13) HY_EXTERN_SW(14) HY_EXTERN_SW(15)
#undef HY_EXTERN_SW

// ------------------------------------------------------ packed-layout scan
// Tile sums of the output widths; the main kernel adds a wavefront scan.
// Per tile of kTile datagrams: the sum of the output widths (packed layout) and, for
// contiguous input, of the input lengths.  Wave w of workgroup b owns tile 4b + w,
// four datagrams per lane; no LDS, no barrier.
template <bool OBF>
__global__ __launch_bounds__(256) void tile_sums_kernel(BatchParams B, uint64_t ntiles) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t tile = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t p0 = tile * kTile + 4ull * lane;
    uint64_t sw = 0, sl = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (p0 + k < B.n) {
            const uint32_t L = pkt_len(B, p0 + k);
            sw += out_width<OBF>(L, B.pkt_cap);
            sl += L;
        }
    }
    sw = wave_sum(sw);
    if (B.in_tile_sums) sl = wave_sum(sl);
    if (lane == 0 && tile < ntiles) {
        B.tile_sums[tile] = sw;
        if (B.in_tile_sums) B.in_tile_sums[tile] = sl;
    }
}

// Exclusive scan of ntiles values in place, one workgroup of 1024 threads per
// array: workgroup 0 scans v, workgroup 1 (contiguous input) the length sums v2;
// each writes its total at [ntiles].  A pass covers 8192 values: wave w owns 512
// consecutive ones, loaded and stored coalesced (64 lanes x 8 B per instruction)
// and transposed through LDS so that lane l sums values 8l .. 8l + 7 of the wave's
// block sequentially.  (Loading each thread's 16 consecutive values directly --
// one cache line per lane -- took 20 us per array for 16384 tiles on the one CU
// that runs this; this takes 12.)
__global__ __launch_bounds__(1024) void scan_tiles_kernel(uint64_t* v, uint64_t* v2, uint64_t ntiles,
                                                         uint64_t* init2 = nullptr) {
    constexpr int PER = 8, BLK = 64 * PER;
    constexpr int PAD = PER + 1;             // LDS row of a lane: PER values + 1 (fewer bank conflicts)
    __shared__ uint64_t s_x[16][64 * PAD];   // per wave: its block, lane-major
    __shared__ uint64_t s_w[16];
    __shared__ uint64_t s_carry;
    uint64_t* const arr = blockIdx.x ? v2 : v;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    if (t == 0) s_carry = 0;
    if (init2 && blockIdx.x == 0 && t < 2) init2[t] = ~0ull;   // the flat prepass's cut record (salamander_flat.h)
    __syncthreads();
    for (uint64_t base = 0; base < ntiles; base += 16 * BLK) {
        const uint64_t wb = base + (uint64_t)wid * BLK;
#pragma unroll
        for (int k = 0; k < PER; ++k) {   // value j = 64 k + lane of the block -> row j / PER, column j % PER
            const int j = 64 * k + lane;
            const uint64_t i = wb + (uint64_t)j;
            s_x[wid][(j / PER) * PAD + j % PER] = i < ntiles ? arr[i] : 0;
        }
        hy_wave_sync();
        uint64_t* row = &s_x[wid][lane * PAD];
        uint64_t run = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) {   // exclusive within the lane's row
            const uint64_t x = row[k];
            row[k] = run;
            run += x;
        }
        const uint64_t inc = wave_incl_scan(run, lane);
        if (lane == 63) s_w[wid] = inc;
        __syncthreads();
        uint64_t wpre = 0;
        for (int w = 0; w < wid; ++w) wpre += s_w[w];
        const uint64_t off = s_carry + wpre + inc - run;   // before this lane's row
#pragma unroll
        for (int k = 0; k < PER; ++k) row[k] += off;
        hy_wave_sync();
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = 64 * k + lane;
            const uint64_t i = wb + (uint64_t)j;
            if (i < ntiles) arr[i] = s_x[wid][(j / PER) * PAD + j % PER];
        }
        __syncthreads();
        if (t == 0) {
            uint64_t tot = 0;
            for (int w = 0; w < 16; ++w) tot += s_w[w];
            s_carry += tot;
        }
        __syncthreads();
    }
    if (t == 0) arr[ntiles] = s_carry;
}

// Contiguous input run on a kernel that takes explicit offsets (slotted output, or
// packed runs shorter than 64): in_off[i] from the scanned per-tile length sums and
// a wave scan.  Wave w of workgroup b owns tile 4b + w, four datagrams per lane.
__global__ __launch_bounds__(256) void in_offsets_kernel(BatchParams B, uint64_t* in_off) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t tile = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile * kTile >= B.n) return;   // whole waves
    const uint64_t p0 = tile * kTile + 4ull * lane;
    uint32_t L[4];
    uint64_t sl = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        L[k] = p0 + k < B.n ? B.in_len[p0 + k] : 0u;
        sl += L[k];
    }
    uint64_t x = B.in_tile_prefix[tile] + wave_incl_scan(sl, (int)lane) - sl;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (p0 + k < B.n) in_off[p0 + k] = x;
        x += L[k];
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

// Kernel choice ("Kernels"): AUTO runs the tile kernel where it
// applies (tile_params) and the wave kernel elsewhere; WAVE forces the wave kernel;
// FLAT runs the flat kernel on contiguous input into packed output (flat_eligible)
// and is AUTO elsewhere; TILE is AUTO.  HYOBFS_KERNEL=wave|tile|flat sets what AUTO
// means in a process.
static int kernel_override() {   // HYOBFS_KERNEL, as HYOBFS_KERNEL_* (0 = auto); read once, thread-safe
    static const int v = [] {
        const char* e = std::getenv("HYOBFS_KERNEL");
        return !e                        ? kKernelAuto
               : std::strcmp(e, "wave") == 0 ? kKernelWave
               : std::strcmp(e, "tile") == 0 ? kKernelTile
               : std::strcmp(e, "flat") == 0 ? kKernelFlat
                                             : kKernelAuto;
    }();
    return v;
}

int resolve_kernel(int ctx_kernel) { return ctx_kernel ? ctx_kernel : kernel_override(); }

template <bool OBF, bool PACKED>
static void launch_main(const BatchParams& bp, const KeyParams& k, hipStream_t s) {
    const int kc = resolve_kernel(bp.kernel);
    TileParams T;
    if (!PACKED && kc != kKernelWave && tile_params<OBF>(bp, T)) {
        switch (k.salt_pos >> 3) {
#define HY_CASE(n) \
    case n: launch_tile_sw<OBF, n>(bp, k, T, s); break;
            HY_CASE(0) HY_CASE(1) HY_CASE(2) HY_CASE(3) HY_CASE(4) HY_CASE(5) HY_CASE(6) HY_CASE(7)
            HY_CASE(8) HY_CASE(9) HY_CASE(10) HY_CASE(11) HY_CASE(12) HY_CASE(13) HY_CASE(14)
            HY_CASE(15)
#undef HY_CASE
        }
        return;
    }
    switch (k.salt_pos >> 3) {
#define HY_CASE(n) \
    case n: launch_wave_sw<OBF, PACKED, n>(bp, k, s); break;
        HY_CASE(0) HY_CASE(1) HY_CASE(2) HY_CASE(3) HY_CASE(4) HY_CASE(5) HY_CASE(6) HY_CASE(7)
        HY_CASE(8) HY_CASE(9) HY_CASE(10) HY_CASE(11) HY_CASE(12) HY_CASE(13) HY_CASE(14)
        HY_CASE(15)
#undef HY_CASE
    }
}

// Contiguous input.  Packed output in runs of 64 (the default): the wave kernel takes
// its input offsets from a scan of the lengths done with the widths'
// (tile_sums_kernel, scan_tiles_kernel).  Otherwise (slotted output, shorter packed
// runs) a prepass writes the input offsets into the scratch -- length sums, their
// scan, in_offsets_kernel -- and the kernels for explicit offsets run on them.
// A tag no earlier call used (the flat kernel's key records, salamander_flat.h): a
// process-wide counter from a clock- and pid-derived start, never 0.
static uint64_t next_epoch() {
    static std::atomic<uint64_t> ctr{[] {
        const uint64_t t = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
        return (t * 0x9e3779b97f4a7c15ull) ^ ((uint64_t)getpid() << 40);
    }()};
    uint64_t e;
    do e = ctr.fetch_add(1, std::memory_order_relaxed) + 1; while (e == 0);
    return e;
}

// The flat kernel (salamander_flat.h) runs when asked for (HYOBFS_KERNEL_FLAT, or
// HYOBFS_KERNEL=flat) on contiguous input into packed output from 16-byte aligned
// input.  AUTO keeps the wave kernel there: on configs[2] it is faster (1.36-1.42 ms
// against 1.53-1.68 ms for the flat kernel's variants, profiles/r06_bimodal/).
static bool flat_eligible(const BatchParams& b) {
    return contiguous_input(b) && b.out_stride == 0 && resolve_kernel(b.kernel) == kKernelFlat &&
           (reinterpret_cast<uintptr_t>(b.in) & 15u) == 0;
}
static bool wave_scans_input(const BatchParams& b) {   // the wave kernel scans the lengths itself
    return contiguous_input(b) && b.out_stride == 0 && !flat_eligible(b) && wave_packed_run_log2() == 6;
}

// scratch: [width sums | length sums] (ntiles + 1 each), then the flat prepass's
// header and tile descriptors, or (when the prepass writes them) the input offsets
// (8 B per datagram)
uint64_t batch_workspace_bytes(bool obf, const BatchParams& b) {
    (void)obf;
    if (b.n == 0) return 0;
    const uint64_t tsums = (div_up(b.n, kTile) + 1) * 8;
    if (!contiguous_input(b)) return b.out_stride == 0 ? tsums : 0;
    if (flat_eligible(b)) return 2 * tsums + flat_workspace_bytes(b.out_cap, b.n);
    return 2 * tsums + (wave_scans_input(b) ? 0 : 8 * b.n);
}

// Which kernel launch_salamander runs for this batch (HYOBFS_KERNEL_*; no launch).
int batch_kernel(bool obf, const BatchParams& b) {
    if (b.n == 0) return kKernelAuto;   // nothing runs
    if (flat_eligible(b)) return kKernelFlat;
    TileParams T;
    BatchParams bp = b;
    if (contiguous_input(b) && !wave_scans_input(b))
        bp.in_off = reinterpret_cast<const uint64_t*>(16);   // offsets from the prepass
    const bool tile = bp.out_stride != 0 && resolve_kernel(bp.kernel) != kKernelWave &&
                      (obf ? tile_params<true>(bp, T) : tile_params<false>(bp, T));
    return tile ? kKernelTile : kKernelWave;
}

template <bool OBF>
static hipError_t launch_contiguous(BatchParams& bp, const KeyParams& k, hipStream_t s, bool& done) {
    done = false;
    if (!bp.scratch) return hipErrorInvalidValue;
    const uint64_t ntiles = div_up(bp.n, kTile);
    bp.tile_sums = static_cast<uint64_t*>(bp.scratch);
    bp.in_tile_sums = bp.tile_sums + ntiles + 1;
    if (flat_eligible(bp)) {   // sums, their scan, the locate prepass, the flat kernel
        FlatParams F;
        F.cut = bp.in_tile_sums + ntiles + 1;
        F.desc = reinterpret_cast<FlatDesc*>(F.cut + 2);
        F.out_total = bp.tile_sums + ntiles;     // the width scan's total
        F.in_total = bp.in_tile_sums + ntiles;   // the length scan's total
        F.ntiles_max = flat_ntiles_max(bp.out_cap);
        F.krec = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(F.cut) + flat_desc_bytes(bp.out_cap) + 255) &
                                            ~(uintptr_t)255);
        F.epoch = next_epoch();
        F.nhash = flat_hashers();
        const dim3 grid((uint32_t)div_up(ntiles, 4)), block(256);
        hipLaunchKernelGGL(tile_sums_kernel<OBF>, grid, block, 0, s, bp, ntiles);
        hipLaunchKernelGGL(scan_tiles_kernel, dim3(2), dim3(1024), 0, s, bp.tile_sums, bp.in_tile_sums, ntiles, F.cut);
        bp.tile_prefix = bp.tile_sums;
        bp.in_tile_prefix = bp.in_tile_sums;
        hipLaunchKernelGGL(flat_locate_kernel<OBF>, grid, block, 0, s, bp, F, ntiles);
        switch (k.salt_pos >> 3) {
#define HY_CASE(n) \
    case n: launch_flat_sw<OBF, n>(bp, k, F, s); break;
            HY_CASE(0) HY_CASE(1) HY_CASE(2) HY_CASE(3) HY_CASE(4) HY_CASE(5) HY_CASE(6) HY_CASE(7)
            HY_CASE(8) HY_CASE(9) HY_CASE(10) HY_CASE(11) HY_CASE(12) HY_CASE(13) HY_CASE(14)
            HY_CASE(15)
#undef HY_CASE
        }
        done = true;
        return hipGetLastError();
    }
    if (wave_scans_input(bp)) return hipSuccess;   // the packed launch below scans both sums
    uint64_t* in_off = bp.in_tile_sums + ntiles + 1;
    const dim3 grid((uint32_t)div_up(ntiles, 4)), block(256);
    hipLaunchKernelGGL(tile_sums_kernel<OBF>, grid, block, 0, s, bp, ntiles);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(1024), 0, s, bp.in_tile_sums, nullptr, ntiles);
    bp.in_tile_prefix = bp.in_tile_sums;
    hipLaunchKernelGGL(in_offsets_kernel, grid, block, 0, s, bp, in_off);
    bp.in_off = in_off;   // from here on an ordinary batch with explicit offsets
    bp.in_tile_sums = nullptr;
    bp.in_tile_prefix = nullptr;
    return hipGetLastError();
}

hipError_t launch_salamander(bool obf, const BatchParams& b, const KeyParams& k, hipStream_t s) {
    if (b.n == 0) return hipSuccess;
    const uint64_t ntiles = div_up(b.n, kTile);
    if (ntiles > 0x7fffffffull) return hipErrorInvalidValue;
    if (k.nblk == 2 && (k.salt_pos >> 3) != 15) return hipErrorInvalidValue;   // by construction
    BatchParams bp = b;
    if (contiguous_input(b)) {
        bool done = false;
        const hipError_t e = obf ? launch_contiguous<true>(bp, k, s, done) : launch_contiguous<false>(bp, k, s, done);
        if (e != hipSuccess || done) return e;
    }
    if (bp.out_stride == 0) {
        if (!bp.tile_sums) return hipErrorInvalidValue;
        const dim3 grid((uint32_t)div_up(ntiles, 4)), block(256);
        if (obf)
            hipLaunchKernelGGL(tile_sums_kernel<true>, grid, block, 0, s, bp, ntiles);
        else
            hipLaunchKernelGGL(tile_sums_kernel<false>, grid, block, 0, s, bp, ntiles);
        hipLaunchKernelGGL(scan_tiles_kernel, dim3(bp.in_tile_sums ? 2 : 1), dim3(1024), 0, s, bp.tile_sums,
                           bp.in_tile_sums, ntiles);
        bp.tile_prefix = bp.tile_sums;
        bp.in_tile_prefix = bp.in_tile_sums;
        if (obf)
            launch_main<true, true>(bp, k, s);
        else
            launch_main<false, true>(bp, k, s);
    } else {
        if (obf)
            launch_main<true, false>(bp, k, s);
        else
            launch_main<false, false>(bp, k, s);
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
