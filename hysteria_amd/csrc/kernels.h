// Private interface between the C ABI layer (hyobfs_api.cpp) and the gfx950
// kernels (salamander.hip).  Not installed; include/hyobfs.h is the ABI.
#pragma once
#ifdef HYOBFS_EMULATE
#include "hip_emu.h"   // tests/emu: CPU emulation for the CPU test tier, never shipped
#else
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>
#include <cstdlib>
#include <cstring>

#include "../../include/hyobfs_gecko.h"

namespace hyobfs {

// Orders one wave's LDS writes before its later LDS reads by other lanes of the
// same wave.  A wave's LDS instructions execute in order, so this only has to
// stop the compiler from moving memory operations across it (wavefront-scope
// fences emit no instruction).
#ifdef HYOBFS_EMULATE
inline void hy_wave_sync() { hyemu_wave_sync(); }
#else
__device__ __forceinline__ void hy_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
#endif

constexpr int kTile = 256;          // datagrams per tile-sum entry of the packed layout's scan
constexpr uint32_t kMaxDatagram = (1u << 24) - 64;  // longest datagram a batch accepts
constexpr uint64_t kMaxStride = 1ull << 24;         // longest slot of a slotted output
// batch kernels (include/hyobfs.h HYOBFS_KERNEL_*)
constexpr int kKernelAuto = 0, kKernelWave = 1, kKernelTile = 2, kKernelFlat = 3;

// BLAKE2b state for the per-packet key, precomputed on the host from the PSK
// alone (salamander.go:88-91 hashes PSK || salt; every block before the one
// holding salt[0] depends on the PSK only).  The device compresses the last
// one or two blocks, which carry the salt.
struct KeyParams {
    uint64_t h[8];       // chaining value entering the first device block
    uint64_t m[32];      // message words of the device blocks, salt bytes = 0
    uint64_t t[2];       // byte counter after each device block
    uint32_t nblk;       // 1 or 2 device blocks
    uint32_t salt_pos;   // byte offset of salt[0] in the device blocks (0..127)
};

// One batch launch (include/hyobfs.h, struct hyobfs_batch, plus derived values).
struct BatchParams {
    uint64_t n;
    const uint8_t* in;
    const uint64_t* in_off;
    uint64_t in_stride;
    const uint32_t* in_len;
    uint32_t len_uniform;
    uint32_t pkt_cap;       // effective per-packet cap (slot and pkt_cap folded), 0 = none
    const uint64_t* salts;
    uint8_t* out;
    uint64_t out_cap;
    uint64_t out_stride;    // 0 = packed
    uint64_t* out_off;
    uint32_t* out_len;
    unsigned long long* out_total;
    const uint64_t* tile_prefix;  // packed: exclusive prefix of tile sums (ntiles+1)
    uint64_t* tile_sums;          // packed: scratch, ntiles+1 entries
    // contiguous input, packed output on the wave kernel: per-tile sums of the input
    // lengths (scratch, ntiles+1) and their exclusive prefix (the input offsets)
    uint64_t* in_tile_sums = nullptr;
    const uint64_t* in_tile_prefix = nullptr;
    void* scratch;                // contiguous input: the stream prepass's scratch (batch_workspace_bytes)
    uint32_t run_log2;            // wave kernel: datagrams per run = 2^run_log2
    uint64_t blk0 = 0;            // wave kernel, packed runs of 64: first workgroup of this launch
    int kernel;                   // HYOBFS_KERNEL_* of the context (0 = auto)
};

// HYOBFS_KERNEL_* that a context's setting resolves to (AUTO: the
// HYOBFS_KERNEL environment variable, else 0)
int resolve_kernel(int ctx_kernel);
hipError_t launch_salamander(bool obfuscate, const BatchParams& b, const KeyParams& k, hipStream_t s);
// the kernel launch_salamander would run (kKernelTile / kKernelWave / kKernelFlat;
// kKernelAuto for an empty batch)
int batch_kernel(bool obfuscate, const BatchParams& b);
// device scratch a launch of this batch needs (0: none); launch_salamander takes it
// from b.tile_sums / b.scratch as laid out by batch_workspace_layout
uint64_t batch_workspace_bytes(bool obfuscate, const BatchParams& b);
// contiguous input: datagram i at in + in_len[0] + ... + in_len[i-1]
inline bool contiguous_input(const BatchParams& b) { return !b.in_off && b.in_stride == 0 && b.in_len && b.n > 1; }
hipError_t launch_keys(const KeyParams& k, const uint64_t* salts, uint8_t* keys, uint64_t n,
                       hipStream_t s);
hipError_t launch_gecko_encode(const KeyParams& k, const hyobfs_gecko_batch& b, hipStream_t s);
hipError_t launch_gecko_parse(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint64_t n,
                              hyobfs_gecko_parsed* out, hipStream_t s);
hipError_t launch_synth_stream(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t start,
                               hipStream_t s);
hipError_t launch_synth_u64(uint64_t* dst, uint64_t n, uint64_t seed, uint64_t first,
                            hipStream_t s);
hipError_t launch_synth_bimodal(uint32_t* dst, uint64_t n, uint64_t seed, uint64_t first,
                                hipStream_t s);

}  // namespace hyobfs
