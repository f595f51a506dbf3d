// gecko.hip -- Gecko framing kernels (include/hyobfs_gecko.h).
//
// Encode: one wavefront per frame.  The wire datagram of frame f is
//     salt(8) || (hdr(5) || pad || chunk) ^ key_f[i % 32]
// (gecko_frame.go:39-61 encodeFrame, then salamander.go:59-72 Obfuscate).  Lane
// l handles wire bytes l, l+64, l+128, ...: loads of the chunk and stores of
// the wire are byte-coalesced across the wave, and the key byte a lane needs
// is the same on every pass ((l - 8) mod 32, as 64 is a multiple of 32), so it
// is read once.  Keys come from keys_kernel (salamander.hip) into the
// workspace.  Gecko carries handshake packets only (low volume), so the
// kernel is written for simplicity over byte-level work.
//
// Parse: one thread per deobfuscated datagram, the checks of ReadFrom
// (gecko.go:170-193) and decodeFrame (gecko_frame.go:65-86) in their order.
#include "kernels.h"
#include "../../include/hyobfs_gecko.h"

namespace hyobfs {

__device__ __forceinline__ uint64_t gk_sm64(uint64_t seed, uint64_t k) {   // SplitMix64 output k
    uint64_t z = seed + (k + 1) * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void gecko_encode_kernel(hyobfs_gecko_batch B) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t f = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (f >= B.n) return;
    const hyobfs_gecko_frame fr = B.frames[f];
    const uint32_t total = fr.idx_total & 0x0f, idx = fr.idx_total >> 4;
    const uint32_t plain = HYOBFS_GECKO_HEADER_LEN + fr.pad_len + fr.chunk_len;
    const uint32_t W = HYOBFS_SALT_LEN + plain;
    if (total < HYOBFS_GECKO_MIN_CHUNKS || total > HYOBFS_GECKO_MAX_CHUNKS || idx >= total ||
        W > HYOBFS_GECKO_BUFFER_SIZE)
        return;   // not a frame writeFragmented can produce: skipped
    const uint8_t* key = static_cast<const uint8_t*>(B.workspace) + 32 * f;
    const uint8_t kb = key[(lane + 32 - HYOBFS_SALT_LEN) & 31];
    const uint64_t salt = B.salts[f];
    const uint8_t* chunk = B.msg + fr.chunk_off;
    uint8_t* out = B.out + B.out_off[f];
    const uint64_t pad0 = f * HYOBFS_GECKO_BUFFER_SIZE;   // this frame's window of the pad stream
    for (uint32_t j = lane; j < W; j += 64) {
        if (j < HYOBFS_SALT_LEN) {
            out[j] = (uint8_t)(salt >> (8 * j));
            continue;
        }
        const uint32_t p = j - HYOBFS_SALT_LEN;
        uint8_t v;
        if (p < HYOBFS_GECKO_HEADER_LEN) {   // 0x80 | msgID | idx<<4|total | padLen big-endian
            v = p == 0 ? (uint8_t)HYOBFS_GECKO_FLAG_FRAGMENT : p == 1 ? fr.msg_id : p == 2 ? fr.idx_total
              : p == 3 ? (uint8_t)(fr.pad_len >> 8) : (uint8_t)fr.pad_len;
        } else if (p < HYOBFS_GECKO_HEADER_LEN + fr.pad_len) {
            const uint64_t g = pad0 + (p - HYOBFS_GECKO_HEADER_LEN);
            v = (uint8_t)(gk_sm64(B.pad_seed, g >> 3) >> (8 * (g & 7)));
        } else {
            v = chunk[p - HYOBFS_GECKO_HEADER_LEN - fr.pad_len];
        }
        out[j] = v ^ kb;
    }
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
    hipError_t e = launch_keys(k, b.salts, static_cast<uint8_t*>(b.workspace), b.n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gecko_encode_kernel, dim3((uint32_t)((b.n + 3) / 4)), dim3(256), 0, s, b);
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
