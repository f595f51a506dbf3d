// gecko.hip -- Gecko framing kernels (include/hyobfs_gecko.h).
//
// Encode: 16 lanes per frame, four frames per wavefront.  The wire datagram of frame f is
//     salt(8) || (hdr(5) || pad || chunk) ^ key_f[i % 32]
// (gecko_frame.go:39-61 encodeFrame, then salamander.go:59-72 Obfuscate).  Lane
// l of a frame handles plaintext windows of 16 bytes at 16l, 16(l+16), ..., four
// in flight (loads first, then stores): a window inside
// the chunk is one unaligned 16-byte load, one inside the padding is two
// SplitMix64 words, a window across header / padding / chunk merges the
// three under byte masks, and each leaves as one 16-byte store (the frame's last
// partial window as bytes).  The
// key half a lane needs is the same on every pass (window index parity = lane
// parity), so it is loaded once.  Keys come from keys_kernel (salamander.hip)
// into the workspace.
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

#ifndef HY_GK_FPW
#define HY_GK_FPW 8
#endif
#ifndef HY_GK_U
#define HY_GK_U 1
#endif
constexpr int kGkFramesPerWave = HY_GK_FPW;       // frames per wavefront
constexpr int kGkLanes = 64 / kGkFramesPerWave;   // lanes per frame
constexpr int kGkU = HY_GK_U;                     // windows per lane in flight

__global__ __launch_bounds__(256) void gecko_encode_kernel(hyobfs_gecko_batch B) {
    const uint32_t lane = threadIdx.x & 63, sl = lane % kGkLanes;
    const uint64_t f = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kGkFramesPerWave + lane / kGkLanes;
    if (f >= B.n) return;
    const hyobfs_gecko_frame fr = B.frames[f];
    const uint32_t total = fr.idx_total & 0x0f, idx = fr.idx_total >> 4;
    const uint32_t hp = HYOBFS_GECKO_HEADER_LEN + fr.pad_len;   // chunk start in the plaintext
    const uint32_t plain = hp + fr.chunk_len;
    if (total < HYOBFS_GECKO_MIN_CHUNKS || total > HYOBFS_GECKO_MAX_CHUNKS || idx >= total ||
        HYOBFS_SALT_LEN + plain > HYOBFS_GECKO_BUFFER_SIZE)
        return;   // not a frame writeFragmented can produce: skipped
    // lane handles plaintext windows [16k, 16k+16), k = sl, sl+16, ...: always the same key half
    gk_u128 kh;
    __builtin_memcpy(&kh, static_cast<const uint8_t*>(B.workspace) + 32 * f + 16 * (sl & 1), 16);
    uint8_t* __restrict__ out = B.out + B.out_off[f];
    if (sl == 0) {
        const uint64_t salt = B.salts[f];
        __builtin_memcpy(out, &salt, HYOBFS_SALT_LEN);
    }
    uint8_t* __restrict__ po = out + HYOBFS_SALT_LEN;
    const uint8_t* __restrict__ chunk = B.msg + fr.chunk_off;
    const uint64_t pad0 = f * HYOBFS_GECKO_BUFFER_SIZE;   // this frame's window of the pad stream
    // 0x80 | msgID | idx<<4|total | padLen big-endian, as the low 5 bytes of a window
    const gk_u128 hdr = (gk_u128)HYOBFS_GECKO_FLAG_FRAGMENT | (gk_u128)fr.msg_id << 8 | (gk_u128)fr.idx_total << 16 |
                        (gk_u128)(fr.pad_len >> 8) << 24 | (gk_u128)(fr.pad_len & 0xff) << 32;
    // pad byte at plaintext position q is byte pad0 + q of the stream: a window's 16
    // bytes are exactly two SplitMix64 words (pad0 and p are multiples of 16)
    auto stream16 = [&](uint32_t p) -> gk_u128 {
#ifdef HY_X_NOPAD   // ablation builds only (timing experiments; wrong output)
        return (gk_u128)(pad0 + p);
#else
        const uint64_t w = (pad0 + p) >> 3;
        return (gk_u128)gk_sm64(B.pad_seed, w + 1) << 64 | gk_sm64(B.pad_seed, w);
#endif
    };
    auto window = [&](uint32_t p) -> gk_u128 {   // plaintext bytes [p, p+16) ^ key, p < plain
        const uint32_t e = min(p + 16, plain);
        gk_u128 v = 0;
        if (p == 0) v = hdr & gk_mask(0, min(e, (uint32_t)HYOBFS_GECKO_HEADER_LEN));
        const uint32_t plo = max(p, (uint32_t)HYOBFS_GECKO_HEADER_LEN), phi = min(e, hp);
        if (plo < phi) {   // padding bytes of the window
            v |= stream16(p) & gk_mask(plo - p, phi - p);
        }
        const uint32_t clo = max(p, hp);
        if (clo < e) {     // chunk bytes of the window
            gk_u128 X = 0;
            if (p >= hp && p + 16 <= plain) {
                X = gk_load16u(chunk + (p - hp));
            } else if (fr.chunk_len >= 16) {   // first or last window of the chunk: one in-bounds load, shifted
                X = p < hp ? gk_load16u(chunk) << (8 * (hp - p))
                           : gk_load16u(chunk + (fr.chunk_len - 16)) >> (8 * (p + 16 - plain));
            } else {
                for (uint32_t j = clo; j < e; ++j) X |= (gk_u128)chunk[j - hp] << (8 * (j - p));
            }
            v |= X & gk_mask(clo - p, e - p);
        }
        return v ^ kh;
    };
    constexpr uint32_t STEP = 16 * kGkLanes;   // bytes per pass of the frame's lanes
    for (uint32_t p0 = 16 * sl; p0 < plain; p0 += STEP * kGkU) {
        gk_u128 v[kGkU];
#pragma unroll
        for (int u = 0; u < kGkU; ++u) {   // all windows' loads first
            const uint32_t p = p0 + STEP * u;
            v[u] = p < plain ? window(p) : (gk_u128)0;
        }
#pragma unroll
        for (int u = 0; u < kGkU; ++u) {
            const uint32_t p = p0 + STEP * u;
            if (p + 16 <= plain) {
                gk_store16u(po + p, v[u]);
            } else if (p < plain) {   // the frame's last partial window
                for (uint32_t j = p; j < plain; ++j) po[j] = (uint8_t)(v[u] >> (8 * (j - p)));
            }
        }
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
    const uint64_t per_block = 4 * kGkFramesPerWave;
    hipLaunchKernelGGL(gecko_encode_kernel, dim3((uint32_t)((b.n + per_block - 1) / per_block)), dim3(256), 0, s, b);
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
