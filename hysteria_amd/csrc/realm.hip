// realm.hip -- realm hole-punch packet mask (include/hyobfs_realm.h).
//
// mask = SHA-256(obfsKey(32) || salt(8)) (punch.go:133-141): a 40-byte message,
// so one SHA-256 compression of a single padded block (FIPS 180-4).  The match
// kernel gives one thread to each received datagram and walks the registered
// attempts in order (punch_conn.go:146-165); only the first 25 plain bytes
// (magic, type, nonce) decide, so it loads 33 bytes per datagram.  The host
// entry points (encode / decode / mask) share the same compression code.
#include "kernels.h"
#include "../../include/hyobfs_realm.h"

namespace hyobfs {

#define HY_HD __host__ __device__ __forceinline__

HY_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// One SHA-256 compression of the block holding key || salt (already padded).
HY_HD void sha256_key_salt(const uint8_t key[32], const uint8_t salt[8], uint8_t mask[32]) {
    const uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    const uint32_t H0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                            0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint32_t w[64];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        w[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 | (uint32_t)key[4 * i + 2] << 8 | key[4 * i + 3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
        w[8 + i] = (uint32_t)salt[4 * i] << 24 | (uint32_t)salt[4 * i + 1] << 16 | (uint32_t)salt[4 * i + 2] << 8 |
                   salt[4 * i + 3];
    w[10] = 0x80000000u;   // the 0x80 terminator
#pragma unroll
    for (int i = 11; i < 15; ++i) w[i] = 0;
    w[15] = 40 * 8;        // message length in bits
#pragma unroll
    for (int i = 16; i < 64; ++i) {
        const uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        const uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = H0[0], b = H0[1], c = H0[2], d = H0[3], e = H0[4], f = H0[5], g = H0[6], h = H0[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const uint32_t t1 = h + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
        const uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    const uint32_t o[8] = {H0[0] + a, H0[1] + b, H0[2] + c, H0[3] + d, H0[4] + e, H0[5] + f, H0[6] + g, H0[7] + h};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        mask[4 * i] = (uint8_t)(o[i] >> 24);
        mask[4 * i + 1] = (uint8_t)(o[i] >> 16);
        mask[4 * i + 2] = (uint8_t)(o[i] >> 8);
        mask[4 * i + 3] = (uint8_t)o[i];
    }
}

__constant__ uint8_t kPunchMagic[8] = {'H', 'Y', 'R', 'L', 'M', 'v', '1', 0};
static const uint8_t kPunchMagicHost[8] = {'H', 'Y', 'R', 'L', 'M', 'v', '1', 0};

// DecodePunchPacket's checks after the length checks (punch.go:86-99), on the first 25 plain bytes.
template <class MagicT>
HY_HD int punch_check(const uint8_t head[HYOBFS_PUNCH_HEADER_LEN], const uint8_t* nonce, const MagicT& magic) {
    for (int i = 0; i < 8; ++i)
        if (head[i] != magic[i]) return HYOBFS_PUNCH_ERR_BAD_MAGIC;
    if (head[8] != HYOBFS_PUNCH_HELLO && head[8] != HYOBFS_PUNCH_ACK) return HYOBFS_PUNCH_ERR_UNKNOWN_TYPE;
    for (int i = 0; i < HYOBFS_PUNCH_NONCE_LEN; ++i)
        if (head[9 + i] != nonce[i]) return HYOBFS_PUNCH_ERR_NONCE_MISMATCH;
    return HYOBFS_OK;
}

__global__ __launch_bounds__(256) void punch_match_kernel(const uint8_t* in, const uint64_t* in_off,
                                                          const uint32_t* in_len, uint64_t n,
                                                          const hyobfs_punch_attempt* attempts, uint32_t m,
                                                          int32_t* match, uint8_t* type, uint32_t* padding) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t len = in_len[i];
    int32_t hit = -1;
    uint8_t ty = 0;
    if (len >= HYOBFS_PUNCH_MIN_WIRE_LEN && len <= HYOBFS_PUNCH_MAX_WIRE_LEN) {
        const uint8_t* p = in + in_off[i];
        uint8_t salt[8], enc[HYOBFS_PUNCH_HEADER_LEN];
        for (int k = 0; k < 8; ++k) salt[k] = p[k];
        for (int k = 0; k < HYOBFS_PUNCH_HEADER_LEN; ++k) enc[k] = p[8 + k];
        for (uint32_t j = 0; j < m && hit < 0; ++j) {
            const hyobfs_punch_attempt& a = attempts[j];
            uint8_t mask[32], head[HYOBFS_PUNCH_HEADER_LEN];
            sha256_key_salt(a.key, salt, mask);
            for (int k = 0; k < HYOBFS_PUNCH_HEADER_LEN; ++k) head[k] = enc[k] ^ mask[k];
            if (punch_check(head, a.nonce, kPunchMagic) == HYOBFS_OK) {
                hit = (int32_t)j;
                ty = head[8];
            }
        }
    }
    match[i] = hit;
    if (type) type[i] = ty;
    if (padding) padding[i] = hit >= 0 ? len - HYOBFS_PUNCH_MIN_WIRE_LEN : 0u;
}

hipError_t launch_punch_match(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint64_t n,
                              const hyobfs_punch_attempt* attempts, uint32_t m, int32_t* match, uint8_t* type,
                              uint32_t* padding, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(punch_match_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, in, in_off, in_len, n,
                       attempts, m, match, type, padding);
    return hipGetLastError();
}

}  // namespace hyobfs

extern "C" {

int hyobfs_punch_match_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint64_t n,
                             const hyobfs_punch_attempt* attempts, uint32_t m, int32_t* match, uint8_t* type,
                             uint32_t* padding, void* stream) {
    if (n == 0) return HYOBFS_OK;
    if (!in || !in_off || !in_len || !match || (m && !attempts)) return HYOBFS_ERR_INVALID;
    return hyobfs::launch_punch_match(in, in_off, in_len, n, attempts, m, match, type, padding,
                                      static_cast<hipStream_t>(stream)) == hipSuccess
               ? HYOBFS_OK
               : HYOBFS_ERR_HIP;
}

void hyobfs_punch_mask(const uint8_t key[32], const uint8_t salt[8], uint8_t mask[32]) {
    hyobfs::sha256_key_salt(key, salt, mask);
}

int64_t hyobfs_punch_encode(uint8_t type, const hyobfs_punch_attempt* a, const uint8_t salt[8],
                            const uint8_t* padding, size_t padding_len, uint8_t* out, size_t cap) {
    if (type != HYOBFS_PUNCH_HELLO && type != HYOBFS_PUNCH_ACK) return HYOBFS_PUNCH_ERR_UNKNOWN_TYPE;
    if (!a || !salt || !out || padding_len > HYOBFS_PUNCH_MAX_PADDING || (padding_len && !padding))
        return HYOBFS_ERR_INVALID;
    const size_t total = HYOBFS_PUNCH_MIN_WIRE_LEN + padding_len;
    if (cap < total) return HYOBFS_ERR_INVALID;
    uint8_t mask[32];
    hyobfs::sha256_key_salt(a->key, salt, mask);
    std::memcpy(out, salt, HYOBFS_PUNCH_SALT_LEN);
    uint8_t* plain = out + HYOBFS_PUNCH_SALT_LEN;
    std::memcpy(plain, hyobfs::kPunchMagicHost, 8);
    plain[8] = type;
    std::memcpy(plain + 9, a->nonce, HYOBFS_PUNCH_NONCE_LEN);
    if (padding_len) std::memcpy(plain + HYOBFS_PUNCH_HEADER_LEN, padding, padding_len);
    for (size_t i = 0; i < HYOBFS_PUNCH_HEADER_LEN + padding_len; ++i) plain[i] ^= mask[i % 32];
    return (int64_t)total;
}

int hyobfs_punch_decode(const uint8_t* packet, size_t len, const hyobfs_punch_attempt* a, uint8_t* type,
                        uint32_t* padding_len) {
    if (len < HYOBFS_PUNCH_MIN_WIRE_LEN) return HYOBFS_PUNCH_ERR_TOO_SHORT;
    if (len > HYOBFS_PUNCH_MAX_WIRE_LEN) return HYOBFS_PUNCH_ERR_TOO_LONG;
    if (!packet || !a) return HYOBFS_ERR_INVALID;
    uint8_t mask[32], head[HYOBFS_PUNCH_HEADER_LEN];
    hyobfs::sha256_key_salt(a->key, packet, mask);
    for (int k = 0; k < HYOBFS_PUNCH_HEADER_LEN; ++k) head[k] = packet[8 + k] ^ mask[k];
    const int rc = hyobfs::punch_check(head, a->nonce, hyobfs::kPunchMagicHost);
    if (rc != HYOBFS_OK) return rc;
    if (type) *type = head[8];
    if (padding_len) *padding_len = (uint32_t)(len - HYOBFS_PUNCH_MIN_WIRE_LEN);
    return HYOBFS_OK;
}

}  // extern "C"
