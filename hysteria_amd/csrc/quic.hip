// quic.hip -- QUIC Initial unprotection for the sniffer (include/hyobfs_quic.h).
//
// Reference: apernet/hysteria extras/sniff/internal/quic (header.go, payload.go,
// packet_protector.go, quic.go).  The ciphers are Go's crypto/aes + cipher.GCM
// and golang.org/x/crypto chacha20 / chacha20poly1305 / hkdf, restated from
// FIPS 197, NIST SP 800-38D, RFC 8439, RFC 5869 and FIPS 180-4.
//
// Two kernels:
//   quic_prep_kernel   one LANE per packet: ParseInitialHeader, the version /
//                      length checks of ReadCryptoPayload, and the client
//                      Initial key schedule (HKDF-SHA-256: ~16 compressions)
//                      -> a 96-byte job record per packet in the workspace.
//   quic_open_kernel   one WAVE (a 64-thread workgroup) per packet: header
//                      protection (one AES / ChaCha20 block, computed by every
//                      lane), packet-number decode, AEAD verify (GHASH or
//                      Poly1305 evaluated as a polynomial split over the 64
//                      lanes: lane l takes blocks m-1-l-64t, Horner in H^64 /
//                      r^64, then one multiply by H^(l+1) / r^(l+1) and a
//                      cross-lane reduction), then decrypt in place (a CTR /
//                      ChaCha20 block per lane per step); for ReadCryptoPayload
//                      also the CRYPTO-frame walk (wave-uniform, padding runs
//                      skipped 64 bytes per ballot) and the assembly.
// The path is compute-bound, low volume (the first packets of a connection):
// correctness and per-packet latency matter more than HBM rate here.
#include "kernels.h"
#include "../../include/hyobfs_quic.h"

#include <cstring>
#include <vector>

namespace hyobfs {
namespace quic {

#define QHD __host__ __device__ __forceinline__

// ------------------------------------------------------------------ SHA-256 (FIPS 180-4)
QHD uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
QHD uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

QHD void sha256_compress(uint32_t st[8], const uint32_t blk[16]) {
    const uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = blk[i];
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        if (i >= 16) {
            const uint32_t x = w[(i - 15) & 15], y = w[(i - 2) & 15];
            w[i & 15] += (rotr(x, 7) ^ rotr(x, 18) ^ (x >> 3)) + w[(i - 7) & 15] + (rotr(y, 17) ^ rotr(y, 19) ^ (y >> 10));
        }
        const uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i & 15];
        const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

QHD void sha256_init(uint32_t st[8]) {
    st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
    st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

// HMAC-SHA-256 with a key of at most 64 bytes, as the two chaining states
// after the ipad / opad blocks (RFC 2104).
struct HmacKey {
    uint32_t in[8], out[8];
};

// key: big-endian words of the key zero-padded to 64 bytes
QHD void hmac_key(HmacKey& k, const uint32_t key[16]) {
    uint32_t b[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) b[i] = key[i] ^ 0x36363636u;
    sha256_init(k.in);
    sha256_compress(k.in, b);
#pragma unroll
    for (int i = 0; i < 16; ++i) b[i] = key[i] ^ 0x5c5c5c5cu;
    sha256_init(k.out);
    sha256_compress(k.out, b);
}

// a 32-byte key given as 8 big-endian words
QHD void hmac_key32(HmacKey& k, const uint32_t key[8]) {
    uint32_t b[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = key[i];
#pragma unroll
    for (int i = 8; i < 16; ++i) b[i] = 0;
    hmac_key(k, b);
}

// outer hash over the inner digest
QHD void hmac_finish(const HmacKey& k, const uint32_t inner[8], uint32_t mac[8]) {
    uint32_t b[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = inner[i];
    b[8] = 0x80000000u;
#pragma unroll
    for (int i = 9; i < 15; ++i) b[i] = 0;
    b[15] = (64 + 32) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) mac[i] = k.out[i];
    sha256_compress(mac, b);
}

// HMAC of a message that fits one padded block (blk already padded, with the
// bit length counting the 64-byte ipad block).
QHD void hmac_block(const HmacKey& k, const uint32_t blk[16], uint32_t mac[8]) {
    uint32_t inner[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) inner[i] = k.in[i];
    sha256_compress(inner, blk);
    hmac_finish(k, inner, mac);
}

// ------------------------------------------------------------------ header parse (header.go:24-89)
struct Hdr {
    int status;
    uint8_t type, dl, sl;
    uint32_t version;
    uint32_t dcid_off, scid_off, token_off, token_len;
    uint64_t length;
    int64_t offset;
};

// quicvarint.Read: 1/2/4/8-byte big-endian with the length in the top 2 bits
QHD bool read_varint(const uint8_t* p, uint64_t len, uint64_t& i, uint64_t& v) {
    if (i >= len) return false;
    const uint32_t n = 1u << (p[i] >> 6);
    if (len - i < n) return false;
    v = p[i] & 0x3f;
    for (uint32_t k = 1; k < n; ++k) v = (v << 8) | p[i + k];
    i += n;
    return true;
}

QHD Hdr parse_initial_header(const uint8_t* p, uint64_t len) {
    Hdr h{};
    h.status = HYOBFS_QUIC_ERR_EOF;
    if (len < 5) return h;   // type byte + 4-byte version (ReadByte / io.ReadFull)
    h.type = p[0];
    h.version = (uint32_t)p[1] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 8 | p[4];
    if (h.version != 0 && (h.type & 0x40) == 0) {
        h.status = HYOBFS_QUIC_ERR_NOT_QUIC;
        return h;
    }
    uint64_t i = 5;
    // a connection ID that runs past the end is io.EOF, or (none of it
    // present) makes the next read fail with io.EOF: EOF either way
    if (i >= len) return h;
    h.dl = p[i++];
    if (len - i < h.dl) return h;
    h.dcid_off = (uint32_t)i;
    i += h.dl;
    if (i >= len) return h;
    h.sl = p[i++];
    if (len - i < h.sl) return h;
    h.scid_off = (uint32_t)i;
    i += h.sl;
    const uint32_t initial_type = h.version == HYOBFS_QUIC_V2 ? 1u : 0u;
    if (((h.type >> 4) & 3u) == initial_type) {
        uint64_t tl;
        if (!read_varint(p, len, i, tl)) return h;
        if (tl > len - i) return h;
        h.token_off = (uint32_t)i;
        h.token_len = (uint32_t)tl;
        i += tl;
    }
    if (!read_varint(p, len, i, h.length)) return h;
    h.offset = (int64_t)i;
    h.status = HYOBFS_OK;
    return h;
}

// decodePacketNumber (packet_protector.go:161-174), with Go's wrapping int64
QHD int64_t decode_packet_number(int64_t largest, int64_t truncated, uint32_t nbytes) {
    const int64_t expected = (int64_t)((uint64_t)largest + 1);
    const int64_t win = (int64_t)1 << (nbytes * 8);
    const int64_t hwin = win / 2;
    const int64_t mask = win - 1;
    const int64_t candidate = (expected & ~mask) | truncated;
    if (candidate <= (int64_t)((uint64_t)expected - (uint64_t)hwin) && candidate < ((int64_t)1 << 62) - win)
        return (int64_t)((uint64_t)candidate + (uint64_t)win);
    if (candidate > (int64_t)((uint64_t)expected + (uint64_t)hwin) && candidate >= win)
        return candidate - win;
    return candidate;
}

// One HKDF-Expand-Label message block: info(L, "tls13 "+label, "") || 0x01,
// padded, bit length counting the ipad block (packet_protector.go:177-193).
inline void label_block(const char* label, uint32_t L, uint32_t blk[16]) {
    uint8_t b[64] = {};
    const size_t ll = std::strlen(label);
    size_t i = 0;
    b[i++] = (uint8_t)(L >> 8);
    b[i++] = (uint8_t)L;
    b[i++] = (uint8_t)(6 + ll);
    std::memcpy(b + i, "tls13 ", 6);
    i += 6;
    std::memcpy(b + i, label, ll);
    i += ll;
    b[i++] = 0;   // empty context
    b[i++] = 1;   // T(1) counter
    const uint32_t bits = (uint32_t)(64 + i) * 8;
    b[i] = 0x80;
    b[62] = (uint8_t)(bits >> 8);
    b[63] = (uint8_t)bits;
    for (int k = 0; k < 16; ++k)
        blk[k] = (uint32_t)b[4 * k] << 24 | (uint32_t)b[4 * k + 1] << 16 | (uint32_t)b[4 * k + 2] << 8 | b[4 * k + 3];
}

const uint8_t kSaltOld[20] = {0xaf, 0xbf, 0xec, 0x28, 0x99, 0x93, 0xd2, 0x4c, 0x9e, 0x97,
                              0x86, 0xf1, 0x9c, 0x61, 0x11, 0xe0, 0x43, 0x90, 0xa8, 0x99};
const uint8_t kSaltV1[20] = {0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17,
                             0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad, 0xcc, 0xbb, 0x7f, 0x0a};
const uint8_t kSaltV2[20] = {0x0d, 0xed, 0xe3, 0xde, 0xf7, 0x00, 0xa6, 0xdb, 0x81, 0x93,
                             0x81, 0xbe, 0x6e, 0x26, 0x9d, 0xcb, 0xf9, 0xbd, 0x2e, 0xd9};

// getSalt (quic.go:28-36)
inline const uint8_t* get_salt(uint32_t v) {
    return v == HYOBFS_QUIC_V1 ? kSaltV1 : v == HYOBFS_QUIC_V2 ? kSaltV2 : kSaltOld;
}

inline void key_words(const uint8_t* key, size_t n, uint32_t w[16]) {
    uint8_t b[64] = {};
    std::memcpy(b, key, n);
    for (int k = 0; k < 16; ++k)
        w[k] = (uint32_t)b[4 * k] << 24 | (uint32_t)b[4 * k + 1] << 16 | (uint32_t)b[4 * k + 2] << 8 | b[4 * k + 3];
}

QHD void words_to_bytes(const uint32_t* w, uint8_t* out, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) out[i] = (uint8_t)(w[i / 4] >> (24 - 8 * (i % 4)));
}

// Everything the prep kernel needs that depends only on constants: the
// HMAC states of the two Initial salts and the HKDF-Expand-Label blocks.
struct PrepConsts {
    HmacKey salt[2];         // V1, V2
    uint32_t client_in[16];  // "client in", 32
    uint32_t key[2][16];     // "quic key" / "quicv2 key", 16
    uint32_t iv[2][16];      // "quic iv" / "quicv2 iv", 12
    uint32_t hp[2][16];      // "quic hp" / "quicv2 hp", 16
};

inline PrepConsts make_prep_consts() {
    PrepConsts c{};
    uint32_t w[16];
    key_words(kSaltV1, 20, w);
    hmac_key(c.salt[0], w);
    key_words(kSaltV2, 20, w);
    hmac_key(c.salt[1], w);
    label_block("client in", 32, c.client_in);
    label_block("quic key", 16, c.key[0]);
    label_block("quicv2 key", 16, c.key[1]);
    label_block("quic iv", 12, c.iv[0]);
    label_block("quicv2 iv", 12, c.iv[1]);
    label_block("quic hp", 16, c.hp[0]);
    label_block("quicv2 hp", 16, c.hp[1]);
    return c;
}

// per-packet record written by the prep kernel
struct Job {
    hyobfs_quic_key key;
    int64_t pn_offset;
    uint32_t len;    // offset + Length: the slice UnProtect sees
    int32_t status;
};
static_assert(sizeof(Job) == 96, "job record layout");
static_assert(sizeof(hyobfs_quic_key) == 80, "hyobfs_quic_key layout");
static_assert(sizeof(hyobfs_quic_result) == 24, "hyobfs_quic_result layout");

// ------------------------------------------------------------------ AES-128 (FIPS 197), T-table in LDS
__constant__ uint8_t kSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76, 0xca, 0x82, 0xc9,
    0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, 0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f,
    0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15, 0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07,
    0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75, 0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3,
    0x29, 0xe3, 0x2f, 0x84, 0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58,
    0xcf, 0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8, 0x51, 0xa3,
    0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2, 0xcd, 0x0c, 0x13, 0xec, 0x5f,
    0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73, 0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88,
    0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb, 0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac,
    0x62, 0x91, 0x95, 0xe4, 0x79, 0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a,
    0xae, 0x08, 0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a, 0x70,
    0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, 0xe1, 0xf8, 0x98, 0x11,
    0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf, 0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42,
    0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

// Te[x] = (2s, s, s, 3s) as little-endian bytes, s = S[x]; S[x] = (Te[x] >> 8) & 0xff.
__device__ __forceinline__ void aes_table_load(uint32_t* te, uint32_t lane) {
    for (uint32_t x = lane; x < 256; x += 64) {
        const uint32_t s = kSbox[x];
        const uint32_t s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff;
        te[x] = s2 | s << 8 | s << 16 | (s2 ^ s) << 24;
    }
}

__device__ __forceinline__ uint32_t sub_word(const uint32_t* te, uint32_t w) {
    return ((te[w & 0xff] >> 8) & 0xff) | (te[(w >> 8) & 0xff] & 0xff00) | ((te[(w >> 16) & 0xff] << 8) & 0xff0000) |
           ((te[w >> 24] << 16) & 0xff000000u);
}

// round keys as little-endian column words, written to LDS as they are made
// (a 4-word window in registers); called by one lane
__device__ __forceinline__ void aes_expand_to(const uint32_t* te, const uint32_t k[4], uint32_t* dst) {
    uint32_t w0 = k[0], w1 = k[1], w2 = k[2], w3 = k[3];
    dst[0] = w0; dst[1] = w1; dst[2] = w2; dst[3] = w3;
    uint32_t rcon = 1;
#pragma unroll
    for (int r = 1; r <= 10; ++r) {
        w0 ^= sub_word(te, (w3 >> 8) | (w3 << 24)) ^ rcon;
        w1 ^= w0;
        w2 ^= w1;
        w3 ^= w2;
        rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1b : 0)) & 0xff;
        dst[4 * r] = w0; dst[4 * r + 1] = w1; dst[4 * r + 2] = w2; dst[4 * r + 3] = w3;
    }
}

// round keys as little-endian column words
__device__ __forceinline__ void aes_expand(const uint32_t* te, const uint32_t k[4], uint32_t rk[44]) {
    rk[0] = k[0]; rk[1] = k[1]; rk[2] = k[2]; rk[3] = k[3];
    uint32_t rcon = 1;
#pragma unroll
    for (int i = 4; i < 44; ++i) {
        uint32_t t = rk[i - 1];
        if (i % 4 == 0) {
            t = sub_word(te, (t >> 8) | (t << 24)) ^ rcon;
            rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1b : 0)) & 0xff;
        }
        rk[i] = rk[i - 4] ^ t;
    }
}

__device__ __forceinline__ void aes_encrypt(const uint32_t* te, const uint32_t* rk, const uint32_t in[4],
                                            uint32_t out[4]) {
    uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const uint32_t t0 = te[s0 & 0xff] ^ rotl(te[(s1 >> 8) & 0xff], 8) ^ rotl(te[(s2 >> 16) & 0xff], 16) ^
                            rotl(te[s3 >> 24], 24) ^ rk[4 * r];
        const uint32_t t1 = te[s1 & 0xff] ^ rotl(te[(s2 >> 8) & 0xff], 8) ^ rotl(te[(s3 >> 16) & 0xff], 16) ^
                            rotl(te[s0 >> 24], 24) ^ rk[4 * r + 1];
        const uint32_t t2 = te[s2 & 0xff] ^ rotl(te[(s3 >> 8) & 0xff], 8) ^ rotl(te[(s0 >> 16) & 0xff], 16) ^
                            rotl(te[s1 >> 24], 24) ^ rk[4 * r + 2];
        const uint32_t t3 = te[s3 & 0xff] ^ rotl(te[(s0 >> 8) & 0xff], 8) ^ rotl(te[(s1 >> 16) & 0xff], 16) ^
                            rotl(te[s2 >> 24], 24) ^ rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    auto sb = [&](uint32_t x) { return (te[x] >> 8) & 0xff; };
    out[0] = (sb(s0 & 0xff) | sb((s1 >> 8) & 0xff) << 8 | sb((s2 >> 16) & 0xff) << 16 | sb(s3 >> 24) << 24) ^ rk[40];
    out[1] = (sb(s1 & 0xff) | sb((s2 >> 8) & 0xff) << 8 | sb((s3 >> 16) & 0xff) << 16 | sb(s0 >> 24) << 24) ^ rk[41];
    out[2] = (sb(s2 & 0xff) | sb((s3 >> 8) & 0xff) << 8 | sb((s0 >> 16) & 0xff) << 16 | sb(s1 >> 24) << 24) ^ rk[42];
    out[3] = (sb(s3 & 0xff) | sb((s0 >> 8) & 0xff) << 8 | sb((s1 >> 16) & 0xff) << 16 | sb(s2 >> 24) << 24) ^ rk[43];
}

// ------------------------------------------------------------------ GF(2^128) (SP 800-38D 6.3)
// Block as a 128-bit big-endian integer (h = bytes 0..7, l = bytes 8..15);
// bit 0 of the field element is the MSB of byte 0.
struct G128 {
    uint64_t h, l;
};

QHD uint32_t bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xff00) | ((x << 8) & 0xff0000) | (x << 24);
}

// 16 block bytes as 4 little-endian words -> G128
QHD G128 g_from_le(const uint32_t w[4]) {
    return G128{(uint64_t)bswap32(w[0]) << 32 | bswap32(w[1]), (uint64_t)bswap32(w[2]) << 32 | bswap32(w[3])};
}

// times x: one right shift with the reduction x^128 = x^7 + x^2 + x + 1
QHD G128 mulx(G128 v) {
    const uint64_t lsb = 0 - (v.l & 1);
    return G128{(v.h >> 1) ^ (lsb & 0xE100000000000000ull), (v.l >> 1) | (v.h << 63)};
}

// P^2: squaring is linear over GF(2): spread the bits of the natural-order
// polynomial (bit i = x^i, the bit reversal of GCM's order), then fold the
// upper 128 bits with x^128 = x^7 + x^2 + x + 1
QHD uint64_t spread32(uint64_t x) {
    x = (x | x << 16) & 0x0000FFFF0000FFFFull;
    x = (x | x << 8) & 0x00FF00FF00FF00FFull;
    x = (x | x << 4) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | x << 2) & 0x3333333333333333ull;
    return (x | x << 1) & 0x5555555555555555ull;
}

QHD G128 gf_sqr(G128 v) {
    const uint64_t n0 = __builtin_bitreverse64(v.h), n1 = __builtin_bitreverse64(v.l);
    const uint64_t s0 = spread32(n0 & 0xffffffffu), s1 = spread32(n0 >> 32);
    const uint64_t s2 = spread32(n1 & 0xffffffffu), s3 = spread32(n1 >> 32);
    const uint64_t o = (s3 >> 63) ^ (s3 >> 62) ^ (s3 >> 57);   // degrees 128..134 of the shifted copies
    const uint64_t r0 = s0 ^ s2 ^ (s2 << 1) ^ (s2 << 2) ^ (s2 << 7) ^ o ^ (o << 1) ^ (o << 2) ^ (o << 7);
    const uint64_t r1 = s1 ^ s3 ^ (s3 << 1 | s2 >> 63) ^ (s3 << 2 | s2 >> 62) ^ (s3 << 7 | s2 >> 57);
    return G128{__builtin_bitreverse64(r0), __builtin_bitreverse64(r1)};
}

// Shoup's 4-bit tables (a wave-uniform multiplier P): tab[i] = P * i(x), nibble
// bit 3 = x^0 .. bit 0 = x^3 in GCM's reflected order; lanes 0..15 write one each.
__device__ __forceinline__ void shoup_build(G128* tab, G128 P, uint32_t lane) {
    if (lane < 16) {
        const G128 p1 = mulx(P), p2 = mulx(p1), p3 = mulx(p2);
        G128 e{0, 0};
        if (lane & 8) { e.h ^= P.h; e.l ^= P.l; }
        if (lane & 4) { e.h ^= p1.h; e.l ^= p1.l; }
        if (lane & 2) { e.h ^= p2.h; e.l ^= p2.l; }
        if (lane & 1) { e.h ^= p3.h; e.l ^= p3.l; }
        tab[lane] = e;
    }
}

// x * P through P's table: Horner over the 32 nibbles of x, last nibble first
__device__ __forceinline__ G128 shoup_mul(G128 x, const G128* tab) {
    G128 z{0, 0};
#pragma unroll 4
    for (int j = 31; j >= 0; --j) {
        if (j != 31) {
            // the 4 dropped bits times x^4: clmul(rem, 0x1C20) in the top 16 bits
            const uint32_t rem = (uint32_t)z.l & 0xf;
            const uint32_t red = ((rem & 1) * 0x1C20u) ^ ((rem & 2) * 0x1C20u) ^ ((rem & 4) * 0x1C20u) ^
                                 ((rem & 8) * 0x1C20u);
            z.l = (z.l >> 4) | (z.h << 60);
            z.h = (z.h >> 4) ^ ((uint64_t)red << 48);
        }
        const uint32_t nib = j >= 16 ? (uint32_t)(x.l >> (4 * (31 - j))) & 0xf : (uint32_t)(x.h >> (4 * (15 - j))) & 0xf;
        const G128 t = tab[nib];
        z.h ^= t.h;
        z.l ^= t.l;
    }
    return z;
}

// ------------------------------------------------------------------ ChaCha20 (RFC 8439 2.3)
QHD void chacha_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d = rotl(d ^ a, 16);
    c += d; b = rotl(b ^ c, 12);
    a += b; d = rotl(d ^ a, 8);
    c += d; b = rotl(b ^ c, 7);
}

QHD void chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], uint32_t out[16]) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4],      key[5],      key[6],      key[7],      counter, nonce[0], nonce[1], nonce[2]};
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = s[i];
    for (int r = 0; r < 10; ++r) {
        chacha_qr(x[0], x[4], x[8], x[12]);
        chacha_qr(x[1], x[5], x[9], x[13]);
        chacha_qr(x[2], x[6], x[10], x[14]);
        chacha_qr(x[3], x[7], x[11], x[15]);
        chacha_qr(x[0], x[5], x[10], x[15]);
        chacha_qr(x[1], x[6], x[11], x[12]);
        chacha_qr(x[2], x[7], x[8], x[13]);
        chacha_qr(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

// ------------------------------------------------------------------ Poly1305 (RFC 8439 2.5), 26-bit limbs
struct P130 {
    uint32_t v[5];
};

QHD P130 p_mul(const P130& a, const P130& r) {
    const uint64_t r0 = r.v[0], r1 = r.v[1], r2 = r.v[2], r3 = r.v[3], r4 = r.v[4];
    const uint64_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
    const uint64_t a0 = a.v[0], a1 = a.v[1], a2 = a.v[2], a3 = a.v[3], a4 = a.v[4];
    uint64_t d0 = a0 * r0 + a1 * s4 + a2 * s3 + a3 * s2 + a4 * s1;
    uint64_t d1 = a0 * r1 + a1 * r0 + a2 * s4 + a3 * s3 + a4 * s2;
    uint64_t d2 = a0 * r2 + a1 * r1 + a2 * r0 + a3 * s4 + a4 * s3;
    uint64_t d3 = a0 * r3 + a1 * r2 + a2 * r1 + a3 * r0 + a4 * s4;
    uint64_t d4 = a0 * r4 + a1 * r3 + a2 * r2 + a3 * r1 + a4 * r0;
    P130 o;
    uint64_t c = d0 >> 26; o.v[0] = (uint32_t)d0 & 0x3ffffff;
    d1 += c; c = d1 >> 26; o.v[1] = (uint32_t)d1 & 0x3ffffff;
    d2 += c; c = d2 >> 26; o.v[2] = (uint32_t)d2 & 0x3ffffff;
    d3 += c; c = d3 >> 26; o.v[3] = (uint32_t)d3 & 0x3ffffff;
    d4 += c; c = d4 >> 26; o.v[4] = (uint32_t)d4 & 0x3ffffff;
    uint64_t t = (uint64_t)o.v[0] + c * 5;
    o.v[0] = (uint32_t)t & 0x3ffffff;
    o.v[1] += (uint32_t)(t >> 26);
    return o;
}

// 16 little-endian bytes as 4 LE words, plus 2^128 when hibit
QHD P130 p_from_block(const uint32_t w[4], uint32_t hibit) {
    P130 o;
    o.v[0] = w[0] & 0x3ffffff;
    o.v[1] = ((w[0] >> 26) | (w[1] << 6)) & 0x3ffffff;
    o.v[2] = ((w[1] >> 20) | (w[2] << 12)) & 0x3ffffff;
    o.v[3] = ((w[2] >> 14) | (w[3] << 18)) & 0x3ffffff;
    o.v[4] = (w[3] >> 8) | (hibit << 24);
    return o;
}

// ------------------------------------------------------------------ device byte access
__device__ __forceinline__ uint32_t le_word(const uint8_t* p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

// bytes [pos, pos+16) of [0, n) as 4 LE words, zero past n
__device__ __forceinline__ void load_block(const uint8_t* p, uint64_t pos, uint64_t n, uint32_t w[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint64_t q = pos + 4 * k + b;
            x |= (q < n ? (uint32_t)p[q] : 0u) << (8 * b);
        }
        w[k] = x;
    }
}

__device__ __forceinline__ void store_xor(uint8_t* p, uint64_t pos, uint64_t n, const uint32_t* ct, const uint32_t* ks,
                                          int words) {
    for (int k = 0; k < words; ++k) {
        const uint32_t x = ct[k] ^ ks[k];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint64_t q = pos + 4 * k + b;
            if (q < n) p[q] = (uint8_t)(x >> (8 * b));
        }
    }
}

template <class T>
__device__ __forceinline__ T wave_xor(T v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m, 64);
    return v;
}

// ------------------------------------------------------------------ prep kernel
__device__ void hmac_dcid(const HmacKey& k, const uint8_t* dcid, uint32_t dl, uint32_t mac[8]) {
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = k.in[i];
    const uint32_t nb = (dl + 9 + 63) / 64;
    for (uint32_t b = 0; b < nb; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            uint32_t x = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t q = 64 * b + 4 * j + t;
                const uint32_t c = q < dl ? dcid[q] : (q == dl ? 0x80u : 0u);
                x |= c << (24 - 8 * t);
            }
            w[j] = x;
        }
        if (b == nb - 1) w[15] = (64 + dl) * 8;
        sha256_compress(st, w);
    }
    hmac_finish(k, st, mac);
}

__global__ __launch_bounds__(256) void quic_prep_kernel(const uint8_t* packets, const uint64_t* off,
                                                        const uint32_t* len, uint64_t n, Job* jobs,
                                                        PrepConsts c) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = packets + off[i];
    const uint32_t L = len[i];
    Job j{};
    j.key.suite = HYOBFS_QUIC_TLS_AES_128_GCM_SHA256;
    // ReadCryptoPayload's checks (payload.go:22-46)
    const Hdr h = parse_initial_header(p, L);
    int st = h.status;
    if (st == HYOBFS_OK && h.version != HYOBFS_QUIC_V1 && h.version != HYOBFS_QUIC_V2) st = HYOBFS_QUIC_ERR_VERSION;
    if (st == HYOBFS_OK && (h.offset == 0 || h.length == 0)) st = HYOBFS_QUIC_ERR_INVALID;
    if (st == HYOBFS_OK && (uint64_t)L - (uint64_t)h.offset < h.length) st = HYOBFS_QUIC_ERR_SHORT;
    if (st == HYOBFS_OK) {
        const int v = h.version == HYOBFS_QUIC_V2;
        uint32_t secret[8], mac[8];
        hmac_dcid(c.salt[v], p + h.dcid_off, h.dl, secret);   // HKDF-Extract
        HmacKey k;
        hmac_key32(k, secret);
        hmac_block(k, c.client_in, secret);                    // "client in"
        hmac_key32(k, secret);
        hmac_block(k, c.key[v], mac);
        words_to_bytes(mac, j.key.key, 16);
        hmac_block(k, c.iv[v], mac);
        words_to_bytes(mac, j.key.iv, 12);
        hmac_block(k, c.hp[v], mac);
        words_to_bytes(mac, j.key.hp, 16);
        j.pn_offset = h.offset;
        j.len = (uint32_t)((uint64_t)h.offset + h.length);
    }
    j.status = st;
    jobs[i] = j;
}

// ------------------------------------------------------------------ open kernel
struct Frame {
    uint64_t off;
    uint32_t len;
    uint32_t pos;
};

struct OpenArgs {
    uint8_t* packets;
    const uint64_t* off;
    const uint32_t* len;
    uint64_t n;
    const hyobfs_quic_key* keys;
    uint32_t key_stride;
    const int64_t* pn_offset;
    const int64_t* pn_max;
    const Job* jobs;
    hyobfs_quic_result* res;
    uint8_t* out;
    const uint64_t* out_off;
    const uint32_t* out_cap;
};

// wave-uniform byte reader over [0, n): each lane holds one byte of a 64-byte window
struct Window {
    const uint8_t* p;
    uint64_t n, base;
    uint32_t mine;
    __device__ void fill(uint64_t at, uint32_t lane) {
        base = at;
        mine = at + lane < n ? p[at + lane] : 0u;
    }
    __device__ uint32_t get(uint64_t i, uint32_t lane) {
        if (i < base || i >= base + 64) fill(i, lane);
        return (uint32_t)__shfl((int)mine, (int)(i - base), 64) & 0xff;
    }
    __device__ bool varint(uint64_t& i, uint64_t& v, uint32_t lane) {
        if (i >= n) return false;
        const uint32_t b0 = get(i, lane);
        const uint32_t k = 1u << (b0 >> 6);
        if (n - i < k) return false;
        v = b0 & 0x3f;
        for (uint32_t t = 1; t < k; ++t) v = (v << 8) | get(i + t, lane);
        i += k;
        return true;
    }
};

#ifndef HY_QUIC_MIN_WAVES
#define HY_QUIC_MIN_WAVES 4   // waves per SIMD the open kernel is register-capped for
#endif

template <bool CRYPTO>
__global__ __launch_bounds__(64, HY_QUIC_MIN_WAVES) void quic_open_kernel(OpenArgs a) {
    __shared__ uint32_t te[256];
    __shared__ G128 gtab[7][16];   // GHASH: Shoup tables of H^(2^k)
    __shared__ uint32_t rkl[44];   // AES-128 round keys of the packet's AEAD key
    __shared__ uint32_t hrkl[44];  // ... and of its header-protection key
    __shared__ Frame fr[HYOBFS_QUIC_MAX_FRAMES];
    __shared__ uint16_t order[HYOBFS_QUIC_MAX_FRAMES];
    const uint32_t lane = threadIdx.x & 63;
    aes_table_load(te, lane);

    for (uint64_t pk = blockIdx.x; pk < a.n; pk += gridDim.x) {
        __syncthreads();   // the previous packet's LDS reads are done
        uint8_t* p = a.packets + a.off[pk];
        hyobfs_quic_key key;
        int64_t pn_off, pn_max;
        uint64_t L;
        int st = HYOBFS_OK;
        if (CRYPTO) {
            const Job& j = a.jobs[pk];
            st = j.status;
            key = j.key;
            pn_off = j.pn_offset;
            pn_max = 2;   // payload.go:47
            L = j.len;
        } else {
            key = a.keys[pk * a.key_stride];
            pn_off = a.pn_offset[pk];
            pn_max = a.pn_max ? a.pn_max[pk] : 0;
            L = a.len[pk];
        }
        hyobfs_quic_result r{};
        // UnProtect (packet_protector.go:46-79)
        if (st == HYOBFS_OK && (pn_off < 0 || (uint64_t)pn_off > L || L - (uint64_t)pn_off < 20))
            st = HYOBFS_QUIC_ERR_TOO_SMALL;
        const bool aes = CRYPTO || key.suite == HYOBFS_QUIC_TLS_AES_128_GCM_SHA256;   // Initial packets: AES-128-GCM
        if (st == HYOBFS_OK && !aes && key.suite != HYOBFS_QUIC_TLS_CHACHA20_POLY1305_SHA256)
            st = HYOBFS_QUIC_ERR_SUITE;
        if (st != HYOBFS_OK) {
            if (lane == 0) {
                r.status = st;
                a.res[pk] = r;
            }
            continue;
        }
        uint32_t kw[8], ivw[3], hpw[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) kw[k] = le_word(key.key + 4 * k);
#pragma unroll
        for (int k = 0; k < 3; ++k) ivw[k] = le_word(key.iv + 4 * k);
#pragma unroll
        for (int k = 0; k < 8; ++k) hpw[k] = le_word(key.hp + 4 * k);

        // header protection mask from the 16-byte sample at pnOffset + 4
        uint32_t sample[4], mw0, mw1;
        load_block(p, (uint64_t)pn_off + 4, L, sample);
        const uint32_t* rk = rkl;   // round keys live in LDS: registers stay free for occupancy
        if (aes) {
            uint32_t m[4];
            if (lane == 0) {
                aes_expand_to(te, hpw, hrkl);
                aes_expand_to(te, kw, rkl);
            }
            __syncthreads();
            aes_encrypt(te, hrkl, sample, m);
            mw0 = m[0];
            mw1 = m[1];
        } else {
            uint32_t ks[16];
            chacha20_block(hpw, sample[0], sample + 1, ks);
            mw0 = ks[0];
            mw1 = ks[1];
        }
        const uint32_t b0 = p[0];
        const bool long_hdr = (b0 & 0x80) != 0;
        const uint32_t first = b0 ^ (mw0 & (long_hdr ? 0x0fu : 0x1fu));
        const uint32_t pn_len = (first & 3) + 1;
        const uint32_t pmask = (mw0 >> 8) | (mw1 << 24);   // mask[1..4]
        int64_t trunc = 0;
        for (uint32_t k = 0; k < pn_len; ++k)
            trunc = (trunc << 8) | ((p[pn_off + k] ^ (pmask >> (8 * k))) & 0xff);
        const int64_t pn = decode_packet_number(pn_max, trunc, pn_len);
        const uint64_t hdr_len = (uint64_t)pn_off + pn_len;
        r.pn = pn;
        r.hdr_len = (uint32_t)hdr_len;
        // nonce = iv ^ (0^32 || BE64(pn))  (packet_protector.go:93-100)
        uint32_t nonce[3] = {ivw[0], ivw[1] ^ bswap32((uint32_t)((uint64_t)pn >> 32)),
                             ivw[2] ^ bswap32((uint32_t)(uint64_t)pn)};
        const uint64_t payload = L - hdr_len;
        bool ok = payload >= 16;
        const uint64_t ct_len = ok ? payload - 16 : 0;
        uint8_t* ct = p + hdr_len;
        // AAD = the unmasked header: substitute the unmasked bytes on the fly
        auto aad_block = [&](uint64_t pos, uint32_t w[4]) {
            load_block(p, pos, hdr_len, w);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint64_t q = pos + k;
                uint32_t fix = 0;
                if (q == 0) fix = (b0 ^ first) & 0xff;
                else if (q >= (uint64_t)pn_off && q < hdr_len) fix = (pmask >> (8 * (q - pn_off))) & 0xff;
                w[k / 4] ^= fix << (8 * (k % 4));
            }
        };
        const uint64_t aad_blocks = (hdr_len + 15) / 16, ct_blocks = (ct_len + 15) / 16;
        const uint64_t m = aad_blocks + ct_blocks + 1;   // + the length block
        auto stream_block = [&](uint64_t s, uint32_t w[4], bool le_lengths) {
            if (s < aad_blocks) {
                aad_block(16 * s, w);
            } else if (s < aad_blocks + ct_blocks) {
                load_block(ct, 16 * (s - aad_blocks), ct_len, w);
            } else if (le_lengths) {   // Poly1305: LE64(aad) || LE64(ct)
                w[0] = (uint32_t)hdr_len; w[1] = (uint32_t)(hdr_len >> 32);
                w[2] = (uint32_t)ct_len; w[3] = (uint32_t)(ct_len >> 32);
            } else {                   // GHASH: BE64(aad bits) || BE64(ct bits), as LE words of those bytes
                const uint64_t ab = hdr_len * 8, cb = ct_len * 8;
                w[0] = bswap32((uint32_t)(ab >> 32)); w[1] = bswap32((uint32_t)ab);
                w[2] = bswap32((uint32_t)(cb >> 32)); w[3] = bswap32((uint32_t)cb);
            }
        };
        const uint64_t nt = lane < m ? (m - 1 - lane) / 64 + 1 : 0;   // blocks this lane takes
        uint32_t tagw[4];
        if (ok) load_block(p, L - 16, L, tagw);
        if (ok && aes) {
            // H = E(K, 0) and Shoup tables of H^(2^k), k = 0..6
            const uint32_t zero[4] = {0, 0, 0, 0};
            uint32_t hw[4];
            aes_encrypt(te, rk, zero, hw);
            G128 P = g_from_le(hw);
            shoup_build(gtab[0], P, lane);
            for (int k = 1; k < 7; ++k) {
                P = gf_sqr(P);
                shoup_build(gtab[k], P, lane);
            }
            __syncthreads();
            // lane l: acc_l = sum_t X_{m-1-l-64t} H^(64t), Horner in the uniform H^64
            G128 acc{0, 0};
            for (uint64_t t = nt; t-- > 0;) {
                uint32_t w[4];
                stream_block(m - 1 - lane - 64 * t, w, false);
                const G128 x = g_from_le(w);
                if (t + 1 != nt) acc = shoup_mul(acc, gtab[6]);
                acc.h ^= x.h;
                acc.l ^= x.l;
            }
            // lane tree: sum_l acc_l H^l, one multiply by the uniform H^(2^k) per level;
            // then times H, so block s carries H^(m-s)
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const int src = (int)((lane + (1u << k)) & 63);
                G128 b{__shfl(acc.h, src, 64), __shfl(acc.l, src, 64)};
                b = shoup_mul(b, gtab[k]);
                acc.h ^= b.h;
                acc.l ^= b.l;
            }
            acc = G128{__shfl(acc.h, 0, 64), __shfl(acc.l, 0, 64)};
            acc = shoup_mul(acc, gtab[0]);
            // tag = E(K, J0) ^ S
            const uint32_t j0[4] = {nonce[0], nonce[1], nonce[2], 0x01000000u};
            uint32_t ej[4];
            aes_encrypt(te, rk, j0, ej);
            const G128 ejg = g_from_le(ej);
            const G128 tg = g_from_le(tagw);
            ok = ((acc.h ^ ejg.h) == tg.h) && ((acc.l ^ ejg.l) == tg.l);
        } else if (ok) {
            // one-time key = ChaCha20(K, 0, nonce)[0:32] (RFC 8439 2.6)
            uint32_t otk[16];
            chacha20_block(kw, 0, nonce, otk);
            const uint32_t rw[4] = {otk[0] & 0x0fffffffu, otk[1] & 0x0ffffffcu, otk[2] & 0x0ffffffcu,
                                    otk[3] & 0x0ffffffcu};
            const P130 R = p_from_block(rw, 0);
            P130 rp[7];
            rp[0] = R;
#pragma unroll
            for (int k = 1; k < 7; ++k) rp[k] = p_mul(rp[k - 1], rp[k - 1]);   // r^(2^k)
            P130 acc{{0, 0, 0, 0, 0}};
            for (uint64_t t = nt; t-- > 0;) {
                uint32_t w[4];
                stream_block(m - 1 - lane - 64 * t, w, true);
                const P130 x = p_from_block(w, 1);
                acc = p_mul(acc, rp[6]);
#pragma unroll
                for (int k = 0; k < 5; ++k) acc.v[k] += x.v[k];
            }
            P130 pw{{1, 0, 0, 0, 0}};
            const uint32_t e = lane + 1;
#pragma unroll
            for (int k = 0; k < 7; ++k)
                if ((e >> k) & 1) pw = p_mul(pw, rp[k]);
            acc = nt ? p_mul(acc, pw) : P130{{0, 0, 0, 0, 0}};
            // sum over lanes (limbs < 2^27 each: the 64-lane sum fits 33 bits)
            uint64_t sum[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                uint64_t v = acc.v[k];
#pragma unroll
                for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
                sum[k] = v;
            }
            // full reduction mod 2^130 - 5
            uint64_t c = 0;
            for (int pass = 0; pass < 3; ++pass) {   // limbs < 2^26, h < 2^130
                for (int k = 0; k < 5; ++k) {
                    sum[k] += c;
                    c = sum[k] >> 26;
                    sum[k] &= 0x3ffffff;
                }
                sum[0] += c * 5;
                c = 0;
            }
            // h >= p  <=>  h + 5 >= 2^130
            uint64_t g[5];
            c = 5;
            for (int k = 0; k < 5; ++k) {
                g[k] = sum[k] + c;
                c = g[k] >> 26;
                g[k] &= 0x3ffffff;
            }
            if (c) for (int k = 0; k < 5; ++k) sum[k] = g[k];
            // to 128 bits + s
            const uint64_t lo = sum[0] | sum[1] << 26 | sum[2] << 52;
            const uint64_t hi = (sum[2] >> 12) | sum[3] << 14 | sum[4] << 40;
            const uint64_t s_lo = (uint64_t)otk[4] | (uint64_t)otk[5] << 32;
            const uint64_t s_hi = (uint64_t)otk[6] | (uint64_t)otk[7] << 32;
            const uint64_t t_lo = lo + s_lo;
            const uint64_t t_hi = hi + s_hi + (t_lo < lo);
            ok = t_lo == ((uint64_t)tagw[0] | (uint64_t)tagw[1] << 32) &&
                 t_hi == ((uint64_t)tagw[2] | (uint64_t)tagw[3] << 32);
        }
        if (ok) {
            // decrypt in place: lane l takes blocks l, l+64, ...
            if (aes) {
                for (uint64_t b = lane; b < ct_blocks; b += 64) {
                    const uint32_t cb[4] = {nonce[0], nonce[1], nonce[2], bswap32((uint32_t)(2 + b))};
                    uint32_t ks[4], w[4];
                    aes_encrypt(te, rk, cb, ks);
                    load_block(ct, 16 * b, ct_len, w);
                    store_xor(ct, 16 * b, ct_len, w, ks, 4);
                }
            } else {
                const uint64_t cblocks = (ct_len + 63) / 64;
                for (uint64_t b = lane; b < cblocks; b += 64) {
                    uint32_t ks[16], w[16];
                    chacha20_block(kw, (uint32_t)(1 + b), nonce, ks);
#pragma unroll
                    for (int q = 0; q < 4; ++q) load_block(ct, 64 * b + 16 * q, ct_len, w + 4 * q);
                    store_xor(ct, 64 * b, ct_len, w, ks, 16);
                }
            }
            r.plain_len = (uint32_t)ct_len;
        } else {
            st = HYOBFS_QUIC_ERR_AUTH;
        }
        // the header stays unmasked whatever the AEAD says (packet_protector.go:57-70)
        if (lane == 0) {
            p[0] = (uint8_t)first;
            for (uint32_t k = 0; k < pn_len; ++k) p[pn_off + k] ^= (uint8_t)(pmask >> (8 * k));
        }
        if (CRYPTO && st == HYOBFS_OK) {
            __syncthreads();   // the plaintext stores of every lane are visible below
            // extractCryptoFrames (payload.go:73-112), wave-uniform
            Window win{ct, ct_len, ~0ull, 0};
            uint64_t i = 0;
            uint32_t nf = 0;
            while (i < ct_len && st == HYOBFS_OK) {
                const uint32_t c0 = win.get(i, lane);
                if (c0 <= 1) {   // a run of one-byte PADDING / PING frames
                    for (;;) {
                        win.fill(i, lane);
                        const unsigned long long live =
                            __ballot(i + lane < ct_len && win.mine > 1u) ;
                        if (live) {
                            i += __builtin_ctzll(live);
                            break;
                        }
                        i += 64;
                        if (i >= ct_len) {
                            i = ct_len;
                            break;
                        }
                    }
                    continue;
                }
                uint64_t typ, fo, dl;
                if (!win.varint(i, typ, lane)) { st = HYOBFS_QUIC_ERR_FRAME_EOF; break; }
                if (typ == 0 || typ == 1) continue;
                if (typ != 6) { st = HYOBFS_QUIC_ERR_FRAME_TYPE; break; }
                if (!win.varint(i, fo, lane)) { st = HYOBFS_QUIC_ERR_FRAME_EOF; break; }
                if (!win.varint(i, dl, lane)) { st = HYOBFS_QUIC_ERR_FRAME_EOF; break; }
                if (dl > HYOBFS_QUIC_MAX_CRYPTO_FRAME_LEN) { st = HYOBFS_QUIC_ERR_FRAME_TOO_LARGE; break; }
                if (dl > ct_len - i) { st = HYOBFS_QUIC_ERR_FRAME_EOF; break; }
                if (nf < HYOBFS_QUIC_MAX_FRAMES && lane == 0) fr[nf] = Frame{fo, (uint32_t)dl, (uint32_t)i};
                ++nf;
                i += dl;
            }
            if (st == HYOBFS_OK && nf == 0) st = HYOBFS_QUIC_ERR_ASSEMBLE;
            if (st == HYOBFS_OK && nf > HYOBFS_QUIC_MAX_FRAMES) st = HYOBFS_QUIC_ERR_FRAMES;
            __syncthreads();
            uint64_t out_len = 0, first_off = 0;
            if (st == HYOBFS_OK && nf == 1) {
                out_len = fr[0].len;
                order[0] = 0;
            } else if (st == HYOBFS_OK) {
                // assembleCryptoFrames (payload.go:116-148): stable rank sort by offset
                for (uint32_t j = lane; j < nf; j += 64) {
                    const uint64_t oj = fr[j].off;
                    uint32_t rank = 0;
                    for (uint32_t k = 0; k < nf; ++k) rank += fr[k].off < oj || (fr[k].off == oj && k < j);
                    order[rank] = (uint16_t)j;
                }
                __syncthreads();
                bool gap = false;
                for (uint32_t k = 1 + lane; k < nf; k += 64) {
                    const Frame& x = fr[order[k - 1]];
                    gap |= fr[order[k]].off != x.off + x.len;
                }
                const Frame& last = fr[order[nf - 1]];
                if (__ballot(gap) || last.off > HYOBFS_QUIC_MAX_CRYPTO_PAYLOAD_LEN ||
                    last.off + last.len > HYOBFS_QUIC_MAX_CRYPTO_PAYLOAD_LEN)
                    st = HYOBFS_QUIC_ERR_ASSEMBLE;
                else
                    out_len = last.off + last.len;
                first_off = fr[order[0]].off;
            }
            if (st == HYOBFS_OK) {
                r.out_len = (uint32_t)out_len;
                if (out_len > a.out_cap[pk]) {
                    st = HYOBFS_QUIC_ERR_OUT_CAP;
                } else {
                    uint8_t* o = a.out + a.out_off[pk];
                    for (uint64_t q = lane; q < (nf > 1 ? first_off : 0); q += 64) o[q] = 0;
                    for (uint32_t k = 0; k < nf; ++k) {
                        const Frame x = fr[order[k]];
                        uint8_t* d = o + (nf > 1 ? x.off : 0);
                        const uint8_t* s = ct + x.pos;
                        for (uint32_t q = lane; q < x.len; q += 64) d[q] = s[q];
                    }
                }
            }
            __syncthreads();   // fr / order are reused by the next packet
        }
        if (lane == 0) {
            r.status = st;
            a.res[pk] = r;
        }
    }
}

inline uint32_t grid_for(uint64_t n, uint64_t per) {
    const uint64_t g = (n + per - 1) / per;
    return (uint32_t)(g < (1u << 20) ? g : (1u << 20));
}

}  // namespace quic
}  // namespace hyobfs

// ------------------------------------------------------------------ C ABI
using namespace hyobfs::quic;

namespace {

// host HMAC / HKDF over byte strings (key <= 64 bytes)
void hmac_host(const uint8_t* key, size_t kl, const uint8_t* msg, size_t ml, uint8_t out[32]) {
    uint32_t kw[16];
    key_words(key, kl, kw);
    HmacKey k;
    hmac_key(k, kw);
    uint32_t st[8];
    for (int i = 0; i < 8; ++i) st[i] = k.in[i];
    std::vector<uint8_t> m(msg, msg + ml);
    m.push_back(0x80);
    while (m.size() % 64 != 56) m.push_back(0);
    const uint64_t bits = (64 + ml) * 8;
    for (int i = 7; i >= 0; --i) m.push_back((uint8_t)(bits >> (8 * i)));
    for (size_t b = 0; b < m.size(); b += 64) {
        uint32_t w[16];
        for (int j = 0; j < 16; ++j)
            w[j] = (uint32_t)m[b + 4 * j] << 24 | (uint32_t)m[b + 4 * j + 1] << 16 | (uint32_t)m[b + 4 * j + 2] << 8 |
                   m[b + 4 * j + 3];
        sha256_compress(st, w);
    }
    uint32_t mac[8];
    hmac_finish(k, st, mac);
    words_to_bytes(mac, out, 32);
}

int expand_label(const uint8_t* secret, size_t sl, const char* label, const uint8_t* ctx, size_t cl, uint8_t* out,
                 size_t L) {
    const size_t ll = std::strlen(label);
    if (sl > 64 || 6 + ll > 255 || cl > 255 || L > 255 * 32 || (L && !out)) return HYOBFS_ERR_INVALID;
    std::vector<uint8_t> info;
    info.push_back((uint8_t)(L >> 8));
    info.push_back((uint8_t)L);
    info.push_back((uint8_t)(6 + ll));
    info.insert(info.end(), {'t', 'l', 's', '1', '3', ' '});
    info.insert(info.end(), label, label + ll);
    info.push_back((uint8_t)cl);
    if (cl) info.insert(info.end(), ctx, ctx + cl);
    uint8_t t[32];
    size_t done = 0;
    std::vector<uint8_t> msg;
    for (uint32_t i = 1; done < L; ++i) {
        if (i == 1) msg.clear();   // T(0) is empty, T(i) = HMAC(T(i-1) || info || i)
        else msg.assign(t, t + 32);
        msg.insert(msg.end(), info.begin(), info.end());
        msg.push_back((uint8_t)i);
        hmac_host(secret, sl, msg.data(), msg.size(), t);
        const size_t k = L - done < 32 ? L - done : 32;
        std::memcpy(out + done, t, k);
        done += k;
    }
    return HYOBFS_OK;
}

}  // namespace

extern "C" {

int hyobfs_quic_parse_initial_header(const uint8_t* data, size_t len, hyobfs_quic_header* out) {
    if (!out || (len && !data)) return HYOBFS_ERR_INVALID;
    const Hdr h = parse_initial_header(data, len);
    std::memset(out, 0, sizeof(*out));
    if (h.status != HYOBFS_OK) return h.status;
    out->type = h.type;
    out->dcid_len = h.dl;
    out->scid_len = h.sl;
    out->version = h.version;
    out->dcid_off = h.dcid_off;
    out->scid_off = h.scid_off;
    out->token_off = h.token_off;
    out->token_len = h.token_len;
    out->length = h.length;
    out->offset = h.offset;
    return HYOBFS_OK;
}

int hyobfs_quic_hkdf_expand_label(const uint8_t* secret, size_t secret_len, const char* label,
                                  const uint8_t* context, size_t context_len, uint8_t* out, size_t length) {
    if (!secret || !label || (context_len && !context)) return HYOBFS_ERR_INVALID;
    return expand_label(secret, secret_len, label, context, context_len, out, length);
}

int hyobfs_quic_initial_secret(const uint8_t* dcid, size_t dcid_len, uint32_t version, int server,
                               uint8_t out[32]) {
    if (!out || (dcid_len && !dcid)) return HYOBFS_ERR_INVALID;
    uint8_t prk[32];
    hmac_host(get_salt(version), 20, dcid, dcid_len, prk);   // HKDF-Extract(salt, dcid)
    return expand_label(prk, 32, server ? "server in" : "client in", nullptr, 0, out, 32);
}

int hyobfs_quic_new_protection_key(uint16_t suite, const uint8_t* secret, size_t secret_len, uint32_t version,
                                   hyobfs_quic_key* out) {
    if (!secret || !out) return HYOBFS_ERR_INVALID;
    size_t kl;
    if (suite == HYOBFS_QUIC_TLS_AES_128_GCM_SHA256) kl = 16;
    else if (suite == HYOBFS_QUIC_TLS_CHACHA20_POLY1305_SHA256) kl = 32;
    else return HYOBFS_QUIC_ERR_SUITE;
    const bool v2 = version == HYOBFS_QUIC_V2;   // quic.go:38-59
    std::memset(out, 0, sizeof(*out));
    out->suite = suite;
    int rc = expand_label(secret, secret_len, v2 ? "quicv2 key" : "quic key", nullptr, 0, out->key, kl);
    if (rc == HYOBFS_OK) rc = expand_label(secret, secret_len, v2 ? "quicv2 iv" : "quic iv", nullptr, 0, out->iv, 12);
    if (rc == HYOBFS_OK) rc = expand_label(secret, secret_len, v2 ? "quicv2 hp" : "quic hp", nullptr, 0, out->hp, kl);
    return rc;
}

int hyobfs_quic_unprotect_batch(uint8_t* packets, const uint64_t* off, const uint32_t* len, uint64_t n,
                                const hyobfs_quic_key* keys, uint32_t key_stride, const int64_t* pn_offset,
                                const int64_t* pn_max, hyobfs_quic_result* res, void* stream) {
    if (n == 0) return HYOBFS_OK;
    if (!packets || !off || !len || !keys || !pn_offset || !res || key_stride > 1) return HYOBFS_ERR_INVALID;
    OpenArgs a{packets, off, len, n, keys, key_stride, pn_offset, pn_max, nullptr, res, nullptr, nullptr, nullptr};
    hipLaunchKernelGGL(quic_open_kernel<false>, dim3(grid_for(n, 1)), dim3(64), 0, static_cast<hipStream_t>(stream), a);
    return hipGetLastError() == hipSuccess ? HYOBFS_OK : HYOBFS_ERR_HIP;
}

uint64_t hyobfs_quic_workspace_size(uint64_t n) { return n * sizeof(Job); }

int hyobfs_quic_read_crypto_payload_batch(uint8_t* packets, const uint64_t* off, const uint32_t* len, uint64_t n,
                                          uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                          hyobfs_quic_result* res, void* workspace, void* stream) {
    if (n == 0) return HYOBFS_OK;
    if (!packets || !off || !len || !out || !out_off || !out_cap || !res || !workspace) return HYOBFS_ERR_INVALID;
    static const PrepConsts consts = make_prep_consts();
    Job* jobs = static_cast<Job*>(workspace);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(quic_prep_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, packets, off, len, n,
                       jobs, consts);
    if (hipGetLastError() != hipSuccess) return HYOBFS_ERR_HIP;
    OpenArgs a{packets, off, len, n, nullptr, 0, nullptr, nullptr, jobs, res, out, out_off, out_cap};
    hipLaunchKernelGGL(quic_open_kernel<true>, dim3(grid_for(n, 1)), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? HYOBFS_OK : HYOBFS_ERR_HIP;
}

}  // extern "C"
