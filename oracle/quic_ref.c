/*
 * quic_ref.c -- C restatement of the QUIC Initial sniff path, TEST
 * INFRASTRUCTURE ONLY: the CPU baseline of scripts/bench_quic.py and a second
 * checker in tests/test_quic.py.  Never linked into the product.
 *
 * Follows (apernet/hysteria extras/sniff/internal/quic):
 *   ReadCryptoPayload       payload.go:21-60
 *   ParseInitialHeader      header.go:24-89
 *   UnProtect               packet_protector.go:46-79 (AES-128-GCM, Initial keys)
 *   decodePacketNumber      packet_protector.go:161-174
 *   hkdfExpandLabel         packet_protector.go:177-193
 *   extractCryptoFrames     payload.go:73-112
 *   assembleCryptoFrames    payload.go:116-148
 * Ciphers from FIPS 197 (AES, T-tables), SP 800-38D (GCM, 4-bit Shoup tables),
 * FIPS 180-4 / RFC 2104 / RFC 5869 (SHA-256, HMAC, HKDF).  Status codes are
 * include/hyobfs_quic.h's.  Pinned like oracle/quic_ref.py (tests/test_quic.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum {
    Q_OK = 0, Q_EOF = -40, Q_NOT_QUIC = -41, Q_VERSION = -42, Q_INVALID = -43, Q_SHORT = -44,
    Q_TOO_SMALL = -45, Q_AUTH = -46, Q_FRAME_TYPE = -47, Q_FRAME_EOF = -48, Q_FRAME_TOO_LARGE = -49,
    Q_ASSEMBLE = -50, Q_OUT_CAP = -51
};
#define V1 0x00000001u
#define V2 0x6b3343cfu
#define MAX_CRYPTO (256u * 1024u)

/* ------------------------------------------------------------ SHA-256 / HMAC / HKDF */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void sha256_block(uint32_t st[8], const uint8_t b[64]) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 | (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
    for (int i = 16; i < 64; ++i)
        w[i] = w[i - 16] + (rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
               (rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10));
    uint32_t a = st[0], bb = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & bb) ^ (a & c) ^ (bb & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
    }
    st[0] += a; st[1] += bb; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* SHA-256 of prefix (one 64-byte block, may be NULL) || msg */
static void sha256_2(const uint8_t* prefix, const uint8_t* msg, size_t n, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint64_t total = n + (prefix ? 64 : 0);
    if (prefix) sha256_block(st, prefix);
    size_t i = 0;
    for (; i + 64 <= n; i += 64) sha256_block(st, msg + i);
    uint8_t tail[128] = {0};
    size_t r = n - i;
    memcpy(tail, msg + i, r);
    tail[r] = 0x80;
    size_t tl = r + 9 <= 64 ? 64 : 128;
    for (int k = 0; k < 8; ++k) tail[tl - 1 - k] = (uint8_t)((total * 8) >> (8 * k));
    sha256_block(st, tail);
    if (tl == 128) sha256_block(st, tail + 64);
    for (int k = 0; k < 8; ++k) {
        out[4 * k] = (uint8_t)(st[k] >> 24); out[4 * k + 1] = (uint8_t)(st[k] >> 16);
        out[4 * k + 2] = (uint8_t)(st[k] >> 8); out[4 * k + 3] = (uint8_t)st[k];
    }
}

static void hmac(const uint8_t* key, size_t kl, const uint8_t* msg, size_t n, uint8_t out[32]) {
    uint8_t ip[64] = {0}, op[64] = {0}, inner[32];
    memcpy(ip, key, kl);
    memcpy(op, key, kl);
    for (int i = 0; i < 64; ++i) { ip[i] ^= 0x36; op[i] ^= 0x5c; }
    sha256_2(ip, msg, n, inner);
    sha256_2(op, inner, 32, out);
}

/* hkdfExpandLabel with an empty context, length <= 32 (one HMAC) */
static void expand_label(const uint8_t secret[32], const char* label, uint32_t L, uint8_t* out) {
    uint8_t info[64];
    size_t ll = strlen(label), i = 0;
    info[i++] = (uint8_t)(L >> 8);
    info[i++] = (uint8_t)L;
    info[i++] = (uint8_t)(6 + ll);
    memcpy(info + i, "tls13 ", 6);
    i += 6;
    memcpy(info + i, label, ll);
    i += ll;
    info[i++] = 0;
    info[i++] = 1;
    uint8_t t[32];
    hmac(secret, 32, info, i, t);
    memcpy(out, t, L);
}

/* ------------------------------------------------------------ AES-128 */
static uint8_t SB[256];
static uint32_t TE[4][256];

static void aes_init(void) {
    uint8_t p = 1, q = 1;
    do {
        p = (uint8_t)(p ^ (p << 1) ^ (p & 0x80 ? 0x1b : 0));
        q ^= (uint8_t)(q << 1);
        q ^= (uint8_t)(q << 2);
        q ^= (uint8_t)(q << 4);
        if (q & 0x80) q ^= 0x09;
        uint8_t x = q ^ (uint8_t)((q << 1) | (q >> 7)) ^ (uint8_t)((q << 2) | (q >> 6)) ^
                    (uint8_t)((q << 3) | (q >> 5)) ^ (uint8_t)((q << 4) | (q >> 4));
        SB[p] = x ^ 0x63;
    } while (p != 1);
    SB[0] = 0x63;
    for (int x = 0; x < 256; ++x) {
        uint32_t s = SB[x], s2 = ((s << 1) ^ (s & 0x80 ? 0x1b : 0)) & 0xff, s3 = s2 ^ s;
        uint32_t t = s2 | s << 8 | s << 16 | s3 << 24;   /* little-endian column word */
        for (int r = 0; r < 4; ++r) TE[r][x] = r ? (t << (8 * r)) | (t >> (32 - 8 * r)) : t;
    }
}

static uint32_t le32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

static void aes_expand(const uint8_t key[16], uint32_t rk[44]) {
    for (int i = 0; i < 4; ++i) rk[i] = le32(key + 4 * i);
    uint32_t rcon = 1;
    for (int i = 4; i < 44; ++i) {
        uint32_t t = rk[i - 1];
        if (i % 4 == 0) {
            t = (t >> 8) | (t << 24);
            t = (uint32_t)SB[t & 0xff] | (uint32_t)SB[(t >> 8) & 0xff] << 8 | (uint32_t)SB[(t >> 16) & 0xff] << 16 |
                (uint32_t)SB[t >> 24] << 24;
            t ^= rcon;
            rcon = ((rcon << 1) ^ (rcon & 0x80 ? 0x1b : 0)) & 0xff;
        }
        rk[i] = rk[i - 4] ^ t;
    }
}

static void aes_encrypt(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]) {
    uint32_t s0 = le32(in) ^ rk[0], s1 = le32(in + 4) ^ rk[1], s2 = le32(in + 8) ^ rk[2], s3 = le32(in + 12) ^ rk[3];
    for (int r = 1; r < 10; ++r) {
        uint32_t t0 = TE[0][s0 & 0xff] ^ TE[1][(s1 >> 8) & 0xff] ^ TE[2][(s2 >> 16) & 0xff] ^ TE[3][s3 >> 24] ^ rk[4 * r];
        uint32_t t1 = TE[0][s1 & 0xff] ^ TE[1][(s2 >> 8) & 0xff] ^ TE[2][(s3 >> 16) & 0xff] ^ TE[3][s0 >> 24] ^ rk[4 * r + 1];
        uint32_t t2 = TE[0][s2 & 0xff] ^ TE[1][(s3 >> 8) & 0xff] ^ TE[2][(s0 >> 16) & 0xff] ^ TE[3][s1 >> 24] ^ rk[4 * r + 2];
        uint32_t t3 = TE[0][s3 & 0xff] ^ TE[1][(s0 >> 8) & 0xff] ^ TE[2][(s1 >> 16) & 0xff] ^ TE[3][s2 >> 24] ^ rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    uint32_t o[4] = {
        ((uint32_t)SB[s0 & 0xff] | (uint32_t)SB[(s1 >> 8) & 0xff] << 8 | (uint32_t)SB[(s2 >> 16) & 0xff] << 16 | (uint32_t)SB[s3 >> 24] << 24) ^ rk[40],
        ((uint32_t)SB[s1 & 0xff] | (uint32_t)SB[(s2 >> 8) & 0xff] << 8 | (uint32_t)SB[(s3 >> 16) & 0xff] << 16 | (uint32_t)SB[s0 >> 24] << 24) ^ rk[41],
        ((uint32_t)SB[s2 & 0xff] | (uint32_t)SB[(s3 >> 8) & 0xff] << 8 | (uint32_t)SB[(s0 >> 16) & 0xff] << 16 | (uint32_t)SB[s1 >> 24] << 24) ^ rk[42],
        ((uint32_t)SB[s3 & 0xff] | (uint32_t)SB[(s0 >> 8) & 0xff] << 8 | (uint32_t)SB[(s1 >> 16) & 0xff] << 16 | (uint32_t)SB[s2 >> 24] << 24) ^ rk[43]};
    for (int k = 0; k < 4; ++k)
        for (int b = 0; b < 4; ++b) out[4 * k + b] = (uint8_t)(o[k] >> (8 * b));
}

/* ------------------------------------------------------------ GHASH (4-bit Shoup tables) */
typedef struct { uint64_t h, l; } g128;

static g128 ld128(const uint8_t* p) {
    g128 r = {0, 0};
    for (int i = 0; i < 8; ++i) { r.h = r.h << 8 | p[i]; r.l = r.l << 8 | p[8 + i]; }
    return r;
}
static g128 mulx(g128 v) {
    uint64_t lsb = 0 - (v.l & 1);
    g128 r = {(v.h >> 1) ^ (lsb & 0xE100000000000000ull), (v.l >> 1) | (v.h << 63)};
    return r;
}
static void ghash_table(g128 H, g128 T[16]) {
    g128 p[4];
    p[0] = H; p[1] = mulx(p[0]); p[2] = mulx(p[1]); p[3] = mulx(p[2]);
    for (int i = 0; i < 16; ++i) {
        g128 e = {0, 0};
        for (int b = 0; b < 4; ++b)
            if (i & (8 >> b)) { e.h ^= p[b].h; e.l ^= p[b].l; }
        T[i] = e;
    }
}
static g128 ghash_mul(g128 x, const g128 T[16]) {
    g128 z = {0, 0};
    for (int j = 31; j >= 0; --j) {
        if (j != 31) {
            uint32_t rem = (uint32_t)z.l & 0xf;
            uint32_t red = (rem & 1) * 0x1C20u ^ (rem & 2) * 0x1C20u ^ (rem & 4) * 0x1C20u ^ (rem & 8) * 0x1C20u;
            z.l = (z.l >> 4) | (z.h << 60);
            z.h = (z.h >> 4) ^ ((uint64_t)red << 48);
        }
        uint32_t nib = j >= 16 ? (uint32_t)(x.l >> (4 * (31 - j))) & 0xf : (uint32_t)(x.h >> (4 * (15 - j))) & 0xf;
        z.h ^= T[nib].h;
        z.l ^= T[nib].l;
    }
    return z;
}
static void ghash_update(g128* y, const g128 T[16], const uint8_t* d, size_t n) {
    for (size_t i = 0; i < n; i += 16) {
        uint8_t b[16] = {0};
        memcpy(b, d + i, n - i < 16 ? n - i : 16);
        g128 x = ld128(b);
        y->h ^= x.h;
        y->l ^= x.l;
        *y = ghash_mul(*y, T);
    }
}

/* AES-128-GCM open in place: verify, then decrypt (cipher.GCM Open) */
static int gcm_open(const uint32_t rk[44], const uint8_t nonce[12], uint8_t* ct, size_t n, const uint8_t tag[16],
                    const uint8_t* aad, size_t an) {
    uint8_t zero[16] = {0}, hb[16], j0[16], ej[16];
    aes_encrypt(rk, zero, hb);
    g128 T[16];
    ghash_table(ld128(hb), T);
    g128 y = {0, 0};
    ghash_update(&y, T, aad, an);
    ghash_update(&y, T, ct, n);
    uint8_t lb[16];
    for (int k = 0; k < 8; ++k) { lb[7 - k] = (uint8_t)((an * 8) >> (8 * k)); lb[15 - k] = (uint8_t)((n * 8) >> (8 * k)); }
    ghash_update(&y, T, lb, 16);
    memcpy(j0, nonce, 12);
    j0[12] = j0[13] = j0[14] = 0;
    j0[15] = 1;
    aes_encrypt(rk, j0, ej);
    g128 e = ld128(ej);
    g128 t = ld128(tag);
    if (((y.h ^ e.h) != t.h) | ((y.l ^ e.l) != t.l)) return Q_AUTH;
    for (size_t i = 0; i < n; i += 16) {
        uint8_t cb[16], ks[16];
        uint32_t ctr = 2 + (uint32_t)(i / 16);
        memcpy(cb, nonce, 12);
        cb[12] = (uint8_t)(ctr >> 24); cb[13] = (uint8_t)(ctr >> 16); cb[14] = (uint8_t)(ctr >> 8); cb[15] = (uint8_t)ctr;
        aes_encrypt(rk, cb, ks);
        for (size_t k = 0; k < 16 && i + k < n; ++k) ct[i + k] ^= ks[k];
    }
    return Q_OK;
}

/* ------------------------------------------------------------ header, frames */
static int varint(const uint8_t* p, uint64_t n, uint64_t* i, uint64_t* v) {
    if (*i >= n) return 0;
    uint32_t k = 1u << (p[*i] >> 6);
    if (n - *i < k) return 0;
    uint64_t x = p[*i] & 0x3f;
    for (uint32_t j = 1; j < k; ++j) x = x << 8 | p[*i + j];
    *v = x;
    *i += k;
    return 1;
}

typedef struct { uint64_t off; uint32_t len, pos, idx; } frame_t;

static int frame_cmp(const void* a, const void* b) {   /* by offset, then packet order (stable) */
    const frame_t *x = a, *y = b;
    if (x->off != y->off) return x->off < y->off ? -1 : 1;
    return x->idx < y->idx ? -1 : x->idx > y->idx;
}

/* ReadCryptoPayload on a private copy of the packet (scratch: len bytes). */
int quic_read_crypto_payload(const uint8_t* pkt, uint32_t len, uint8_t* scratch, uint8_t* out, uint32_t cap,
                             uint32_t* out_len) {
    static const uint8_t salt_v1[20] = {0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17,
                                        0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad, 0xcc, 0xbb, 0x7f, 0x0a};
    static const uint8_t salt_v2[20] = {0x0d, 0xed, 0xe3, 0xde, 0xf7, 0x00, 0xa6, 0xdb, 0x81, 0x93,
                                        0x81, 0xbe, 0x6e, 0x26, 0x9d, 0xcb, 0xf9, 0xbd, 0x2e, 0xd9};
    *out_len = 0;
    /* ParseInitialHeader */
    if (len < 5) return Q_EOF;
    uint8_t type = pkt[0];
    uint32_t ver = (uint32_t)pkt[1] << 24 | (uint32_t)pkt[2] << 16 | (uint32_t)pkt[3] << 8 | pkt[4];
    if (ver != 0 && !(type & 0x40)) return Q_NOT_QUIC;
    uint64_t i = 5, v;
    if (i >= len) return Q_EOF;
    uint32_t dl = pkt[i++];
    if (len - i < dl) return Q_EOF;
    const uint8_t* dcid = pkt + i;
    i += dl;
    if (i >= len) return Q_EOF;
    uint32_t sl = pkt[i++];
    if (len - i < sl) return Q_EOF;
    i += sl;
    if (((type >> 4) & 3u) == (ver == V2 ? 1u : 0u)) {
        if (!varint(pkt, len, &i, &v) || v > len - i) return Q_EOF;
        i += v;
    }
    uint64_t length;
    if (!varint(pkt, len, &i, &length)) return Q_EOF;
    uint64_t offset = i;
    if (ver != V1 && ver != V2) return Q_VERSION;
    if (offset == 0 || length == 0) return Q_INVALID;
    if ((uint64_t)len - offset < length) return Q_SHORT;
    uint32_t L = (uint32_t)(offset + length);
    /* client Initial keys */
    uint8_t prk[32], secret[32], key[16], iv[12], hp[16];
    hmac(ver == V2 ? salt_v2 : salt_v1, 20, dcid, dl, prk);
    expand_label(prk, "client in", 32, secret);
    expand_label(secret, ver == V2 ? "quicv2 key" : "quic key", 16, key);
    expand_label(secret, ver == V2 ? "quicv2 iv" : "quic iv", 12, iv);
    expand_label(secret, ver == V2 ? "quicv2 hp" : "quic hp", 16, hp);
    /* UnProtect(packet[:offset+Length], offset, 2) */
    if (L - offset < 20) return Q_TOO_SMALL;
    memcpy(scratch, pkt, L);
    uint32_t hrk[44], rk[44];
    uint8_t mask[16];
    aes_expand(hp, hrk);
    aes_encrypt(hrk, scratch + offset + 4, mask);
    scratch[0] ^= mask[0] & ((scratch[0] & 0x80) ? 0x0f : 0x1f);
    uint32_t pn_len = (scratch[0] & 3) + 1;
    int64_t trunc = 0;
    for (uint32_t k = 0; k < pn_len; ++k) {
        scratch[offset + k] ^= mask[1 + k];
        trunc = trunc << 8 | scratch[offset + k];
    }
    int64_t expected = 3, win = (int64_t)1 << (pn_len * 8), hwin = win / 2;
    int64_t cand = (expected & ~(win - 1)) | trunc, pn = cand;
    if (cand <= expected - hwin && cand < ((int64_t)1 << 62) - win) pn = cand + win;
    else if (cand > expected + hwin && cand >= win) pn = cand - win;
    uint32_t hdr = (uint32_t)offset + pn_len;
    if (L - hdr < 16) return Q_AUTH;
    uint8_t nonce[12];
    memcpy(nonce, iv, 12);
    for (int k = 0; k < 8; ++k) nonce[4 + k] ^= (uint8_t)((uint64_t)pn >> (56 - 8 * k));
    aes_expand(key, rk);
    uint32_t n = L - hdr - 16;
    uint8_t* pl = scratch + hdr;
    if (gcm_open(rk, nonce, pl, n, pl + n, scratch, hdr) != Q_OK) return Q_AUTH;
    /* extractCryptoFrames */
    frame_t fr_stack[64];
    frame_t* fr = fr_stack;
    uint32_t nf = 0, capf = 64;
    uint64_t j = 0, typ, fo, fl;
    int st = Q_OK;
    while (j < n) {
        if (!varint(pl, n, &j, &typ)) { st = Q_FRAME_EOF; break; }
        if (typ == 0 || typ == 1) continue;
        if (typ != 6) { st = Q_FRAME_TYPE; break; }
        if (!varint(pl, n, &j, &fo) || !varint(pl, n, &j, &fl)) { st = Q_FRAME_EOF; break; }
        if (fl > MAX_CRYPTO) { st = Q_FRAME_TOO_LARGE; break; }
        if (fl > n - j) { st = Q_FRAME_EOF; break; }
        if (nf == capf) {
            frame_t* g = malloc(sizeof(frame_t) * capf * 2);
            memcpy(g, fr, sizeof(frame_t) * nf);
            if (fr != fr_stack) free(fr);
            fr = g;
            capf *= 2;
        }
        fr[nf] = (frame_t){fo, (uint32_t)fl, (uint32_t)j, nf};
        ++nf;
        j += fl;
    }
    uint64_t outn = 0;
    if (st == Q_OK && nf == 0) st = Q_ASSEMBLE;
    if (st == Q_OK && nf == 1) {
        outn = fr[0].len;
    } else if (st == Q_OK) {   /* assembleCryptoFrames */
        qsort(fr, nf, sizeof(frame_t), frame_cmp);
        for (uint32_t k = 1; k < nf && st == Q_OK; ++k)
            if (fr[k].off != fr[k - 1].off + fr[k - 1].len) st = Q_ASSEMBLE;
        if (st == Q_OK && (fr[nf - 1].off > MAX_CRYPTO || fr[nf - 1].off + fr[nf - 1].len > MAX_CRYPTO))
            st = Q_ASSEMBLE;
        if (st == Q_OK) outn = fr[nf - 1].off + fr[nf - 1].len;
    }
    if (st == Q_OK) {
        *out_len = (uint32_t)outn;
        if (outn > cap) {
            st = Q_OUT_CAP;
        } else if (nf == 1) {
            memcpy(out, pl + fr[0].pos, fr[0].len);
        } else {
            memset(out, 0, fr[0].off);
            for (uint32_t k = 0; k < nf; ++k) memcpy(out + fr[k].off, pl + fr[k].pos, fr[k].len);
        }
    }
    if (fr != fr_stack) free(fr);
    return st;
}

/* ------------------------------------------------------------ batches on host threads */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

typedef struct {
    const uint8_t* pkts; const uint64_t* off; const uint32_t* len; uint64_t a, b;
    uint8_t* out; uint32_t cap; int32_t* status; uint32_t* out_len;
} job_t;

static void* worker(void* arg) {
    job_t* j = arg;
    uint8_t* scratch = malloc(1 << 17);
    for (uint64_t i = j->a; i < j->b; ++i) {
        uint32_t L = j->len[i];
        if (L > (1u << 17)) { j->status[i] = Q_SHORT; continue; }
        j->status[i] = quic_read_crypto_payload(j->pkts + j->off[i], L, scratch, j->out + i * (uint64_t)j->cap, j->cap,
                                                &j->out_len[i]);
    }
    free(scratch);
    return NULL;
}

void quic_ref_init(void) { pthread_once(&g_once, aes_init); }

int quic_read_crypto_payload_batch(const uint8_t* pkts, const uint64_t* off, const uint32_t* len, uint64_t n,
                                   uint8_t* out, uint32_t cap, int32_t* status, uint32_t* out_len, int nthreads) {
    quic_ref_init();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (job_t){pkts, off, len, n * t / nthreads, n * (t + 1) / nthreads, out, cap, status, out_len};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}
