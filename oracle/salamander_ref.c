/*
 * oracle/salamander_ref.c -- CPU restatement of Hysteria's "Salamander"
 * per-datagram obfuscation.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle and the CPU
 * baseline.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker.  The product path
 * (hysteria_amd/csrc, libhyobfs.so) never links or calls it.
 *
 * What it restates (all paths relative to the apernet/hysteria reference):
 *   - extras/obfs/salamander.go:13-17   constants: PSK >= 4, salt 8, key 32
 *   - extras/obfs/salamander.go:34-46   newSalamanderObfuscator (PSK check)
 *   - extras/obfs/salamander.go:59-72   Obfuscate: out = salt || in ^ key[i%32]
 *   - extras/obfs/salamander.go:74-86   Deobfuscate: reject len(in) <= 8
 *   - extras/obfs/salamander.go:88-91   keyLocked: BLAKE2b-256(PSK || salt)
 *   - PROTOCOL.md:129-153               normative packet format
 *   - golang.org/x/crypto@v0.54.0/blake2b.Sum256 (extras/go.mod:18; not in the
 *     reference tree): RFC 7693 BLAKE2b, unkeyed, digest length 32.  This file
 *     restates RFC 7693 section 3 from the published algorithm.
 *
 * Parity pinning: the reference's own tests hold no known-answer vector
 * (extras/obfs/salamander_test.go:32-45 checks round-trip identity only), and
 * no Go toolchain exists on either machine.  The BLAKE2b here is pinned to
 * RFC 7693 Appendix A and to two independent implementations (CPython
 * hashlib.blake2b, coreutils b2sum) through tests/golden/, see DESIGN.md.
 *
 * The batch entry points define the batch semantics of include/hyobfs.h
 * (per-packet rules exactly as salamander.go; layout rules documented there).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>
#include <stdlib.h>

#define SM_PSK_MIN_LEN 4   /* salamander.go:14 */
#define SM_SALT_LEN 8      /* salamander.go:15 */
#define SM_KEY_LEN 32      /* salamander.go:16 (blake2b.Size256) */

/* ---------------------------------------------------------------- BLAKE2b */

static const uint64_t B2B_IV[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
    0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
    0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

static const uint8_t B2B_SIGMA[12][16] = {
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

static inline uint64_t rotr64(uint64_t x, unsigned n) {
    return (x >> n) | (x << (64 - n));
}

static inline uint64_t load64_le(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

/* RFC 7693 section 3.2, function F. */
static void b2b_compress(uint64_t h[8], const uint8_t block[128], uint64_t t,
                         int last) {
    uint64_t m[16], v[16];
    for (int i = 0; i < 16; ++i) m[i] = load64_le(block + 8 * i);
    for (int i = 0; i < 8; ++i) {
        v[i] = h[i];
        v[i + 8] = B2B_IV[i];
    }
    v[12] ^= t; /* low word of the 128-bit counter; messages here are < 2^64 */
    if (last) v[14] = ~v[14];
#define B2B_G(a, b, c, d, x, y)          \
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
    for (int r = 0; r < 12; ++r) {
        const uint8_t* s = B2B_SIGMA[r];
        B2B_G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        B2B_G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        B2B_G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        B2B_G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        B2B_G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        B2B_G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        B2B_G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        B2B_G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef B2B_G
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

/* Unkeyed BLAKE2b with digest length outlen (1..64), RFC 7693 section 3.3. */
void oracle_blake2b(uint8_t* out, size_t outlen, const uint8_t* in,
                    size_t inlen) {
    uint64_t h[8];
    uint8_t block[128];
    for (int i = 0; i < 8; ++i) h[i] = B2B_IV[i];
    h[0] ^= 0x01010000ULL ^ (uint64_t)outlen; /* kk = 0 */
    size_t done = 0;
    /* all but the last block: full, non-final */
    while (inlen - done > 128) {
        b2b_compress(h, in + done, (uint64_t)(done + 128), 0);
        done += 128;
    }
    memset(block, 0, sizeof block);
    if (inlen - done) memcpy(block, in + done, inlen - done);
    b2b_compress(h, block, (uint64_t)inlen, 1);
    for (size_t i = 0; i < outlen; ++i) out[i] = (uint8_t)(h[i / 8] >> (8 * (i % 8)));
}

/* ------------------------------------------------------------- Salamander */

/* newSalamanderObfuscator (salamander.go:34-37): 0 = ok, -1 = ErrPSKTooShort */
int oracle_salamander_check_psk(size_t psk_len) {
    return psk_len < SM_PSK_MIN_LEN ? -1 : 0;
}

/* keyLocked (salamander.go:88-91): BLAKE2b-256(PSK || salt[0:8]) */
void oracle_salamander_key(const uint8_t* psk, size_t psk_len,
                           const uint8_t salt[8], uint8_t key[32]) {
    uint8_t buf[4096 + 8];
    uint8_t* ki = buf;
    uint8_t* heap = NULL;
    if (psk_len > 4096) { /* stack buffer covers every realistic PSK */
        heap = (uint8_t*)malloc(psk_len + 8);
        if (!heap) abort();
        ki = heap;
    }
    memcpy(ki, psk, psk_len);
    memcpy(ki + psk_len, salt, SM_SALT_LEN);
    oracle_blake2b(key, SM_KEY_LEN, ki, psk_len + SM_SALT_LEN);
    free(heap);
}

/* Obfuscate (salamander.go:59-72).  The salt that the reference draws from
   RandSrc (math/rand, :65) is an explicit argument here.  Returns the bytes
   written to out, 0 if out is too small. */
size_t oracle_salamander_obfuscate(const uint8_t* psk, size_t psk_len,
                                   const uint8_t* in, size_t in_len,
                                   const uint8_t salt[8], uint8_t* out,
                                   size_t out_len) {
    size_t n = in_len + SM_SALT_LEN;
    if (out_len < n) return 0;
    uint8_t key[SM_KEY_LEN];
    memcpy(out, salt, SM_SALT_LEN);
    oracle_salamander_key(psk, psk_len, out, key);
    for (size_t i = 0; i < in_len; ++i)
        out[i + SM_SALT_LEN] = in[i] ^ key[i % SM_KEY_LEN];
    return n;
}

/* Deobfuscate (salamander.go:74-86).  Returns len(in)-8, or 0 when
   len(in) <= 8 or out is too small.  out may alias in + 0 (writes trail
   reads by 8 bytes), as in the reference. */
size_t oracle_salamander_deobfuscate(const uint8_t* psk, size_t psk_len,
                                     const uint8_t* in, size_t in_len,
                                     uint8_t* out, size_t out_len) {
    if (in_len <= SM_SALT_LEN) return 0;
    size_t n = in_len - SM_SALT_LEN;
    if (out_len < n) return 0;
    uint8_t key[SM_KEY_LEN];
    oracle_salamander_key(psk, psk_len, in, key);
    for (size_t i = 0; i < n; ++i) out[i] = in[SM_SALT_LEN + i] ^ key[i % SM_KEY_LEN];
    return n;
}

/* ------------------------------------------------------------------ batch */
/*
 * Batch semantics of include/hyobfs.h, restated on the CPU:
 *   packet i:  L = in_len ? in_len[i] : len_uniform
 *              in bytes at in + (in_off ? in_off[i] : i * in_stride)
 *   obfuscate: W = L + 8                    valid iff W <= cap_i
 *   deobf.   : W = L - 8                    valid iff W > 0 && W <= cap_i
 *   cap_i    : pkt_cap (0 = unlimited), further limited to out_stride when
 *              the output is slotted (out_stride > 0)
 *   out_off_i: slotted -> i * out_stride
 *              packed  -> exclusive prefix sum of the valid W's
 *   a packet whose region [out_off_i, out_off_i + W) would pass out_cap is
 *   dropped (its W still counts in the prefix sum, so every later packet is
 *   dropped too); a dropped packet writes nothing and reports out_len 0.
 * Returns the number of bytes written (sum of out_len).
 */
static uint64_t batch_common(int obf, const uint8_t* psk, size_t psk_len,
                             uint64_t n, const uint8_t* in,
                             const uint64_t* in_off, uint64_t in_stride,
                             const uint32_t* in_len, uint32_t len_uniform,
                             const uint64_t* salts, uint8_t* out,
                             uint64_t out_cap, uint64_t out_stride,
                             uint32_t pkt_cap, uint64_t* out_off,
                             uint32_t* out_len) {
    uint64_t cursor = 0, total = 0;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t L = in_len ? in_len[i] : len_uniform;
        const uint8_t* src = in + (in_off ? in_off[i] : i * in_stride);
        int64_t W = obf ? (int64_t)L + 8 : (int64_t)L - 8;
        uint64_t cap = pkt_cap ? pkt_cap : UINT64_MAX;
        if (out_stride && out_stride < cap) cap = out_stride;
        int valid = W > 0 && (uint64_t)W <= cap;
        if (!obf && W <= 0) valid = 0;
        if (!valid) W = 0;
        uint64_t off = out_stride ? i * out_stride : cursor;
        /* packed offsets are a pure prefix sum of the per-packet rule above;
           the out_cap clip never moves later packets */
        if (!out_stride) cursor += (uint64_t)W;
        if (valid && off + (uint64_t)W > out_cap) {
            valid = 0;
            W = 0;
        }
        if (out_off) out_off[i] = off;
        if (out_len) out_len[i] = (uint32_t)W;
        if (!valid) continue;
        if (obf) {
            uint8_t salt[8];
            for (int b = 0; b < 8; ++b) salt[b] = (uint8_t)(salts[i] >> (8 * b));
            oracle_salamander_obfuscate(psk, psk_len, src, L, salt, out + off,
                                        (size_t)W);
        } else {
            oracle_salamander_deobfuscate(psk, psk_len, src, L, out + off,
                                          (size_t)W);
        }
        total += (uint64_t)W;
    }
    return total;
}

uint64_t oracle_obfuscate_batch(const uint8_t* psk, size_t psk_len, uint64_t n,
                                const uint8_t* in, const uint64_t* in_off,
                                uint64_t in_stride, const uint32_t* in_len,
                                uint32_t len_uniform, const uint64_t* salts,
                                uint8_t* out, uint64_t out_cap,
                                uint64_t out_stride, uint32_t pkt_cap,
                                uint64_t* out_off, uint32_t* out_len) {
    return batch_common(1, psk, psk_len, n, in, in_off, in_stride, in_len,
                        len_uniform, salts, out, out_cap, out_stride, pkt_cap,
                        out_off, out_len);
}

uint64_t oracle_deobfuscate_batch(const uint8_t* psk, size_t psk_len,
                                  uint64_t n, const uint8_t* in,
                                  const uint64_t* in_off, uint64_t in_stride,
                                  const uint32_t* in_len, uint32_t len_uniform,
                                  uint8_t* out, uint64_t out_cap,
                                  uint64_t out_stride, uint32_t pkt_cap,
                                  uint64_t* out_off, uint32_t* out_len) {
    return batch_common(0, psk, psk_len, n, in, in_off, in_stride, in_len,
                        len_uniform, NULL, out, out_cap, out_stride, pkt_cap,
                        out_off, out_len);
}

/* ------------------------------------------------ synthetic inputs (seeded) */
/* SplitMix64 in counter form: output k of the stream seeded with s is
   mix(s + (k + 1) * golden).  BASELINE.md "Synthetic inputs". */
static inline uint64_t sm64_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t k) {
    return sm64_mix(seed + (k + 1) * 0x9e3779b97f4a7c15ULL);
}
/* bytes [start, start+nbytes) of the little-endian byte stream of the
   SplitMix64(seed) outputs */
void oracle_fill_stream(uint64_t seed, uint64_t start, uint64_t nbytes,
                        uint8_t* dst) {
    for (uint64_t b = 0; b < nbytes; ++b) {
        uint64_t g = start + b;
        dst[b] = (uint8_t)(oracle_splitmix64_at(seed, g >> 3) >> (8 * (g & 7)));
    }
}
void oracle_fill_salts(uint64_t seed, uint64_t first, uint64_t n, uint64_t* dst) {
    for (uint64_t i = 0; i < n; ++i) dst[i] = oracle_splitmix64_at(seed, first + i);
}
/* bimodal Internet mix: 40 % 64 B, 60 % 1350 B (BASELINE.json configs[2]) */
void oracle_fill_bimodal_lengths(uint64_t seed, uint64_t first, uint64_t n,
                                 uint32_t* dst) {
    for (uint64_t i = 0; i < n; ++i)
        dst[i] = (oracle_splitmix64_at(seed, first + i) % 5) < 2 ? 64u : 1350u;
}

/* ------------------------------------------------------ CPU baseline timer */
/* The CPU baseline times the reference's own per-packet surface: one call of
   Obfuscate (or Deobfuscate) per datagram into a fresh output, like
   BenchmarkSalamanderObfuscator_* (salamander_test.go:10-30), over the same
   uniform batch layout the GPU bench uses.  nthreads workers split the packet
   range, each with its own obfuscator. */
typedef struct {
    int obf;
    const uint8_t* psk;
    size_t psk_len;
    uint64_t lo, hi;
    const uint8_t* in;
    uint64_t in_stride;
    uint32_t len;
    const uint64_t* salts;
    uint8_t* out;
    uint64_t out_stride;
} cpu_job;

static void* cpu_worker(void* arg) {
    cpu_job* j = (cpu_job*)arg;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        if (j->obf) {
            uint8_t salt[8];
            for (int b = 0; b < 8; ++b) salt[b] = (uint8_t)(j->salts[i] >> (8 * b));
            oracle_salamander_obfuscate(j->psk, j->psk_len, j->in + i * j->in_stride,
                                        j->len, salt, j->out + i * j->out_stride,
                                        j->out_stride);
        } else {
            oracle_salamander_deobfuscate(j->psk, j->psk_len,
                                          j->in + i * j->in_stride, j->len,
                                          j->out + i * j->out_stride, j->out_stride);
        }
    }
    return NULL;
}

int oracle_run_uniform_threads(int obf, const uint8_t* psk, size_t psk_len,
                               uint64_t n, const uint8_t* in, uint64_t in_stride,
                               uint32_t len, const uint64_t* salts, uint8_t* out,
                               uint64_t out_stride, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    cpu_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (cpu_job){obf, psk, psk_len, n * t / nthreads,
                            n * (t + 1) / nthreads, in, in_stride, len, salts,
                            out, out_stride};
        if (nthreads > 1) {
            if (pthread_create(&th[t], NULL, cpu_worker, &jobs[t]) != 0) return -1;
        } else {
            cpu_worker(&jobs[t]);
        }
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}
