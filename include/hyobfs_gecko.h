/*
 * hyobfs_gecko.h -- Gecko framing (extras/obfs/gecko_frame.go, gecko.go) on
 * top of the Salamander context of hyobfs.h.
 *
 * Gecko fragments QUIC long-header packets into 2..8 chunks, each sent as its
 * own Salamander datagram
 *     salt(8) || ( 0x80 | msgID | chunkIdx<<4|total | padLen(BE16) | pad | chunk ) ^ key
 * and padded so the datagram lands in [min_pkt, max_pkt]; short-header packets
 * pass through as plain Salamander datagrams.  The per-byte work -- header,
 * padding, chunk copy and the Salamander XOR -- runs on the GPU in one pass
 * over a batch of frames (hyobfs_gecko_encode_batch); the receive side parses
 * deobfuscated datagrams on the GPU (hyobfs_gecko_parse_batch).  The random
 * choices (chunk counts, pad lengths, msgIDs) and reassembly stay on the host,
 * as in the reference (gecko.go:199-304).
 *
 * Plain C ABI: pointers, sizes, integer status codes.
 */
#ifndef HYOBFS_GECKO_H
#define HYOBFS_GECKO_H

#include <stddef.h>
#include <stdint.h>

#include "hyobfs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* gecko_frame.go:9-15, gecko.go:17-26 */
#define HYOBFS_GECKO_FLAG_FRAGMENT 0x80
#define HYOBFS_GECKO_HEADER_LEN 5
#define HYOBFS_GECKO_MIN_CHUNKS 2
#define HYOBFS_GECKO_MAX_CHUNKS 8
#define HYOBFS_GECKO_BUFFER_SIZE 2048
#define HYOBFS_GECKO_DEFAULT_MIN_PACKET 512
#define HYOBFS_GECKO_DEFAULT_MAX_PACKET 1200
#define HYOBFS_GECKO_REASSEMBLY_TTL_MS 8000
#define HYOBFS_GECKO_MAX_REASSEMBLY 4096
#define HYOBFS_GECKO_MAX_PER_SOURCE 8

/* frame status codes: errFrameTruncated / errFrameInvalid (gecko_frame.go:18-21) */
#define HYOBFS_GECKO_ERR_TRUNCATED (-20)
#define HYOBFS_GECKO_ERR_INVALID (-21)
/* per-datagram parse results (hyobfs_gecko_parsed.status) */
#define HYOBFS_GECKO_PASS 0        /* top bit clear: short header or garbage, passed through (gecko.go:183-185) */
#define HYOBFS_GECKO_FRAGMENT 1    /* a valid fragment frame */
#define HYOBFS_GECKO_EMPTY (-22)   /* zero-length datagram: skipped by ReadFrom (gecko.go:178-180) */

/* frameHeader (gecko_frame.go:30-35) */
typedef struct hyobfs_gecko_header {
    uint16_t pad_len;
    uint8_t msg_id;
    uint8_t chunk_idx;     /* < total_chunks */
    uint8_t total_chunks;  /* [2, 8] */
    uint8_t reserved_[3];
} hyobfs_gecko_header;

/*
 * encodeFrame (gecko_frame.go:39-61), host memory.  Writes header, pad_len
 * random bytes (getrandom, like crypto/rand) and the payload into out.
 * Returns the frame length, HYOBFS_GECKO_ERR_INVALID (chunk count or index
 * out of range) or HYOBFS_GECKO_ERR_TRUNCATED (cap too small).
 */
int64_t hyobfs_gecko_encode_frame(const hyobfs_gecko_header* h, const uint8_t* payload, size_t len,
                                  uint8_t* out, size_t cap);
/*
 * decodeFrame (gecko_frame.go:65-86), host memory.  On success fills *h and
 * *payload_off (the payload is in[*payload_off, len)) and returns HYOBFS_OK;
 * otherwise HYOBFS_GECKO_ERR_TRUNCATED or HYOBFS_GECKO_ERR_INVALID, checked in
 * the reference's order.
 */
int hyobfs_gecko_decode_frame(const uint8_t* in, size_t len, hyobfs_gecko_header* h, size_t* payload_off);
/*
 * randomPadLen (gecko.go:131-138) with the randomness passed in: rnd is a
 * uniform 32-bit value (randIntn's BigEndian.Uint32 of 4 random bytes,
 * gecko.go:145-153).  Padding puts salt + header + pad + chunk in
 * [min_pkt, max_pkt]; 0 when the chunk alone exceeds max_pkt.
 */
uint32_t hyobfs_gecko_pad_len(int min_pkt, int max_pkt, uint32_t chunk_len, uint32_t rnd);

/* ------------------------------------------------ device batch: send side */
/* One wire datagram (frame) of a fragmented message, planned on the host
 * (writeFragmented, gecko.go:107-129): the chunk is msg[chunk_off, +chunk_len). */
typedef struct hyobfs_gecko_frame {
    uint64_t chunk_off;
    uint32_t chunk_len;
    uint16_t pad_len;
    uint8_t msg_id;
    uint8_t idx_total;     /* chunkIdx << 4 | totalChunks, the wire's byte 2 */
} hyobfs_gecko_frame;

typedef struct hyobfs_gecko_batch {
    uint64_t n;                          /* frames */
    const uint8_t* msg;                  /* message bytes (device) */
    const hyobfs_gecko_frame* frames;    /* n frames (device) */
    const uint64_t* salts;               /* n Salamander salts (device), as hyobfs_batch.salts */
    /* Padding (the reference fills it from crypto/rand, gecko_frame.go:55): a keyed
       keystream, ChaCha with 8 rounds (the RFC 8439 block: constants, pad_key as
       8 little-endian words, a 32-bit block counter, pad_nonce as 3 words), each
       64-byte block's bytes in column order (bytes 16c..16c+15 = state words c,
       c+4, c+8, c+12 after the final addition).  Pad byte j of frame i is
       keystream byte out_off[i] + 13 + j: its offset in `out`, so every pad byte
       of a batch takes a different keystream byte.  Block b (64-bit) uses
       counter = b mod 2^32 and nonce word 0 XOR (b >> 32): no block repeats at
       any offset.  Draw a fresh key per batch (hyobfs_gecko_random_pad_key,
       getrandom); an explicit key makes the output reproducible (tests,
       oracle/gecko_ref.py).  An all-zero pad_key is rejected
       (HYOBFS_ERR_INVALID): it is what a caller that forgot the key passes. */
    uint8_t pad_key[32];
    uint8_t pad_nonce[12];
    uint32_t reserved_;
    uint8_t* out;                        /* device */
    const uint64_t* out_off;             /* frame i's wire datagram at out + out_off[i] (device);
                                            its length is 8 + 5 + pad_len + chunk_len */
    void* workspace;                     /* ignored (ABI 3: the encode kernel needs no scratch) */
    uint64_t workspace_bytes;            /* ignored */
    uint64_t out_cap;                    /* ignored (ABI 2 used it for the wire-tile kernel, since removed) */
} hyobfs_gecko_batch;

/* 0: kept for callers of ABI 1 (the wave-group kernel needs no workspace). */
uint64_t hyobfs_gecko_workspace_size(uint64_t n);
/* A fresh 256-bit pad key and 96-bit nonce from the OS (getrandom, the source of
   crypto/rand).  Returns HYOBFS_OK or HYOBFS_ERR_IO. */
int hyobfs_gecko_random_pad_key(uint8_t key[32], uint8_t nonce[12]);
/*
 * Encode and obfuscate every frame in one pass on the context's device:
 * out = salt || (header || pad || chunk) ^ BLAKE2b-256(PSK || salt)[i % 32]
 * (encodeFrame + Salamander Obfuscate, gecko.go:120-128 -> salamander.go:59-72).
 * Asynchronous on `stream` (NULL = null stream).  A frame the reference could
 * not have produced (total chunks outside [2, 8], chunk index >= total, or a
 * datagram longer than HYOBFS_GECKO_BUFFER_SIZE) is skipped on the device: its
 * output bytes are left untouched.  HYOBFS_ERR_INVALID for a missing pointer
 * or an all-zero pad_key.
 */
int hyobfs_gecko_encode_batch(hyobfs_salamander* ctx, const hyobfs_gecko_batch* b, void* stream);

/* --------------------------------------------- device batch: receive side */
typedef struct hyobfs_gecko_parsed {
    int32_t status;        /* HYOBFS_GECKO_PASS / _FRAGMENT / _EMPTY / _ERR_TRUNCATED / _ERR_INVALID */
    uint16_t pad_len;
    uint8_t msg_id;
    uint8_t idx_total;     /* chunkIdx << 4 | totalChunks */
    uint32_t payload_off;  /* payload = datagram[payload_off, payload_off + payload_len) */
    uint32_t payload_len;
} hyobfs_gecko_parsed;

/*
 * Classify and parse n deobfuscated datagrams (ReadFrom, gecko.go:170-193 ->
 * decodeFrame): datagram i is in[in_off[i], +in_len[i]) (device pointers, as
 * produced by hyobfs_salamander_deobfuscate_batch; in_len[i] == 0 marks a
 * dropped one).  One thread per datagram on the current device.
 */
int hyobfs_gecko_parse_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint64_t n,
                             hyobfs_gecko_parsed* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HYOBFS_GECKO_H */
