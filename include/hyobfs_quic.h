/*
 * hyobfs_quic.h -- QUIC Initial packet unprotection for the sniffer
 * (apernet/hysteria extras/sniff/internal/quic), batched on the GPU.
 *
 *   Go (reference)                                        C ABI
 *   ----------------------------------------------------  ------------------------------------------
 *   ParseInitialHeader(data)           header.go:24-89    hyobfs_quic_parse_initial_header (host)
 *   hkdf.Extract + hkdfExpandLabel     payload.go:34-35,  hyobfs_quic_initial_secret (host)
 *                                      packet_protector.go:177-193
 *   NewProtectionKey(suite, secret, v) packet_protector.go:21-23,102-156
 *                                                         hyobfs_quic_new_protection_key (host)
 *   (*PacketProtector).UnProtect(packet, pnOffset, pnMax)
 *                                      packet_protector.go:46-79
 *                                                         hyobfs_quic_unprotect_batch (device)
 *   ReadCryptoPayload(packet)          payload.go:21-60   hyobfs_quic_read_crypto_payload_batch (device)
 *     extractCryptoFrames              payload.go:73-112
 *     assembleCryptoFrames             payload.go:116-148
 *
 * The batched calls take n packets at packets[off[i], +len[i]) in device
 * memory and work IN PLACE, as the reference does: UnProtect removes header
 * protection from the packet's first byte and packet-number bytes and opens
 * the AEAD into the payload's own storage (payload[:0], :74), so afterwards
 * the packet holds header || plaintext || (the 16 tag bytes, unchanged).  When
 * authentication fails the header is unmasked but the payload is left as it
 * was (the reference's buffer is then either untouched or zeroed, depending on
 * Go's GCM implementation).  Results are per packet (hyobfs_quic_result);
 * calls are asynchronous on `stream`.
 *
 * Plain C ABI: pointers, sizes, integer status codes.
 */
#ifndef HYOBFS_QUIC_H
#define HYOBFS_QUIC_H

#include <stddef.h>
#include <stdint.h>

#include "hyobfs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* quic.go:3-13 */
#define HYOBFS_QUIC_V1 0x00000001u
#define HYOBFS_QUIC_V2 0x6b3343cfu
/* crypto/tls cipher suite ids (packet_protector.go:103-130) */
#define HYOBFS_QUIC_TLS_AES_128_GCM_SHA256 0x1301
#define HYOBFS_QUIC_TLS_CHACHA20_POLY1305_SHA256 0x1303
/* payload.go:17-18 */
#define HYOBFS_QUIC_MAX_CRYPTO_FRAME_LEN (256 * 1024)
#define HYOBFS_QUIC_MAX_CRYPTO_PAYLOAD_LEN (256 * 1024)
/* crypto frames one packet may carry in the device parser (no reference
   counterpart: the reference keeps a Go slice) */
#define HYOBFS_QUIC_MAX_FRAMES 256

/* per-packet status, by the reference's error */
#define HYOBFS_QUIC_ERR_EOF (-40)          /* header.go: io.EOF / io.ErrUnexpectedEOF / varint read */
#define HYOBFS_QUIC_ERR_NOT_QUIC (-41)     /* "not a QUIC packet", header.go:45-47 */
#define HYOBFS_QUIC_ERR_VERSION (-42)      /* "unsupported version", payload.go:27-29 */
#define HYOBFS_QUIC_ERR_INVALID (-43)      /* "invalid packet" (offset or Length 0), payload.go:30-32 */
#define HYOBFS_QUIC_ERR_SHORT (-44)        /* "packet is too short", payload.go:44-46 */
#define HYOBFS_QUIC_ERR_TOO_SMALL (-45)    /* "packet with long header is too small", packet_protector.go:47-49;
                                              also a short-header packet with no room for the 16-byte sample
                                              (the reference's slice expression panics there) or pnOffset < 0 */
#define HYOBFS_QUIC_ERR_AUTH (-46)         /* "decryption failed" (AEAD Open), packet_protector.go:74-77 */
#define HYOBFS_QUIC_ERR_FRAME_TYPE (-47)   /* "encountered unexpected frame type", payload.go:83-85 */
#define HYOBFS_QUIC_ERR_FRAME_EOF (-48)    /* varint EOF / io.ErrUnexpectedEOF in a frame, payload.go:76-104 */
#define HYOBFS_QUIC_ERR_FRAME_TOO_LARGE (-49) /* "crypto frame data too large", payload.go:99-101 */
#define HYOBFS_QUIC_ERR_ASSEMBLE (-50)     /* "unable to assemble crypto frames", payload.go:55-58 */
#define HYOBFS_QUIC_ERR_OUT_CAP (-51)      /* assembled data larger than out_cap[i] (out_len = the size needed) */
#define HYOBFS_QUIC_ERR_FRAMES (-52)       /* more than HYOBFS_QUIC_MAX_FRAMES crypto frames */
#define HYOBFS_QUIC_ERR_SUITE (-53)        /* "not supported cipher suite", packet_protector.go:155 */

/* ProtectionKey (packet_protector.go:82-86) as derived key material: the AEAD
   key (16 bytes used for AES-128-GCM, 32 for ChaCha20-Poly1305), the 12-byte
   IV, and the header-protection key (16 / 32 bytes). */
typedef struct hyobfs_quic_key {
    uint32_t suite;    /* HYOBFS_QUIC_TLS_* */
    uint8_t iv[12];
    uint8_t key[32];
    uint8_t hp[32];
} hyobfs_quic_key;     /* 80 bytes */

/* Header (header.go:13-20); connection IDs and token as offsets into data. */
typedef struct hyobfs_quic_header {
    uint8_t type;
    uint8_t dcid_len;
    uint8_t scid_len;
    uint8_t pad_;
    uint32_t version;
    uint32_t dcid_off;
    uint32_t scid_off;
    uint32_t token_off;
    uint32_t token_len;
    uint64_t length;   /* Length field */
    int64_t offset;    /* bytes read so far = the packet-number offset */
} hyobfs_quic_header;

/* Per-packet result of the batched calls. */
typedef struct hyobfs_quic_result {
    int32_t status;     /* HYOBFS_OK or HYOBFS_QUIC_ERR_* */
    uint32_t hdr_len;   /* pnOffset + pnLen: the plaintext starts here */
    uint32_t plain_len; /* plaintext bytes (payload - 16-byte tag) */
    uint32_t out_len;   /* read_crypto_payload: assembled CRYPTO bytes written to out */
    int64_t pn;         /* decoded packet number (decodePacketNumber, packet_protector.go:161-174) */
} hyobfs_quic_result;   /* 24 bytes */

/* ParseInitialHeader (header.go:24-89): HYOBFS_OK, HYOBFS_QUIC_ERR_EOF or
   HYOBFS_QUIC_ERR_NOT_QUIC.  Host memory. */
int hyobfs_quic_parse_initial_header(const uint8_t* data, size_t len, hyobfs_quic_header* out);

/* The Initial secret of one side: HKDF-Extract(getSalt(v), dcid) then
   hkdfExpandLabel(., "client in" | "server in", "", 32) (payload.go:34-35,
   packet_protector_test.go:39-40).  server != 0 selects "server in". */
int hyobfs_quic_initial_secret(const uint8_t* dcid, size_t dcid_len, uint32_t version, int server,
                               uint8_t out[32]);

/* newProtectionKey (packet_protector.go:102-156): key/iv/hp from a 32-byte
   traffic secret with the version's labels (quic.go:38-59).
   HYOBFS_QUIC_ERR_SUITE for a suite other than the two above. */
int hyobfs_quic_new_protection_key(uint16_t suite, const uint8_t* secret, size_t secret_len, uint32_t version,
                                   hyobfs_quic_key* out);

/* hkdfExpandLabel (packet_protector.go:177-193) with SHA-256, length <= 255*32. */
int hyobfs_quic_hkdf_expand_label(const uint8_t* secret, size_t secret_len, const char* label,
                                  const uint8_t* context, size_t context_len, uint8_t* out, size_t length);

/*
 * UnProtect over a batch, on the current device.  Packet i is
 * packets[off[i], +len[i]), its key keys[i * key_stride] (key_stride 0: one
 * key for all), its packet-number offset pn_offset[i] and largest packet
 * number pn_max[i] (pn_max NULL: 0 for all).  All arrays are device memory.
 * res[i] gets the status, hdr_len, plain_len and pn.
 */
int hyobfs_quic_unprotect_batch(uint8_t* packets, const uint64_t* off, const uint32_t* len, uint64_t n,
                                const hyobfs_quic_key* keys, uint32_t key_stride, const int64_t* pn_offset,
                                const int64_t* pn_max, hyobfs_quic_result* res, void* stream);

/* Device workspace read_crypto_payload_batch needs for n packets. */
uint64_t hyobfs_quic_workspace_size(uint64_t n);

/*
 * ReadCryptoPayload over a batch of client Initial packets, on the current
 * device: parse the long header, derive the client Initial key from the
 * destination connection ID (HKDF on the device), UnProtect
 * packets[off[i], +offset+Length) with pnMax 2 in place, extract the CRYPTO
 * frames and assemble them into out[out_off[i], +out_cap[i]); res[i].out_len
 * = the assembled length.  workspace: hyobfs_quic_workspace_size(n) bytes of
 * device memory.  Frames sharing one offset keep packet order (the
 * reference's sort.Slice is not stable past 12 frames).
 */
int hyobfs_quic_read_crypto_payload_batch(uint8_t* packets, const uint64_t* off, const uint32_t* len, uint64_t n,
                                          uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                          hyobfs_quic_result* res, void* workspace, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HYOBFS_QUIC_H */
