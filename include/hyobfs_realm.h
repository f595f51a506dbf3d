/*
 * hyobfs_realm.h -- realm hole-punch packet mask (extras/realm/punch.go).
 *
 * A punch packet is  salt(8) || plain ^ SHA-256(obfsKey(32) || salt)[i % 32]
 * with plain = magic "HYRLMv1\0"(8) || type(1) || nonce(16) || padding(0..1024)
 * (punch.go:13-100, :133-141).  Every inbound datagram is tried against every
 * registered attempt's (nonce, obfsKey) (punch_conn.go:146-165); the device
 * batch does all (datagram, attempt) pairs at once, one SHA-256 compression
 * per pair: only the first 25 plain bytes decide a match.
 *
 * Plain C ABI: pointers, sizes, integer status codes.
 */
#ifndef HYOBFS_REALM_H
#define HYOBFS_REALM_H

#include <stddef.h>
#include <stdint.h>

#include "hyobfs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* punch.go:13-31, client.go:21-22 */
#define HYOBFS_PUNCH_MAX_PADDING 1024
#define HYOBFS_PUNCH_SALT_LEN 8
#define HYOBFS_PUNCH_HEADER_LEN 25
#define HYOBFS_PUNCH_MIN_WIRE_LEN (HYOBFS_PUNCH_SALT_LEN + HYOBFS_PUNCH_HEADER_LEN)
#define HYOBFS_PUNCH_MAX_WIRE_LEN (HYOBFS_PUNCH_MIN_WIRE_LEN + HYOBFS_PUNCH_MAX_PADDING)
#define HYOBFS_PUNCH_NONCE_LEN 16
#define HYOBFS_PUNCH_KEY_LEN 32
#define HYOBFS_PUNCH_HELLO 0x01
#define HYOBFS_PUNCH_ACK 0x02
/* ErrInvalidPunchPacket (punch.go:24), by reason */
#define HYOBFS_PUNCH_ERR_TOO_SHORT (-30)
#define HYOBFS_PUNCH_ERR_TOO_LONG (-31)
#define HYOBFS_PUNCH_ERR_BAD_MAGIC (-32)
#define HYOBFS_PUNCH_ERR_UNKNOWN_TYPE (-33)
#define HYOBFS_PUNCH_ERR_NONCE_MISMATCH (-34)

/* One registered attempt's metadata, decoded from hex (decodePunchMetadata, punch.go:102-113). */
typedef struct hyobfs_punch_attempt {
    uint8_t nonce[HYOBFS_PUNCH_NONCE_LEN];
    uint8_t key[HYOBFS_PUNCH_KEY_LEN];
} hyobfs_punch_attempt;

/*
 * EncodePunchPacket (punch.go:42-71) with the random parts passed in: salt
 * (8 bytes) and padding (padding_len <= 1024 bytes).  Writes 33 + padding_len
 * bytes to out.  Returns that length, HYOBFS_PUNCH_ERR_UNKNOWN_TYPE, or
 * HYOBFS_ERR_INVALID when cap is too small.  Host memory.
 */
int64_t hyobfs_punch_encode(uint8_t type, const hyobfs_punch_attempt* a, const uint8_t salt[8],
                            const uint8_t* padding, size_t padding_len, uint8_t* out, size_t cap);
/*
 * DecodePunchPacket (punch.go:73-100): on success returns HYOBFS_OK with the
 * packet type and padding length; otherwise one of the HYOBFS_PUNCH_ERR_*
 * codes, checked in the reference's order (length, magic, type, nonce).
 */
int hyobfs_punch_decode(const uint8_t* packet, size_t len, const hyobfs_punch_attempt* a, uint8_t* type,
                        uint32_t* padding_len);
/* xorPunchPacket's mask (punch.go:133-141): SHA-256(key || salt). */
void hyobfs_punch_mask(const uint8_t key[32], const uint8_t salt[8], uint8_t mask[32]);

/*
 * decodePunchPacket over a batch (punch_conn.go:146-165), on the current
 * device: datagram i is in[in_off[i], +in_len[i]); attempts[0..m) on the
 * device.  match[i] = the lowest attempt index the datagram decodes under,
 * or -1; type[i] and padding[i] describe that match.  (The reference walks a
 * map, so which of several matching attempts wins is unspecified there; a
 * real collision needs a SHA-256 prefix collision.)  Asynchronous on stream.
 */
int hyobfs_punch_match_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint64_t n,
                             const hyobfs_punch_attempt* attempts, uint32_t m, int32_t* match, uint8_t* type,
                             uint32_t* padding, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HYOBFS_REALM_H */
