// gecko_host.cpp -- host side of the Gecko frame codec (include/hyobfs_gecko.h):
// encodeFrame / decodeFrame (gecko_frame.go:39-86) and randomPadLen
// (gecko.go:131-138).  Plain host C++; the device batch calls live in
// gecko.hip and hyobfs_api.cpp.
#include <errno.h>
#include <sys/random.h>

#include <algorithm>
#include <cstring>

#include "../../include/hyobfs_gecko.h"

namespace {

bool fill_random(uint8_t* p, size_t n) {   // crypto/rand.Read
    while (n) {
        const ssize_t r = getrandom(p, n, 0);
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) return false;
        p += r;
        n -= (size_t)r;
    }
    return true;
}

bool chunks_ok(unsigned total, unsigned idx) {
    return total >= HYOBFS_GECKO_MIN_CHUNKS && total <= HYOBFS_GECKO_MAX_CHUNKS && idx < total;
}

}  // namespace

extern "C" {

int hyobfs_gecko_random_pad_key(uint8_t key[32], uint8_t nonce[12]) {   // crypto/rand, gecko_frame.go:55
    if (!key || !nonce) return HYOBFS_ERR_INVALID;
    return fill_random(key, 32) && fill_random(nonce, 12) ? HYOBFS_OK : HYOBFS_ERR_IO;
}

int64_t hyobfs_gecko_encode_frame(const hyobfs_gecko_header* h, const uint8_t* payload, size_t len, uint8_t* out,
                                  size_t cap) {
    if (!h || !chunks_ok(h->total_chunks, h->chunk_idx)) return HYOBFS_GECKO_ERR_INVALID;
    const size_t needed = HYOBFS_GECKO_HEADER_LEN + (size_t)h->pad_len + len;
    if (!out || cap < needed) return HYOBFS_GECKO_ERR_TRUNCATED;
    out[0] = HYOBFS_GECKO_FLAG_FRAGMENT;
    out[1] = h->msg_id;
    out[2] = (uint8_t)(h->chunk_idx << 4 | (h->total_chunks & 0x0f));
    out[3] = (uint8_t)(h->pad_len >> 8);   // big-endian
    out[4] = (uint8_t)h->pad_len;
    if (!fill_random(out + HYOBFS_GECKO_HEADER_LEN, h->pad_len)) return HYOBFS_ERR_IO;
    if (len) std::memmove(out + HYOBFS_GECKO_HEADER_LEN + h->pad_len, payload, len);
    return (int64_t)needed;
}

int hyobfs_gecko_decode_frame(const uint8_t* in, size_t len, hyobfs_gecko_header* h, size_t* payload_off) {
    if (len < HYOBFS_GECKO_HEADER_LEN || !in) return HYOBFS_GECKO_ERR_TRUNCATED;
    if (!(in[0] & HYOBFS_GECKO_FLAG_FRAGMENT)) return HYOBFS_GECKO_ERR_INVALID;
    hyobfs_gecko_header r{};
    r.msg_id = in[1];
    r.chunk_idx = in[2] >> 4;
    r.total_chunks = in[2] & 0x0f;
    r.pad_len = (uint16_t)((in[3] << 8) | in[4]);
    if (!chunks_ok(r.total_chunks, r.chunk_idx)) return HYOBFS_GECKO_ERR_INVALID;
    if (HYOBFS_GECKO_HEADER_LEN + (size_t)r.pad_len > len) return HYOBFS_GECKO_ERR_TRUNCATED;
    if (h) *h = r;
    if (payload_off) *payload_off = HYOBFS_GECKO_HEADER_LEN + r.pad_len;
    return HYOBFS_OK;
}

uint32_t hyobfs_gecko_pad_len(int min_pkt, int max_pkt, uint32_t chunk_len, uint32_t rnd) {
    const int64_t base = HYOBFS_SALT_LEN + HYOBFS_GECKO_HEADER_LEN + (int64_t)chunk_len;
    const int64_t lo = std::max<int64_t>(min_pkt, base);
    if (lo > max_pkt) return 0;
    const int64_t span = (int64_t)max_pkt - lo + 1;   // randIntn(span)
    const int64_t r = span <= 1 ? 0 : (int64_t)(rnd % (uint32_t)span);
    return (uint32_t)(lo - base + r);
}

}  // extern "C"
