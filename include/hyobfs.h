/*
 * hyobfs.h -- C ABI of libhyobfs: Hysteria "Salamander" packet obfuscation on
 * AMD Instinct MI355X (gfx950).
 *
 * The ABI replaces, one for one, the Go surface of the reference's hot path
 * (paths relative to apernet/hysteria):
 *
 *   Go (reference)                                       C ABI (this header)
 *   ---------------------------------------------------  -----------------------------------
 *   newSalamanderObfuscator(psk)  extras/obfs/salamander.go:34-46
 *                                                        hyobfs_salamander_new
 *   ErrPSKTooShort                extras/obfs/salamander.go:21
 *                                                        HYOBFS_ERR_PSK_TOO_SHORT
 *   (o *salamanderObfuscator).Obfuscate(in, out) int     salamander.go:59-72
 *                                                        hyobfs_salamander_obfuscate
 *   (o *salamanderObfuscator).Deobfuscate(in, out) int   salamander.go:74-86
 *                                                        hyobfs_salamander_deobfuscate
 *   keyLocked(salt) [32]byte      salamander.go:88-91    hyobfs_salamander_key
 *   obfuscator interface          extras/obfs/conn.go:15-18
 *                                                        the two calls above (per datagram)
 *                                                        + the *_batch calls (N datagrams)
 *   RandSrc (math/rand, :29,43,65) salt source           hyobfs_salamander_seed / _next_salts
 *   obfsPacketConn.ReadFrom/WriteTo  extras/obfs/conn.go:73-99
 *                                                        include/hyobfs_conn.h
 *
 * Rules kept from the reference:
 *   - A per-packet call returns the number of bytes written to out, and 0 for
 *     an invalid packet or a too-small out buffer (conn.go:12-14).  There is no
 *     per-packet error value.
 *   - Obfuscate writes len(in)+8 bytes: the 8-byte salt, then in[i] ^ key[i%32];
 *     it returns 0 when out_len < in_len + 8 (salamander.go:60-62).
 *   - Deobfuscate writes len(in)-8 bytes and returns 0 when in_len <= 8 or
 *     out_len < in_len - 8 (salamander.go:75-77).
 *   - key = BLAKE2b-256(PSK || salt), unkeyed (salamander.go:88-91).
 *   - Construction fails with HYOBFS_ERR_PSK_TOO_SHORT for PSK < 4 bytes.
 *
 * The salt: the reference draws it from a time-seeded math/rand source inside
 * Obfuscate (salamander.go:43,65).  Here the caller passes it (a Go adapter
 * reads its own RandSrc under its lock, so wire bytes stay identical), or asks
 * the context's generator for it (hyobfs_salamander_next_salts).
 *
 * Threading: a context may be used from several threads.  The per-packet
 * calls serialise on the context (like the reference's lk, salamander.go:64-67);
 * batch calls only enqueue work on the caller's stream.
 *
 * Every compute call runs on the GPU.  There is no CPU fallback: without a
 * usable gfx950 device hyobfs_salamander_new fails with HYOBFS_ERR_NO_DEVICE.
 */
#ifndef HYOBFS_H
#define HYOBFS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version.  4 (this header) against 3:
 *   - new kernel HYOBFS_KERNEL_FLAT (3): contiguous input into packed output on the
 *     flat kernel (16-byte aligned in; 3 meant STREAM in ABI 2 and was rejected in
 *     ABI 3);
 *   - contiguous input with packed output needs more scratch (the flat kernel's tile
 *     descriptors, 24 B per 16 KiB of out_cap, and key records, 64 B per datagram):
 *     ask hyobfs_batch_workspace_bytes;
 *   - hyobfs_conn_free on a connection that was never closed closes its fd (in ABI 2
 *     it detached and left the socket open; include/hyobfs_conn.h).
 * 3 against 2:
 *   - HYOBFS_KERNEL_STREAM (3) is gone (the stream kernel lost to the wave-group
 *     kernel on every measured layout); hyobfs_salamander_set_kernel rejects 3;
 *   - hyobfs_gecko_workspace_bytes is gone, and hyobfs_gecko_batch's workspace,
 *     workspace_bytes and out_cap are ignored (the Gecko wire-tile kernel is gone);
 *   - contiguous input with slotted output needs 2 x hyobfs_batch_workspace_size(n)
 *     + 8 n bytes of scratch (was 8 n + block sums): ask hyobfs_batch_workspace_bytes;
 *   - new: hyobfs_device_pci_bus_id.
 * 2 against 1:
 *   - struct hyobfs_gecko_batch: pad_seed (u64) became pad_key[32], pad_nonce[12]
 *     and reserved_ (hyobfs_gecko.h), so the fields after it moved;
 *   - HYOBFS_KERNEL_* values: 2 is TILE (was PERSISTENT), 3..6 are rejected;
 *   - hyobfs_conn_close no longer frees the connection: hyobfs_conn_free does
 *     (include/hyobfs_conn.h), and calls after close fail with EBADF;
 *   - new status HYOBFS_ERR_CLOSED; a zero Gecko pad key is rejected;
 *   - CONTIGUOUS input (struct hyobfs_batch): in_off == NULL, in_stride == 0 and
 *     in_len != NULL now put the datagrams back to back.  In ABI 1 the same fields
 *     put every datagram at `in`.  With in_len == NULL (len_uniform), in_stride 0
 *     still means "every datagram at in".  A v1 caller that relied on that must
 *     pass in_off (all zeros) instead.
 * Bindings compare hyobfs_abi_version() with the version they were written
 * for and refuse a mismatch (hysteria_amd/_lib.py does). */
#define HYOBFS_ABI_VERSION 4

#define HYOBFS_PSK_MIN_LEN 4  /* smPSKMinLen, salamander.go:14 */
#define HYOBFS_SALT_LEN 8     /* smSaltLen,   salamander.go:15 */
#define HYOBFS_KEY_LEN 32     /* smKeyLen,    salamander.go:16 */
#define HYOBFS_UDP_BUFFER_SIZE 2048 /* udpBufferSize, conn.go:10 */

/* status codes (negative = error) */
#define HYOBFS_OK 0
#define HYOBFS_ERR_PSK_TOO_SHORT (-1) /* ErrPSKTooShort, salamander.go:21 */
#define HYOBFS_ERR_INVALID (-2)       /* bad argument (NULL, misaligned, ...) */
#define HYOBFS_ERR_HIP (-3)           /* HIP runtime error */
#define HYOBFS_ERR_NOMEM (-4)         /* allocation failed */
#define HYOBFS_ERR_NO_DEVICE (-5)     /* no usable gfx950 device */
#define HYOBFS_ERR_IO (-6)            /* socket error (hyobfs_conn_*); errno kept */
#define HYOBFS_ERR_CLOSED (-7)        /* call on a closed connection (Go: net.ErrClosed) */

typedef struct hyobfs_salamander hyobfs_salamander; /* opaque context */

/* ------------------------------------------------------------------ basics */
int hyobfs_abi_version(void);
/* sha256 (16 hex digits) of the kernel sources this library was built from
   (scripts/src_sha.py); "unknown" for builds outside the Makefile.  bench.py
   uses committed PMC traffic figures only when they match it. */
const char* hyobfs_build_id(void);
const char* hyobfs_status_string(int status);
/* number of HIP devices visible to this process (0 when none) */
int hyobfs_device_count(void);
/* PCI bus id of HIP device `device` ("dddd:bb:dd.f", NUL-terminated, len >= 13):
   which physical card a process bound (bench.py records it per rank). */
int hyobfs_device_pci_bus_id(int device, char* buf, int len);

/* ------------------------------------------------------------- lifecycle */
/* newSalamanderObfuscator (salamander.go:34-46) + GPU binding.  Copies the
   PSK, precomputes its BLAKE2b prefix, binds the context to HIP device
   `device`.  *out is set only on HYOBFS_OK. */
int hyobfs_salamander_new(const uint8_t* psk, size_t psk_len, int device,
                          hyobfs_salamander** out);
/* Drops the caller's reference.  A connection made on the context
   (hyobfs_conn_wrap) holds its own reference until hyobfs_conn_free, so the
   context is destroyed only when the last of them goes (any order). */
void hyobfs_salamander_free(hyobfs_salamander* ctx);
int hyobfs_salamander_device(const hyobfs_salamander* ctx);

/* Batch kernel of this context (no reference counterpart: a tuning knob).
   HYOBFS_KERNEL_AUTO runs the tile kernel on slotted batches whose region edges
   are all multiples of 8 (one length, slot and input stride multiples of 8,
   payloads of 16 bytes or more, nothing dropped) -- the uniform 1200-byte batch
   of the benchmark -- and the wave-group kernel on every other batch (packed
   output, ragged lengths, any alignment; contiguous input scans its lengths
   alongside the widths).  HYOBFS_KERNEL_WAVE forces the wave-group kernel;
   HYOBFS_KERNEL_FLAT runs the flat kernel on contiguous input into packed output
   from 16-byte aligned input (one-shot workgroups per 16 KiB of output, keys from
   hasher workgroups; measured slower than the wave kernel on the ragged configs[2]
   batch) and is AUTO elsewhere; HYOBFS_KERNEL_TILE is AUTO.  The
   HYOBFS_KERNEL environment variable (wave|tile|flat) overrides AUTO.  Returns HYOBFS_ERR_INVALID for an unknown value.
   May be called while other threads run batches on the context (an atomic
   setting; a batch uses the value it read when it started).  Outputs are
   identical. */
enum {
    HYOBFS_KERNEL_AUTO = 0,
    HYOBFS_KERNEL_WAVE = 1,
    HYOBFS_KERNEL_TILE = 2,
    HYOBFS_KERNEL_FLAT = 3
};
int hyobfs_salamander_set_kernel(hyobfs_salamander* ctx, int kernel);

/* Salt source (the reference's RandSrc, salamander.go:29,43,65).  The context
   seeds itself from the clock at creation like the reference; _seed makes it
   deterministic.  _next_salts writes n salts (8 bytes each, in host memory). */
void hyobfs_salamander_seed(hyobfs_salamander* ctx, uint64_t seed);
void hyobfs_salamander_next_salts(hyobfs_salamander* ctx, uint8_t* salts, size_t n);

/* ---------------------------------------------------------- per datagram */
/* keyLocked (salamander.go:88-91) computed on the GPU: key = BLAKE2b-256(PSK||salt). */
int hyobfs_salamander_key(hyobfs_salamander* ctx, const uint8_t salt[8],
                          uint8_t key[32]);
/* keyLocked for n salts at once: keys[32*i..] = BLAKE2b-256(PSK || salts[i]).
   Device pointers, enqueued on stream (a hipStream_t; NULL = the null stream). */
int hyobfs_salamander_keys_batch(hyobfs_salamander* ctx, const uint64_t* salts,
                                 uint8_t* keys, uint64_t n, void* stream);
/* Obfuscate (salamander.go:59-72) with an explicit salt.  Host buffers, synchronous. */
size_t hyobfs_salamander_obfuscate(hyobfs_salamander* ctx, const uint8_t* in,
                                   size_t in_len, const uint8_t salt[8],
                                   uint8_t* out, size_t out_len);
/* Obfuscate drawing the salt from the context's generator (the exact
   reference call shape: Obfuscate(in, out) int). */
size_t hyobfs_salamander_obfuscate_auto(hyobfs_salamander* ctx, const uint8_t* in,
                                        size_t in_len, uint8_t* out, size_t out_len);
/* Deobfuscate (salamander.go:74-86).  Host buffers, synchronous. */
size_t hyobfs_salamander_deobfuscate(hyobfs_salamander* ctx, const uint8_t* in,
                                     size_t in_len, uint8_t* out, size_t out_len);

/* ------------------------------------------------------------------ batch */
/*
 * A batch of n datagrams in device-accessible memory (device memory, or
 * mapped pinned host memory).  Per packet i:
 *
 *   input   : len  L_i = in_len ? in_len[i] : len_uniform
 *             bytes at in + (in_off ? in_off[i] : i * in_stride)       (any alignment)
 *             CONTIGUOUS input: in_off == NULL, in_stride == 0 and in_len != NULL
 *             put datagram i at in + L_0 + ... + L_{i-1} (back to back; no
 *             offset array).  Without in_len, in_stride == 0 puts every
 *             datagram at `in`.
 *   salt    : obfuscate only: salts[i], 8 bytes, little-endian u64
 *             (salt byte b = (salts[i] >> 8b) & 0xff)
 *   output  : W_i = L_i + 8 (obfuscate) or L_i - 8 (deobfuscate)
 *             valid iff W_i > 0 and W_i <= cap_i, where cap_i = pkt_cap
 *             (0 = unlimited), further limited to out_stride when slotted
 *             (that is `len(out)` of the per-packet call)
 *   layout  : out_stride > 0  -> slotted: out_off_i = i * out_stride
 *             out_stride == 0 -> packed : out_off_i = exclusive prefix sum of
 *                                the valid W's (the datagrams sit back to back)
 *             a packet whose region passes out_cap is dropped (packed: so is
 *             every later one, offsets never move)
 *   result  : out_off[i] (if non-NULL) = out_off_i; out_len[i] (if non-NULL)
 *             = W_i, or 0 for a dropped packet (the reference's "return 0");
 *             *out_total (if non-NULL, device memory) = bytes written.
 *             Bytes of `out` outside valid regions are not written.
 *
 * `out` must be 16-byte aligned.  All pointers are device-accessible; the
 * call only enqueues work on `stream` (a hipStream_t; NULL = the HIP null
 * stream, as everywhere in HIP) and returns.  workspace: device scratch of at
 * least hyobfs_batch_workspace_bytes(b) bytes (0 for slotted batches with
 * explicit offsets; hyobfs_batch_workspace_size(n) for packed ones), or NULL:
 * then the scratch is allocated stream-ordered from a context-owned memory pool
 * and freed behind the launch on the same stream (any number of caller streams
 * and threads; the pool keeps at most 32 MiB cached between calls).
 */
typedef struct hyobfs_batch {
    uint64_t n;
    const uint8_t* in;
    const uint64_t* in_off;
    uint64_t in_stride;
    const uint32_t* in_len;
    uint32_t len_uniform;
    uint32_t pkt_cap;
    const uint64_t* salts;
    uint8_t* out;
    uint64_t out_cap;
    uint64_t out_stride;
    uint64_t* out_off;
    uint32_t* out_len;
    uint64_t* out_total;
    void* workspace;
    uint64_t workspace_bytes;
} hyobfs_batch;

/* Scratch of a packed batch with explicit or strided input offsets: (ceil(n/256)+1) x 8. */
uint64_t hyobfs_batch_workspace_size(uint64_t n);
/* Scratch any batch needs, whatever the kernel choice: the above for packed
   batches with explicit offsets; for contiguous input twice that (width and
   length sums), plus, into packed output from 16-byte aligned input, the flat
   kernel's scratch (16 B + 24 B per 16 KiB of out_cap, rounded up to 256, + 256 B
   + 64 B per datagram), or, into slotted output (or with
   HYOBFS_PACKED_RUN_LOG2 shortening the packed runs), 8 B per datagram (the input
   offsets a prepass writes); 0 for other slotted batches. */
uint64_t hyobfs_batch_workspace_bytes(const hyobfs_batch* b);
/* Which batch kernel a call with this batch would run under the context's
   setting (HYOBFS_KERNEL_TILE, _FLAT or _WAVE; HYOBFS_KERNEL_AUTO for an
   empty batch), or a negative status for an invalid batch.  No device work:
   tests use it to prove which kernel their case exercised. */
int hyobfs_salamander_batch_kernel(hyobfs_salamander* ctx, const hyobfs_batch* b, int obfuscate);
int hyobfs_salamander_obfuscate_batch(hyobfs_salamander* ctx, const hyobfs_batch* b,
                                      void* stream);
int hyobfs_salamander_deobfuscate_batch(hyobfs_salamander* ctx, const hyobfs_batch* b,
                                        void* stream);

/* ---------------------------------------------------- multi-GPU shards */
/*
 * The path shards by datagram index with no exchange step: every datagram
 * depends only on (PSK, salt, payload) (salamander.go:59-86), so shard i is
 * an ordinary batch on the device of ctxs[i], with buffers on that device.
 * The sharded calls launch every shard on its context's stream, then wait
 * for all of them; the return value is the first failing shard's status
 * (HYOBFS_OK when all succeed).  Contexts must be distinct (one per shard);
 * two shards may share a device.  No collective and no peer traffic.
 */
int hyobfs_salamander_obfuscate_batch_sharded(hyobfs_salamander* const* ctxs,
                                              const hyobfs_batch* batches, int nshards);
int hyobfs_salamander_deobfuscate_batch_sharded(hyobfs_salamander* const* ctxs,
                                                const hyobfs_batch* batches, int nshards);
/*
 * Shard planning (host only, no device call): split datagrams [0, n) into
 * nshards contiguous index ranges [bounds[i], bounds[i+1]) of equal traffic,
 * weighting datagram k by in_len[k] + 8 (its wire or payload bytes; a
 * ragged batch is split by cumulative bytes, a uniform one by count).
 * in_len == NULL means every datagram has the same length.  bounds has
 * nshards + 1 entries, bounds[0] = 0 and bounds[nshards] = n.
 */
int hyobfs_shard_bounds(const uint32_t* in_len, uint64_t n, int nshards, uint64_t* bounds);

/* ------------------------------------------------- host-resident batches */
/*
 * The path starts and ends in host memory (UDP socket buffers).  These calls
 * take a hyobfs_batch whose pointers are HOST pointers, in the slotted layout
 * of recvmmsg/sendmmsg rings: in_off == NULL (input slot i at i * in_stride),
 * out_stride > 0 (output slot i at i * out_stride); in_len, salts, out_len
 * are host arrays (in_len may be NULL with len_uniform).  out_off/out_total
 * and workspace are ignored.  The batch runs in chunks of `chunk` datagrams
 * (0 = library default) through device buffers owned by the context, on
 * three streams, so the host-to-device copy of chunk k+1, the kernels of
 * chunk k and the device-to-host copy of chunk k-1 overlap.  Synchronous:
 * returns when every output byte is in host memory.  Host buffers allocated
 * with hyobfs_host_alloc (pinned) copy at full PCIe rate; pageable memory
 * works but is staged by the runtime.  The device-to-host copy moves whole
 * output slots: bytes of a slot past out_len[i] are unspecified afterwards.
 * When in, out, in_len, salts (obfuscate) and out_len are ALL device-mapped
 * host memory (hyobfs_host_alloc), the batch instead runs as one batch call
 * on the mapped pointers (zero-copy, `chunk` unused; HYOBFS_HOST_ZEROCOPY=0
 * turns this off) and, like the device batches, writes only the regions.
 */
int hyobfs_salamander_obfuscate_host(hyobfs_salamander* ctx, const hyobfs_batch* b,
                                     uint64_t chunk);
int hyobfs_salamander_deobfuscate_host(hyobfs_salamander* ctx, const hyobfs_batch* b,
                                       uint64_t chunk);
/* pinned, device-mapped host memory (hipHostMalloc) */
void* hyobfs_host_alloc(size_t bytes);
void hyobfs_host_free(void* p);

/* ----------------------------------------------- synthetic inputs (bench) */
/* Device-side generators of the seeded inputs of BASELINE.md ("Synthetic
   inputs"), so large batches never cross PCIe.  SplitMix64 counter form:
   x_k = mix(seed + (k+1) * 0x9e3779b97f4a7c15). */
int hyobfs_synth_stream(uint8_t* dst, uint64_t nbytes, uint64_t seed,
                        uint64_t start_byte, void* stream);
int hyobfs_synth_u64(uint64_t* dst, uint64_t n, uint64_t seed, uint64_t first,
                     void* stream);
int hyobfs_synth_bimodal_lengths(uint32_t* dst, uint64_t n, uint64_t seed,
                                 uint64_t first, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HYOBFS_H */
