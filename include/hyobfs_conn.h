/*
 * hyobfs_conn.h -- obfsPacketConn (apernet/hysteria extras/obfs/conn.go) over
 * a UDP socket, with the Salamander work on the GPU (include/hyobfs.h).
 *
 *   Go (reference)                                     C ABI
 *   -------------------------------------------------  ---------------------------------
 *   WrapPacketConnSalamander(conn, psk)  salamander.go:51-57
 *     + wrapPacketConn(conn, ob)         conn.go:56-71  hyobfs_conn_wrap(fd, ctx, ...)
 *   (*obfsPacketConn).ReadFrom(p)        conn.go:73-88  hyobfs_conn_read_from
 *   (*obfsPacketConn).WriteTo(p, addr)   conn.go:90-99  hyobfs_conn_write_to
 *   (*obfsPacketConn).Close()            conn.go:101-103 hyobfs_conn_close
 *   Set{Read,Write}Deadline              conn.go:109-119 hyobfs_conn_set_{read,write}_deadline
 *   LocalAddr / Set*Buffer / SyscallConn conn.go:105-133 the caller keeps the fd
 *   (new) batched receive / send                        hyobfs_conn_read_batch / _write_batch
 *
 * Reference behaviour kept:
 *   - ReadFrom drops datagrams that do not deobfuscate (len <= 8 or larger than
 *     the caller's buffer) and reads again; a socket error or an empty read
 *     is returned as is (conn.go:77-86).
 *   - WriteTo obfuscates into a 2048-byte buffer (udpBufferSize, conn.go:10); a
 *     payload longer than 2040 bytes makes Obfuscate return 0, the wrapper then
 *     sends an EMPTY datagram and still reports len(p) (conn.go:92-98).
 *   - one read and one write may run concurrently (readMutex/writeMutex).
 * Batched calls move up to `batch` datagrams per recvmmsg/sendmmsg and one GPU
 * batch (pinned rings owned by the connection).
 */
#ifndef HYOBFS_CONN_H
#define HYOBFS_CONN_H

#include <stddef.h>
#include <stdint.h>

#include "hyobfs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* udpBufferSize, conn.go:10: receive/send buffer per datagram */
#define HYOBFS_UDP_BUFFER_SIZE 2048

typedef struct hyobfs_conn hyobfs_conn;

/* one datagram of a batched call; addr is a struct sockaddr_storage */
typedef struct hyobfs_dgram {
    uint8_t* buf;       /* payload (read: destination, write: source) */
    uint32_t len;       /* write: payload length; read: bytes received */
    uint32_t cap;       /* read: capacity of buf */
    uint8_t addr[128];  /* struct sockaddr_storage */
    uint32_t addrlen;
    uint32_t pad_;
} hyobfs_dgram;

/* Wrap a bound UDP socket.  The connection owns fd from here on: hyobfs_conn_close,
   or hyobfs_conn_free on a connection that was not closed, closes it (a binding
   that keeps its own socket passes a dup).  The connection takes a reference on
   ctx (released by hyobfs_conn_free).  batch = the largest number of datagrams per
   batched call (0 = 1024). */
int hyobfs_conn_wrap(int fd, hyobfs_salamander* ctx, uint32_t batch, hyobfs_conn** out);
/* Close() (conn.go:101-103): shuts the connection down but does NOT free it.
   A coalescing connection first sends every datagram write_to accepted; every
   thread blocked in a call on the connection is woken (-1, errno EBADF, as a Go
   ReadFrom returns net.ErrClosed once Close closes the inner conn); close waits
   for them to leave, then closes the socket.  Afterwards every call returns
   -1 / errno EBADF (status calls HYOBFS_ERR_CLOSED), whether it started before
   or after close -- the handle stays valid until hyobfs_conn_free.  A second
   close returns HYOBFS_ERR_CLOSED. */
int hyobfs_conn_close(hyobfs_conn* c);
/* Frees the connection and releases its context reference.  No call on c may
   be in progress or start later (a Go finalizer has exactly that guarantee).
   On a connection that was not closed it shuts down first: the coalescer sends
   what was accepted, its threads stop, and the socket is closed (the fd is the
   connection's, as a Go UDPConn's finalizer closes its own). */
void hyobfs_conn_free(hyobfs_conn* c);

/* ReadFrom: bytes written to p (>= 0), or -1 with errno set (socket error). */
int64_t hyobfs_conn_read_from(hyobfs_conn* c, uint8_t* p, size_t cap, void* addr, uint32_t* addrlen);
/* WriteTo: len on success (also for the empty-datagram quirk), -1 with errno set. */
int64_t hyobfs_conn_write_to(hyobfs_conn* c, const uint8_t* p, size_t len, const void* addr,
                             uint32_t addrlen);
/* Receive up to n datagrams (blocks for the first).  Invalid ones (len <= 8
   or larger than the entry's cap) are dropped, as ReadFrom drops them; an
   empty datagram is returned as an entry with len 0, as ReadFrom returns it
   as a 0-byte read (conn.go:77-80).  Returns the count (>= 0), or -1 with
   errno set. */
int hyobfs_conn_read_batch(hyobfs_conn* c, hyobfs_dgram* msgs, uint32_t n);
/* Obfuscate and send n datagrams with one GPU batch.  Returns the count sent,
   or -1 with errno set. */
int hyobfs_conn_write_batch(hyobfs_conn* c, const hyobfs_dgram* msgs, uint32_t n);

/* SetReadDeadline / SetWriteDeadline (conn.go:109-119, net.Conn semantics): an
   absolute CLOCK_REALTIME time in ns since the Unix epoch (Go: t.UnixNano()),
   0 = no deadline.  It applies to future calls AND to calls blocked right now
   (they re-read it); once passed, read_from / write_to return -1 with errno
   EAGAIN (Go: os.ErrDeadlineExceeded).  A read deadline takes precedence over
   the socket's SO_RCVTIMEO.  SetDeadline = both. */
int hyobfs_conn_set_read_deadline(hyobfs_conn* c, int64_t unix_ns);
int hyobfs_conn_set_write_deadline(hyobfs_conn* c, int64_t unix_ns);

/* Coalescing mode (no reference counterpart: a throughput knob behind the
   unchanged per-datagram surface, conn.go:73-99).  After this call:
     - hyobfs_conn_write_to copies the datagram into the filling batch and
       returns len(p) at once (the > 2040-byte quirk included).  A flusher
       thread seals the batch when it holds max_batch datagrams or max_wait_us
       after its first one, obfuscates it as one GPU batch and sends it with
       sendmmsg while the next batch fills.  Like a UDP sendto, a datagram is
       accepted once queued.  DIVERGENCE from conn.go:93-98 (which returns the
       socket error to the WriteTo whose datagram failed): a send that fails
       after its write_to returned is counted in the stats and its errno is
       returned by the NEXT write_to on the connection (-1, that call's
       datagram not accepted), once.  Salts come from the context's RandSrc
       (hyobfs_salamander_seed / _next_salts), not from a caller-supplied
       source; the wire format is unchanged.  Writers block while both
       batches are busy (backpressure).
     - hyobfs_conn_read_from is served from batches a reader thread receives
       with recvmmsg and deobfuscates as one GPU batch: invalid datagrams are
       dropped and an empty datagram is a 0-byte read, as ReadFrom does; the
       socket's SO_RCVTIMEO bounds the wait (-1, errno EAGAIN).
     - many threads may call write_to / read_from at once; the batched calls
       return -1 with errno EBUSY.
   Latency added per datagram: up to max_wait_us plus one GPU batch.  Call once,
   before the connection is used; hyobfs_conn_close / _free send what was
   accepted (before _close closes the socket), then stop the threads.  A
   write_to that races close is either refused (EBADF) or sent, never
   accepted and dropped. */
int hyobfs_conn_set_coalescing(hyobfs_conn* c, uint32_t max_batch, uint32_t max_wait_us);
/* Blocks until every datagram write_to accepted so far was handed to the socket
   (HYOBFS_ERR_CLOSED after close, which has sent them all). */
int hyobfs_conn_flush(hyobfs_conn* c);
/* Coalescing counters: accepted, tx batches, tx errors, received, rx batches, rx
   dropped (still readable after close). */
int hyobfs_conn_stats(hyobfs_conn* c, uint64_t out[6]);

#ifdef __cplusplus
}
#endif
#endif /* HYOBFS_CONN_H */
