// conn_coalesce.h -- private: the batching engine behind the per-datagram
// WriteTo / ReadFrom of a coalescing hyobfs_conn (include/hyobfs_conn.h,
// hyobfs_conn_set_coalescing).  Not installed.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/hyobfs.h"

namespace hyobfs {

struct Coalescer;

// Starts the flusher and reader threads on fd.  nullptr on allocation failure.
Coalescer* coalescer_new(int fd, hyobfs_salamander* ctx, uint32_t max_batch, uint32_t max_wait_us);
// Sends what was accepted, stops the threads, frees everything (not the fd).
void coalescer_free(Coalescer* q);
// WriteTo: accepted datagrams return len (also > 2040: the empty-datagram quirk).
int64_t coalescer_write(Coalescer* q, const uint8_t* p, size_t len, const void* addr, uint32_t addrlen);
// ReadFrom: bytes written to p, or -1 with errno (EAGAIN on the socket's receive timeout).
int64_t coalescer_read(Coalescer* q, uint8_t* p, size_t cap, void* addr, uint32_t* addrlen);
// Blocks until every datagram accepted so far has been handed to the socket.
int coalescer_flush(Coalescer* q);
void coalescer_stats(const Coalescer* q, uint64_t out[6]);

}  // namespace hyobfs
