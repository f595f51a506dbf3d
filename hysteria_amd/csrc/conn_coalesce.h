// conn_coalesce.h -- private: the batching engine behind the per-datagram
// WriteTo / ReadFrom of a coalescing hyobfs_conn (include/hyobfs_conn.h,
// hyobfs_conn_set_coalescing).  Not installed.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <atomic>

#include "../../include/hyobfs.h"

namespace hyobfs {

struct Coalescer;

// Absolute deadlines of a connection (CLOCK_REALTIME ns since the epoch, 0 = none),
// owned by the connection: SetReadDeadline / SetWriteDeadline.
struct Deadlines {
    std::atomic<int64_t> read{0}, write{0};
};
int64_t realtime_ns();

// Context lifetime (hyobfs_api.cpp): a connection retains its context, so
// hyobfs_salamander_free (a Go finalizer, say) never frees it under a live
// connection; the last release destroys it.
void ctx_retain(hyobfs_salamander* ctx);
void ctx_release(hyobfs_salamander* ctx);

// Asynchronous batches for the coalescer (hyobfs_api.cpp): a stream and an event on
// the context's device.  The coalescer's staging is mapped pinned host memory
// (hyobfs_host_alloc), which the kernels read and write in place, so a batch is one
// kernel launch on the coalescer's stream (hyobfs_salamander_*_batch) and a later
// wait on the event recorded behind it: the host works on the previous batch (its
// sendmmsg, or handing it to readers) while the GPU runs this one.
struct GpuQueue;
GpuQueue* gpu_queue_new(hyobfs_salamander* ctx);
void gpu_queue_free(GpuQueue* g);
// Launches the batch on the queue's stream and records event `slot` (0..3) behind it.
int gpu_queue_submit(GpuQueue* g, const hyobfs_batch* b, bool obfuscate, int slot);
// Waits for event `slot`: the batch submitted with it is done (and its output visible).
int gpu_queue_wait(GpuQueue* g, int slot);

// Starts the flusher and reader threads on fd.  nullptr on allocation failure.
Coalescer* coalescer_new(int fd, hyobfs_salamander* ctx, uint32_t max_batch, uint32_t max_wait_us,
                         const Deadlines* dl);
// Wakes blocked callers so they re-read the deadlines (after a change).
void coalescer_poke(Coalescer* q);
// Sends what was accepted, wakes blocked callers (-1, EBADF), stops the threads.
void coalescer_stop(Coalescer* q);
// coalescer_stop, then frees everything (not the fd) once no caller is inside.
void coalescer_free(Coalescer* q);
// WriteTo: accepted datagrams return len (also > 2040: the empty-datagram quirk);
// -1 with the errno of an earlier datagram whose send failed (reported once).
int64_t coalescer_write(Coalescer* q, const uint8_t* p, size_t len, const void* addr, uint32_t addrlen);
// ReadFrom: bytes written to p, or -1 with errno (EAGAIN on the socket's receive timeout).
int64_t coalescer_read(Coalescer* q, uint8_t* p, size_t cap, void* addr, uint32_t* addrlen);
// Blocks until every datagram accepted so far has been handed to the socket.
int coalescer_flush(Coalescer* q);
void coalescer_stats(const Coalescer* q, uint64_t out[6]);

}  // namespace hyobfs
