/*
 * ftar_dev.h -- the device layer the host C schedules call (internal to libftar).
 *
 * One ftar_dev per rank process: the HIP device it drives, one non-blocking stream
 * the schedules enqueue on, exportable (IPC) allocations, and the segment kernel.
 * Implemented in ftar_dev_{hip,launch,gate,trace}.cpp + ftar_kernels.hip.  The schedules never see a HIP
 * type: everything crosses this header as plain pointers and sizes.
 */
#ifndef FTAR_DEV_H
#define FTAR_DEV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FDEV_HANDLE_BYTES 64

/* One piece of work of a segment kernel.
 *   FDEV_COPY:   out[i] = x[i]
 *   FDEV_REDUCE: out[i] = x[i] <op> y[i]; x has the MPI "inout" role and y the "in"
 *                role of MPI_Reduce_local(in=y, inout=x) (matters only for MAX/MIN
 *                with NaN or signed zeros; SUM/PROD are commutative bit for bit).
 * `out` may alias `x` (in-place reduce).  Pointers may be peer (xGMI) mappings. */
#define FDEV_COPY 0
#define FDEV_REDUCE 1

#define FDEV_REMOTE_X 1
#define FDEV_REMOTE_Y 2
#define FDEV_REMOTE_OUT 4 /* `out` is a peer mapping (a push: remote stores) */

typedef struct {
    int kind;
    int remote;       /* FDEV_REMOTE_* bits, for the byte accounting only */
    void *out;
    const void *x;
    const void *y;
    size_t n;         /* elements */
    void *out2;       /* optional second destination receiving the same values (local) */
} fdev_seg;

#define FDEV_MAX_SEGS 16 /* a relayed exchange step: 2 own pulls + 2 x 6 relay duties */

/* kernel tags (profiling buckets) */
#define FDEV_TAG_LOCAL 0   /* local copies */
#define FDEV_TAG_STEP0 1   /* dominant exchange kernel: Raben RS step 0 / RD step */
#define FDEV_TAG_STEP 2    /* other exchange kernels */
#define FDEV_TAG_RECOV 3   /* recovery transfers */
#define FDEV_TAG_BG 4      /* background stream (Raben step-0 redundancy copy) */
#define FDEV_NTAGS 5

typedef struct ftar_dev ftar_dev;

typedef struct {
    double ms[FDEV_NTAGS];      /* device time per tag (profiling on) */
    int launches[FDEV_NTAGS];
    double link_bytes;          /* bytes read through peer mappings */
    double hbm_bytes;           /* algorithmic local HBM bytes */
} fdev_counters;

int fdev_device_count(int *n);
int fdev_open(int device, ftar_dev **out);
void fdev_close(ftar_dev *d);
int fdev_device(const ftar_dev *d);
/* The device's physical identity (its PCI bus id, "dddd:bb:dd.f"): equal only for the same
 * GPU, whatever HIP ordinal each process's visibility mask gives it. */
int fdev_physical_id(ftar_dev *d, char *out, size_t n);

int fdev_alloc_shared(ftar_dev *d, size_t bytes, void **ptr, void *handle /* FDEV_HANDLE_BYTES */);
/* blocks fdev_alloc_shared had to re-allocate because their IPC export was refused */
int fdev_export_retries(const ftar_dev *d);
int fdev_free(ftar_dev *d, void *ptr);
int fdev_import(ftar_dev *d, const void *handle, void **ptr);
/* Export the device allocation holding [ptr, ptr + bytes): its IPC handle, a per-process
 * unique allocation id (a freed and re-used address gets a new one) and ptr's offset in
 * it; handle NULL: the id and offset only, nothing exported.  Nonzero if the memory
 * cannot be shared (the caller then stages it). */
int fdev_export_range(ftar_dev *d, const void *ptr, size_t bytes, void *handle, uint64_t *id, size_t *offset);
/* Map host memory [p, p + bytes) -- page-aligned, possibly shared with other processes (the
 * control block's flag page) -- into this device's address space; *devp: the address its
 * kernels use.  fdev_host_unmap undoes it.  Host-sim: the address itself. */
int fdev_host_map(ftar_dev *d, void *p, size_t bytes, void **devp);
void fdev_host_unmap(ftar_dev *d, void *p);
int fdev_unimport(ftar_dev *d, void *ptr);
/* 0 if the device can access [ptr, ptr + bytes): this device's memory inside one
 * allocation, pinned host memory mapped at its own address, or managed memory; nonzero
 * for pageable host memory, another GPU's memory, host memory mapped elsewhere, or a
 * range past the end of its allocation (the device entry points refuse those instead of
 * faulting). */
int fdev_check_ptr(ftar_dev *d, const void *ptr, size_t bytes);
/* 1 if `ptr` is pinned host memory mapped into the device at its own address (the
 * kernels can read and write it in place over PCIe) */
int fdev_host_pinned(const void *ptr);

/* Enqueue one segment kernel on the rank's stream. */
int fdev_run(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag);
/* Tree reduce of nsrc (2, 4, 8 or 16) sources into out on the rank's stream:
 * out[i] = ((src0 op src1) op (src2 op src3)) op ...; bit j of remote_mask marks src[j]
 * as a peer mapping (byte accounting). */
#define FDEV_MAX_TREE 16
int fdev_tree(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, unsigned remote_mask, void *out,
              size_t n, int tag);
/* The same tree, its result also stored to `nmore` (<= 7) further destinations: peer
 * mappings when `more_remote` (the push mesh's allgather: the owner's block into every peer),
 * else this device's memory (the caller's rbuf; byte accounting only). */
int fdev_tree_out(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, unsigned remote_mask, void *out,
                  void *const *more, int nmore, int more_remote, size_t n, int tag);
/* ntree (<= FDEV_MAX_BATCH) trees of nsrc (2, 4 or 8) sources in ONE launch: tree t
 * reduces src[t * nsrc + j], j < nsrc, into out[t] over n[t] elements (remote_mask[t] as
 * in fdev_tree).  Meant for small vectors: a tree beyond the device's workgroup budget
 * makes it one launch per tree (same result). */
#define FDEV_MAX_BATCH 8
int fdev_tree_batch(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, const unsigned *remote_mask,
                    void *const *out, const size_t *n, int ntree, int tag);
/* The same batch queued AHEAD of the barrier that makes its operands ready: the launch's
 * workgroups wait on a gate word in pinned host memory until fdev_gate_open (go: they
 * run; skip: they return without touching memory), so the launch latency overlaps the
 * wait for the peers.  Only a short signalled launch can be gated, and only when every
 * launch queued since the last drain signalled (a fenced marker would wait behind the
 * closed gate): *gated = 0 and nothing is queued otherwise (and with kernel timing on).
 * Until the gate opens, fdev_sync waits for the launches queued BEFORE it only. */
int fdev_tree_batch_gated(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc,
                          const unsigned *remote_mask, void *const *out, const size_t *n, int ntree, int tag,
                          int *gated);
/* The same, with this rank's staging copy folded in ahead of the gate: the launch first
 * copies stage_n elements from stage_src to stage_dst (all of it, whatever the gate
 * says) and signals that; the drain before the barrier waits for that signal. */
int fdev_tree_batch_staged_gated(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc,
                                 const unsigned *remote_mask, void *const *out, const size_t *n, int ntree, int tag,
                                 void *stage_dst, const void *stage_src, size_t stage_n, int *gated);
/* fdev_run's segment kernel queued behind a gate, on the same terms (stage_dst != NULL:
 * with the staging phase folded in, as fdev_tree_batch_staged_gated). */
int fdev_run_gated(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag, void *stage_dst,
                   const void *stage_src, size_t stage_n, int *gated);
/* Open the pending gate (no-op without one).  skip = 1: the gated launch does nothing.
 * Any other launch or stream wait queued while a gate is pending opens it as skip first
 * (nothing may wait behind a closed gate): a caller about to open its gate checks
 * fdev_gate_pending and relaunches if the gated launch was given up.
 * A gate the DEVICE gave up on (still closed after FTAR_GATE_TIMEOUT_MS of its wall clock:
 * the workgroups returned without touching memory) is caught by the next fdev_sync, which
 * relaunches the same plan ungated and drains it (fdev_gate_relaunches counts them). */
int fdev_gate_open(ftar_dev *d, int skip);

/* Device-side order between ranks (the mesh allgather behind the peers' reduce-scatter, with
 * no host barrier between them).  fdev_peer_wait queues, on the main stream: a
 * fenced marker (everything queued so far released to HBM device-wide, this GPU's caches
 * invalidated), then a one-wavefront kernel that stores `token` into `flag` -- this rank's
 * line of the job's flag page, host memory every rank's GPU maps (fdev_host_map) -- and waits
 * until every peer's flag holds `token`.  The NEXT launch on the main stream runs only if that
 * wait succeeded: when the host gives it up (fdev_peer_wait_abort: a peer died), or it times
 * out (FTAR_GATE_TIMEOUT_MS), its workgroups return untouched, and after the drain
 * fdev_peer_wait_verdict returns 0.  Host-sim: the wait spins on the host, calling `poll`
 * (which may call fdev_peer_wait_abort); the GPU build ignores poll (the drain's poll does
 * that).  Tokens only grow: a flag holding a later token satisfies an earlier wait. */
#define FDEV_MAX_PEERS 15
int fdev_peer_wait(ftar_dev *d, void *flag, void *const *peer_flags, int npeers, uint64_t token,
                   int (*poll)(void *), void *arg);
void fdev_peer_wait_abort(ftar_dev *d);
/* after the drain of the launch behind the wait: 1 it ran (or none was armed), 0 it was skipped */
int fdev_peer_wait_verdict(ftar_dev *d);
/* 1 while a gated launch waits for its gate. */
int fdev_gate_pending(const ftar_dev *d);
int fdev_gate_relaunches(const ftar_dev *d);
/* Per-rank knobs of the device layer (not collective). */
#define FDEV_KNOB_FLAG_SYNC 0   /* 0/1: short launches signal their completion (off: fenced markers, no gates) */
#define FDEV_KNOB_TREE_UNROLL 1 /* 1, 2, 4: vectors per lane and source in fdev_tree at 4 / 8 sources */
int fdev_set_knob(ftar_dev *d, int knob, int value);
int fdev_get_knob(const ftar_dev *d, int knob);
/* Enqueue on the rank's background stream, ordered after everything queued so far on
 * the main stream (it then overlaps later main-stream work). */
int fdev_run_bg(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag);
/* Runtime copy (hipMemcpyAsync: SDMA / blit engine) of `bytes` on the main (bg = 0) or
 * background (bg = 1) stream; `remote` = the source is a peer mapping. */
int fdev_copy(ftar_dev *d, int bg, void *dst, const void *src, size_t bytes, int remote, int tag);
/* Spin until the background stream drained. */
int fdev_sync_bg(ftar_dev *d, int (*poll)(void *), void *arg);
/* Order the rank's work after everything queued on `user_stream` (hipStream_t): nothing to
 * do if it is idle, else the host waits for it (never a marker queued on the caller's
 * stream).  fdev_user_host_waits counts the calls that waited. */
int fdev_order_after(ftar_dev *d, void *user_stream);
int fdev_user_host_waits(const ftar_dev *d);
/* Spin (busy, the process stays in R state) until the stream drained.  `poll` is
 * called between queries; a nonzero return aborts the wait with that value. */
int fdev_sync(ftar_dev *d, int (*poll)(void *), void *arg);
/* The next fdev_sync must be a fenced marker even if only signalled launches were queued:
 * peers are about to read memory the caller wrote (its send buffer, read in place). */
void fdev_fence_next_drain(ftar_dev *d);
/* 1 while work queued on the rank's stream has not completed (kill-point diagnostics). */
int fdev_busy(ftar_dev *d);

int fdev_h2d(ftar_dev *d, void *dst, const void *src, size_t bytes);
int fdev_d2h(ftar_dev *d, void *dst, const void *src, size_t bytes);
/* Host-buffer pipeline: chunk copies on their own streams (created on first use).
 * fdev_h2d_async lands chunk `slot` (< FDEV_MAX_CHUNKS) and marks it with a fenced event;
 * fdev_wait_h2d spins until it landed (visible to peers); fdev_d2h_async copies after
 * everything queued on the rank's stream so far; fdev_sync_d2h waits for all of them. */
#define FDEV_MAX_CHUNKS 16
int fdev_h2d_async(ftar_dev *d, void *dst, const void *src, size_t bytes, int slot);
int fdev_wait_h2d(ftar_dev *d, int slot, int (*poll)(void *), void *arg);
int fdev_d2h_async(ftar_dev *d, void *dst, const void *src, size_t bytes);
int fdev_sync_d2h(ftar_dev *d, int (*poll)(void *), void *arg);
int fdev_alloc_plain(ftar_dev *d, size_t bytes, void **ptr);

void fdev_profiling(ftar_dev *d, int on);
void fdev_counters_reset(ftar_dev *d);
void fdev_counters_get(ftar_dev *d, fdev_counters *out);

/* FTAR_TRACE (test instrumentation; tests/fence_check.py): a per-rank log of every launch with
 * the registered regions it reads and writes and its system-scope release / acquire, every
 * fenced marker, drain, gate verdict, and the barrier arrivals the schedules note.  Nothing is
 * logged (and nothing costs anything) unless fdev_trace_open was called. */
int fdev_trace_open(ftar_dev *d, const char *path);
/* name [base, base + bytes) as buffer `name` of original rank `owner` (own or peer mapping) */
void fdev_trace_region(ftar_dev *d, const void *base, size_t bytes, int owner, const char *name);
void fdev_trace_unregion(ftar_dev *d, const void *base);
/* memory this rank's launches did not write but the caller did (an exported send buffer) */
void fdev_trace_external_write(ftar_dev *d, const void *p, size_t bytes);
void fdev_trace_note(ftar_dev *d, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

/* Standalone local reduce on a caller stream (MPI_Reduce_local). */
int fdev_reduce_local(const void *in, void *inout, size_t n, int dtype, int op, void *stream);
int fdev_set_reduce_variant(int v);

const char *fdev_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
