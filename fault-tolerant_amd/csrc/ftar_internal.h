/*
 * ftar_internal.h -- the communicator and helpers shared by the two schedules.
 */
#ifndef FTAR_INTERNAL_H
#define FTAR_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "../../include/ftar.h"
#include "ftar_ctrl.h"
#include "ftar_dev.h"

/* workspace buffers (exported to every peer) */
#define WS_IN 0  /* this rank's input vector (Raben: after the pre-step) */
#define WS_W 1   /* accumulator: Raben rbuf, RD ping-pong A */
#define WS_T 2   /* Raben tmp (step-0 redundancy copy), RD ping-pong B */
#define WS_R 3   /* relay staging: stripes this rank forwards for other ranks */
/* the caller's buffers of the current call: never exported, so only the rank itself
 * names them (a plan's x_buf / dst_buf, resolved by ftar_local) */
#define WS_UIN 4  /* sbuf / src */
#define WS_UOUT 5 /* rbuf / dst */


struct ftar_comm {
    ftar_job job;
    int wrank, wsize; /* original rank / size (Data.original_rank/_size) */
    int device;
    ftar_dev *dev;
    void *user_stream;

    /* current communicator: comm rank -> original rank */
    int order[FTAR_MAX_RANKS];
    int size;
    uint64_t members; /* survivors (bit per original rank) */
    uint64_t acked;   /* failures already acknowledged (MPIX_Comm_failure_ack) */

    ftar_kill kills[FTAR_MAX_KILLS];
    int kill_call[FTAR_MAX_KILLS]; /* call index the kill applies to, -1 = every call */
    int nkills;
    int ncalls; /* allreduce calls started on this rank */

    /* exported workspace and the peers' mappings of theirs */
    void *ws[FTAR_NBUF];
    size_t ws_bytes;
    void *peer[FTAR_MAX_RANKS][FTAR_NBUF];
    size_t peer_bytes[FTAR_MAX_RANKS];
    uint64_t peer_gen[FTAR_MAX_RANKS]; /* the peer's ws_gen our mappings of its workspace belong to */

    const void *uin; /* the current call's buffers (WS_UIN / WS_UOUT) */
    void *uout;
    /* peers' exported send buffers (mesh Raben reads them in place): up to FTAR_UCACHE
     * mappings per peer, keyed by the peer's allocation id.  Every rank keeps the same cache
     * of its OWN allocations (xcache: the mirror of what each peer holds of it), so the
     * exporter knows without a round trip whether its peers hold this call's send buffer: a
     * hit is read in place, a miss with a free slot is exported and mapped, a miss in a full
     * cache is staged in IN (a local copy) -- a caller cycling through more send buffers than
     * the cache holds never closes and re-opens mappings call after call (0.4 ms per close,
     * tools/ipc_probe.hip).  Entries stay until finalize (or the exporter's death): the runtime
     * refused to re-open a mapping of an allocation this process had closed before (round 6,
     * 4 and 8 ranks, "invalid device pointer"), so a mapping, once made, is never closed and
     * re-made; a freed send buffer's memory stays allocated until then. */
#define FTAR_UCACHE 8
    struct {
        uint64_t id;
        void *base;
        uint64_t last; /* the call that last used it */
    } ucache[FTAR_MAX_RANKS][FTAR_UCACHE];
    struct {
        uint64_t id, last;
    } xcache[FTAR_UCACHE];
    /* this call's IN: the caller's exported sbuf itself (in_alias) or the staged copy;
     * peer_in[w] likewise for every peer (NULL: its staged IN) -- see ftar_buf */
    const void *in_alias;
    size_t in_bytes;
    void *peer_in[FTAR_MAX_RANKS];
    int export_user;     /* FTAR_EXPORT (default 1): let peers read sbuf in place where possible */
    size_t stage_max;    /* FTAR_STAGE_MAX bytes: inputs up to this size are staged, never read in place */
    int host_pipe;       /* FTAR_HOST_PIPE (default 1): chunk-pipelined host-buffer Raben where it applies */

    /* host staging for the _host entry points */
    void *hsend, *hrecv;
    size_t hbytes;

    int64_t pubval; /* value published at every sync (RD: accumulator buffer id) */

    int profiling;
    ftar_stats stats;
    double t0; /* start of the current user call (ftar_stats_begin) */
    void *pwflag_dev; /* the control block's flag page as this rank's GPU maps it (fdev_host_map) */
    int chunk_cont; /* the host pipeline's chunks 2..n of one user call (see ftar_stats_begin) */
    int verbose;
    int overlap;         /* FTAR_OVERLAP (default 1): Raben step-0 redundancy copy on the background stream */
    int relay;           /* FTAR_RELAY (default 1): stripe exchanges over 2-hop paths */
    size_t relay_min;    /* FTAR_RELAY_MIN bytes: smallest per-rank window that is relayed */
    int copy_engine;     /* FTAR_COPY_ENGINE (default 0): direct pulls by hipMemcpyAsync */
    int redundancy;      /* FTAR_REDUNDANCY: 2 auto (default: the step-0 copy moves where a spare exists and the
                            comm spans GPUs), 1 always, 0 never (a replay reads the dead rank's IN) */
    int mesh;            /* FTAR_MESH (default 1): one-hop Raben at power-of-two p without a spare */
    int push;            /* FTAR_PUSH (default 0): the mesh by remote stores -- 1 reduce-scatter, 2 both phases */
    int mesh_wait;       /* FTAR_MESH_WAIT (default 1): the mesh's allgather ordered behind the peers' trees on the device */
    double watch_t;      /* ftar_watch_peers: when the members were last checked for deaths */
    int gate;            /* FTAR_GATE (default 1): small exchange launches queued ahead of their barrier, gated */
    double gate_hold_s;  /* FTAR_GATE_HOLD_US: a barrier waiting longer gives the pending gated launch up (0 = never) */
    size_t gate_max;     /* FTAR_GATE_MAX bytes (default 1 MiB): largest vector whose launches are queued ahead */
    size_t oneshot_max;  /* FTAR_ONESHOT_MAX bytes: mesh Raben in one launch up to this size */
    double loop_seconds; /* FTAR_LOOP_SECONDS: stretch the tolerant step loop to this long (harness knob) */
    /* the step's last peer read (FTAR_LOOP_SECONDS re-pulls it into pad while it waits) */
    const void *pad_src;
    size_t pad_bytes;
    void *pad; /* local scratch of FTAR_PAD_BYTES, allocated on the first padded step */
    /* A segment launch queued behind a gate (ftar_prelaunch): the segments it was planned
     * with, to be compared with the step's own when it comes (ftar_run_gated_or). */
    struct ftar_gplan {
        int valid, dtype, op, tag, nseg;
        fdev_seg segs[FDEV_MAX_SEGS];
    } gplan;
    /* the next step's predicted segments: ftar_xfer_step queues them gated right behind
     * the current step's launch (set by the schedule, consumed by the transport) */
    struct ftar_gplan gnext;
};

#define FTAR_PAD_BYTES ((size_t)16 << 20)

size_t ftar_esize(int dtype);
int ftar_check_op(int dtype, int op);
int ftar_my_comm_rank(const ftar_comm *c);
int ftar_comm_rank_of(const ftar_comm *c, int w);

/* collective: grow the _host entry points' staging to `bytes` (aborts the job on failure) */
int ftar_ensure_staging(ftar_comm *c, size_t bytes);
/* collective: grow the exported workspace to hold `bytes` per buffer */
int ftar_ensure_workspace(ftar_comm *c, size_t bytes);
/* the device-wait flag of original rank w: its line of the control block's flag page, as this
 * rank's GPU addresses it (NULL: the page is not mapped, the mesh orders on the host) */
void *ftar_flag(ftar_comm *c, int w);
/* fdev_sync's poll while a launch waits on the device for the peers (fdev_peer_wait): the
 * failure detector, and a dead member gives the wait up (fdev_peer_wait_abort) */
int ftar_watch_peers(void *arg);
int ftar_drain_watch(ftar_comm *c);
/* pointer to buffer b of original rank w (own or peer mapping) */
void *ftar_buf(ftar_comm *c, int w, int b);
/* this rank's buffer b: a workspace buffer or the call's WS_UIN / WS_UOUT */
void *ftar_local(ftar_comm *c, int b);
/* Every call, before its first barrier: let IN be the caller's sbuf itself (exported to
 * the peers, returns 1) when `alias_ok` and the memory can be shared, else publish that
 * the peers read the staged copy the caller then makes (returns 0). */
int ftar_stage_input(ftar_comm *c, const void *sbuf, size_t bytes, int alias_ok);
/* After the call's first barrier: map the peers' exported inputs (ftar_buf(w, WS_IN)). */
void ftar_resolve_inputs(ftar_comm *c);
/* End of a call: IN is the workspace buffer again everywhere. */
void ftar_inputs_done(ftar_comm *c);
/* This call's input of original rank w as peers may read it after w died: w's exported
 * sbuf mapping or its staged IN, only if w published it for THIS call and our mapping
 * belongs to w's current workspace generation and covers `bytes`; NULL otherwise. */
const void *ftar_dead_input(ftar_comm *c, int w, size_t bytes);

/* agree over the survivors; returns newly failed original ranks (not yet acked) */
uint64_t ftar_sync(ftar_comm *c);
/* the per-step agree of a schedule loop; `nsteps` = steps of the loop (spreads the
 * FTAR_LOOP_SECONDS harness delay over them) */
uint64_t ftar_step_sync(ftar_comm *c, int nsteps);
/* value original rank w published before the last completed sync */
int64_t ftar_peer_pub(ftar_comm *c, int w);
/* the same, or 0 (no *v) for a rank that died before publishing it */
int ftar_peer_pub_try(ftar_comm *c, int w, int64_t *v);
/* agree outside the tolerant region: any new failure aborts the job */
void ftar_sync_fatal(ftar_comm *c);
/* drain the device stream (busy wait, abort-aware) */
void ftar_host_copy_failed(ftar_comm *c, const char *what); /* aborts the job */
int ftar_drain(ftar_comm *c);
/* enqueue one segment kernel */
int ftar_run(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag);
/* Queue a step's segment launch ahead of the barrier that readies its operands, behind a
 * gate (fdev_run_gated); returns 1 if it was queued.  ftar_run_gated_or runs a step's
 * segments: it opens the pending gate if that launch was planned with exactly these
 * segments, else gives it up (skip) and launches them. */
int ftar_prelaunch(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag, void *stage_dst,
                   const void *stage_src, size_t stage_n);
void ftar_run_gated_or(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag);
/* bookkeeping of every launch: the control slot's in-flight word (FTAR_INFLIGHT_*) and,
 * for a peer read (`remote` != NULL, `bytes` of it), the step's re-pull source */
void ftar_note_launch(ftar_comm *c, const void *remote, size_t bytes);
/* enqueue on the background stream (after the main stream's current work) */
int ftar_run_bg(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag);
int ftar_drain_bg(ftar_comm *c);
int ftar_is_dead(ftar_comm *c, int w);
/* 1 if the comm's members drive more than one GPU (uniform: the same on every member) */
int ftar_spans_devices(const ftar_comm *c);
/* Exchange entry (see ftar_ctrl_enter): a partner's exchange failed iff it died before
 * entering it -- what the reference's failed Sendrecv means -- independent of when the
 * death is noticed (a rank that dies after its exchange point is still read). */
void ftar_enter(ftar_comm *c);
int ftar_peer_entered(ftar_comm *c, int w);
/* After this rank has queued its pulls of the step it entered (before draining them):
 * publish that, then pass the FTAR_PT_DURING kill point of (phase, step). */
void ftar_launched(ftar_comm *c, int phase, int step);
/* After the step's pulls drained: this rank's side of the exchange completed. */
void ftar_exchange_done(ftar_comm *c);
/* The reference's Sendrecv with original rank w failed (0) iff w died before completing
 * its side of the exchange -- mid-transfer included (FTAR_PT_DURING). */
int ftar_peer_done(ftar_comm *c, int w);

/* the whole call on a comm of one rank (both schedules): copy, drain, closing barrier */
int ftar_single_rank(ftar_comm *c, const void *sbuf, void *rbuf, size_t bytes);

/* deterministic fault injection at (phase, step, point) */
void ftar_maybe_die(ftar_comm *c, int phase, int step, int point);

/* remove `dead` (comm rank), moving the entry at comm rank `repl` into its place */
void ftar_regroup(ftar_comm *c, int dead, int repl);
/* drop failed ranks from the survivor world keeping the order */
void ftar_shrink(ftar_comm *c, uint64_t failed);

void ftar_stats_begin(ftar_comm *c);
void ftar_stats_end(ftar_comm *c);

/* ---- exchange transport (ftar_xfer.c) ------------------------------------
 * One exchange step of a schedule, described for EVERY receiving rank so each rank
 * can work out its relay duties.  A pull moves a window [off, off+n) of buffer src_buf
 * of original rank `src` into buffer dst_buf of the receiver (COPY), or reduces it
 * with the receiver's x_buf window (REDUCE; `swap` puts the pulled operand first). */
typedef struct {
    int kind, swap;
    int src, src_buf;
    int dst_buf, x_buf;
    int64_t off, n;
    int to_uout; /* also store the result in the caller's output buffer (same offset) */
} ftar_pull;

#define FTAR_MAX_PULLS 2
typedef struct {
    int npull[FTAR_MAX_RANKS];                   /* by comm rank; 0 = not receiving */
    ftar_pull pull[FTAR_MAX_RANKS][FTAR_MAX_PULLS];
} ftar_plan;

typedef struct {
    int relayed;       /* the step used 2-hop relays */
    int skipped;       /* this rank did not pull (its source was dead at the start) */
    uint64_t mid_dead; /* failures seen at the mid-step barrier (uniform) */
    int missing;       /* this rank lost stripes of relays that died before the barrier */
} ftar_xstate;

void ftar_plan_clear(ftar_plan *p);
/* phase 1 (+ mid barrier + phase 2 when relayed); `skip` = this rank's source is dead;
 * (kphase, kstep) place the FTAR_PT_AFTER injection point after phase 1 */
/* Launch a direct step's pull segments: one segment kernel, or with copy_engine the
 * runtime copy engine for every remote operand (reduces staged through R). */
void ftar_run_pulls(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag, int bg);
/* `extra` local segments (no peer reads) ride along in the step's first launch, even
 * when this rank's pulls are skipped */
void ftar_xfer_step(ftar_comm *c, const ftar_plan *p, int dtype, int op, int tag, int skip, int kphase, int kstep,
                    const fdev_seg *extra, int nextra, ftar_xstate *st);
/* after the step's agree returned `known`: re-pull stripes lost with relays that died
 * before the mid barrier, then one more (uniform) barrier */
void ftar_xfer_repair(ftar_comm *c, const ftar_plan *p, int dtype, int op, ftar_xstate *st, uint64_t known);
/* the segments of this rank's direct pulls in plan p, appended to segs[ns..]; returns ns */
int ftar_xfer_direct_segs(ftar_comm *c, const ftar_plan *p, size_t es, fdev_seg *segs, int ns);
double ftar_link_bytes(ftar_comm *c);
int ftar_xfer_would_relay(ftar_comm *c, const ftar_plan *p, size_t es);

int ftar_hibit(int value, int start);
int ftar_floor_pow2(int n);

#define FTAR_CHECK(x)                                                                                       \
    do {                                                                                                    \
        int _rc = (x);                                                                                      \
        if (_rc) return _rc;                                                                                \
    } while (0)

#endif
