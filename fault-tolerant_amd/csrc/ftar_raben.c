/*
 * ftar_raben.c -- fault-tolerant Rabenseifner Allreduce on MI355X (per rank, host C).
 *
 * Restates src/raben/rabenseifner.c:3-395 and src/raben/errhandler.c:3-468 for ranks
 * that own one GPU each.  Every MPI_Sendrecv + MPI_Reduce_local pair becomes ONE
 * receiver-driven kernel that reads the partner's window straight out of its HBM
 * over xGMI (IPC peer mapping) and reduces it into the local window:
 *
 *   RS step 0 (:206-211 full exchange + :231-237 reduce):
 *       A0[rw0] = IN[rw0] + peer.IN[rw0]       (reduce half)
 *       T[sw0] = peer.IN[sw0]                  (redundancy copy, where a spare can use it:
 *                                               a replay otherwise reads peer.IN itself)
 *   RS step k>=1 (:219-237):  Ak[rwk] = A(k-1)[rwk] + peer.A(k-1)[rwk]
 *   AG step k (:299-315):     W[swk] = peer.W[swk]
 * The accumulators Ak are W, except with an idle spare, where the steps alternate W and T's
 * free half (rb_acc) so that no step overwrites its own input: a partner that dies
 * mid-exchange costs no pre-image (see the reduce-scatter loop).
 *
 * Buffers (exported workspace, ftar_internal.h): IN = this rank's vector after the
 * pre-step (the reference's sbuf after :128), W = rbuf, T = tmp_buf.  The reference's
 * tmp also stages the step>=1 windows; here those are fused into the reduce, which
 * leaves T holding the partner's vector where recovery reads it (:191-197).
 * No rank ever writes a window a peer reads in the same step, and each step ends at
 * the agree+barrier of the reference (:258-260, :330-332), so pulls need no locks.
 *
 * Deviations: sbuf is never written (IN is a private shadow); the
 * impersonator accumulates the dead rank's replay in W's half it does not own yet,
 * not in sbuf/tmp, so a second impersonation by the same rank stays correct; a
 * recovery that needs redundancy a replacement rank never received aborts instead of
 * replaying garbage; new_entry pulls only the dead rank's live window.
 */
#include "ftar_internal.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define MAXSTEPS 32
/* host-buffer pipeline: vectors of at least HOST_PIPE_MIN bytes go through in chunks of
 * HOST_PIPE_CHUNK bytes (at most HOST_PIPE_MAX chunks, FDEV_MAX_CHUNKS) */
#define HOST_PIPE_MIN ((size_t)16 << 20)
#define HOST_PIPE_CHUNK ((size_t)8 << 20)
#define HOST_PIPE_MAX 16

typedef struct {
    ftar_comm *c;
    int dtype, op;
    size_t es, count;
    int steps, adjsize, rem;
    int rank, vrank, corr, has_recov;
    int keep_recov; /* step 0 also pulls the partner's other half into T (recovery data) */
    int alt;        /* RS accumulators alternate W / T (an idle spare at the call's start; rb_acc) */
    int bg_pending; /* step-0 redundancy copy still running on the background stream */
    int fast_io;    /* power of two, no recovery data: sbuf/rbuf used in place (see below) */
    int out_done;   /* the last allgather step already stored this rank's result in rbuf */
    int mesh;       /* fast_io on the full mesh: one-hop reduce-scatter and allgather */
    int push;       /* the mesh's reduce-scatter by remote stores into the owners' R (FTAR_OPT_PUSH) */
    int64_t slot;   /* push: elements per source slot in an owner's R */
    int oneshot;    /* mesh of a small vector: every block in its owner's tree, one launch */
    int own_in_rbuf; /* the mesh's tree stored this rank's final block in rbuf too: the allgather skips it */
    int io_safe;     /* sbuf == rbuf or the two do not overlap: rbuf may be written while peers read sbuf */
    int devwait;     /* the mesh's allgather ordered behind the peers' trees on the device (rb_mesh_devwait) */
    /* the one-shot launch queued ahead of the barrier (rb_oneshot_prelaunch): its plan, to
     * be checked against the one the inputs' resolution gives */
    int gated;
    struct rb_batch {
        const void *src[FDEV_MAX_BATCH * FDEV_MAX_BATCH];
        void *out[FDEV_MAX_BATCH];
        size_t n[FDEV_MAX_BATCH];
        unsigned remote[FDEV_MAX_BATCH];
    } gplan;
    int in0_w[FTAR_MAX_RANKS]; /* world rank whose IN held vrank v's input at RS step 0 */
    int64_t rindex[MAXSTEPS], sindex[MAXSTEPS], rcount[MAXSTEPS], scount[MAXSTEPS];
} rb_ctx;

static int rb_real(const rb_ctx *x, int v) { return (v < x->rem) ? v * 2 : v + x->rem; }

static void rb_vrank(rb_ctx *x)
{
    x->rank = ftar_my_comm_rank(x->c);
    if (x->rank < 2 * x->rem) x->vrank = (x->rank % 2 == 0) ? x->rank / 2 : -1;
    else x->vrank = x->rank - x->rem;
}

/* Windows of virtual rank v at every step (raben/rabenseifner.c:170-249).  The
 * reference compares real ranks (rank < dest); the vrank->rank map is monotone, so
 * that is bit s of v being 0. */
static void rb_windows(int v, size_t count, int steps, int64_t *rindex, int64_t *sindex, int64_t *rcount,
                       int64_t *scount)
{
    int64_t wsize = (int64_t)count;
    rindex[0] = sindex[0] = 0;
    for (int s = 0; s < steps; s++) {
        int lower = !((v >> s) & 1);
        if (lower) {
            rcount[s] = wsize / 2;
            scount[s] = wsize - rcount[s];
            sindex[s] = rindex[s] + rcount[s];
        } else {
            scount[s] = wsize / 2;
            rcount[s] = wsize - scount[s];
            rindex[s] = sindex[s] + scount[s];
        }
        if (s + 1 < steps) {
            rindex[s + 1] = rindex[s];
            sindex[s + 1] = rindex[s];
            wsize = rcount[s];
        }
    }
}

static void *at(const rb_ctx *x, void *base, int64_t idx) { return (char *)base + (size_t)idx * x->es; }

/* The buffer holding every rank's reduce-scatter window after step s (uniform: the same on
 * every rank and for the whole call).  Without a spare, W: every failure aborts, and the
 * steps reduce in place.  With a spare a partner's death mid-exchange is recoverable and the
 * received window must then be discarded (corr, :238-241): the steps reduce OUT OF PLACE,
 * alternating W and T -- whose half rw0 is free, T holding the partner's other half sw0 -- so
 * the step's input window stays intact and nothing has to be restored (round 4 stored the
 * pre-image, rcount x es bytes per step: 96 MiB per 256 MiB call at p = 9).  The parity ends
 * in W at the last step, where the allgather reads the final blocks.  Every later window lies
 * in the earlier ones, and a rank only writes its own receive windows, so a partner's send
 * window at step s stays what it held after step s - 1 (the replay of rb_handler_rs reads it
 * there). */
static int rb_acc(const rb_ctx *x, int s) { return (!x->alt || (x->steps - 1 - s) % 2 == 0) ? WS_W : WS_T; }

static int rb_vrank_of(const rb_ctx *x, int cr)
{
    if (cr < 2 * x->rem) return (cr % 2 == 0) ? cr / 2 : -1;
    return cr - x->rem;
}

/* Every receiver's pull(s) at a reduce-scatter (ag = 0) or allgather (ag = 1) step:
 * what ftar_xfer needs to stripe the exchange over relays (raben/rabenseifner.c:170-249,
 * :299-315). */
static void rb_plan(const rb_ctx *x, int step, int mask, int ag, ftar_plan *P)
{
    ftar_comm *c = x->c;
    ftar_plan_clear(P);
    int64_t ri[MAXSTEPS], si[MAXSTEPS], rc[MAXSTEPS], sc[MAXSTEPS];
    for (int cr = 0; cr < c->size; cr++) {
        int v = rb_vrank_of(x, cr);
        if (v == -1) continue;
        rb_windows(v, x->count, x->steps, ri, si, rc, sc);
        int src = c->order[rb_real(x, v ^ mask)];
        ftar_pull *pl = P->pull[cr];
        memset(pl, 0, sizeof(ftar_pull) * FTAR_MAX_PULLS);
        if (ag) { /* the last allgather step lands in rbuf: only there (fast_io) or also in W */
            int last = step == 0;
            pl[0] = (ftar_pull){FDEV_COPY, 0, src, WS_W, (x->fast_io && last) ? WS_UOUT : WS_W, WS_W, si[step],
                                sc[step], !x->fast_io && last};
            P->npull[cr] = 1;
        } else if (step == 0) { /* fast_io: the local operand is sbuf itself */
            pl[0] = (ftar_pull){FDEV_REDUCE, 0, src, WS_IN, rb_acc(x, 0), x->fast_io ? WS_UIN : WS_IN, ri[0], rc[0], 0};
            pl[1] = (ftar_pull){FDEV_COPY, 0, src, WS_IN, WS_T, WS_T, si[0], sc[0], 0};
            P->npull[cr] = x->keep_recov ? 2 : 1;
        } else { /* the partner's window of the previous step, reduced into this step's accumulator */
            pl[0] = (ftar_pull){FDEV_REDUCE, 0, src, rb_acc(x, step - 1), rb_acc(x, step), rb_acc(x, step - 1), ri[step],
                                rc[step], 0};
            P->npull[cr] = 1;
        }
    }
}

static void run_reduce(rb_ctx *x, void *out, const void *xin, const void *yin, int64_t n, int remote, int tag)
{
    fdev_seg s = {FDEV_REDUCE, remote, out, xin, yin, (size_t)n, NULL};
    ftar_run(x->c, x->dtype, x->op, &s, 1, tag);
}

static void run_copy(rb_ctx *x, void *out, const void *src, int64_t n, int remote, int tag)
{
    fdev_seg s = {FDEV_COPY, remote, out, src, NULL, (size_t)n, NULL};
    ftar_run(x->c, x->dtype, x->op, &s, 1, tag);
}

/* errhandler_reduce_scatter (raben/errhandler.c:3-282) in pull form */
static void rb_handler_rs(rb_ctx *x, uint64_t newf, int fs)
{
    ftar_comm *c = x->c;
    int nf = __builtin_popcountll(newf);
    c->acked |= newf; /* MPIX_Comm_failure_ack (:20-21) */
    if (nf > 1 || fs == 0) ftar_abort(c, 1); /* :37-38 */
    int dead_w = __builtin_ctzll(newf);
    int dead = ftar_comm_rank_of(c, dead_w);
    int idle_die = (dead < x->rem * 2 && dead % 2 == 1);
    if (idle_die) { /* :50-76 */
        ftar_regroup(c, dead, x->rem * 2 - 1);
    } else {
        int vdead = (dead < x->rem * 2) ? dead / 2 : dead - x->rem; /* :80-88 */
        int org = rb_real(x, vdead ^ 1);                           /* :89-90 */
        int new_entry = x->rem * 2 - 1;                            /* :207 */
        if (new_entry == -1) ftar_abort(c, 1);                     /* :210-211 */
        int org_w = c->order[org];
        int64_t dri[MAXSTEPS], dsi[MAXSTEPS], drc[MAXSTEPS], dsc[MAXSTEPS];
        rb_windows(vdead, x->count, x->steps, dri, dsi, drc, dsc);
        if (x->rank == org) {
            if (!x->has_recov) ftar_abort(c, 1); /* deviation: a replacement holds no step-0 half */
            if (x->bg_pending) { /* the dead rank's half of its vector must be in T */
                ftar_drain_bg(c);
                x->bg_pending = 0;
            }
            /* replay the dead rank's steps 0..fs (:106-200) into W's half this rank sent at
             * step 0 (= the dead rank's reduce window, unused here until the allgather).
             * The dead rank's step-0 half: the reference's tmp copy (:191-197) where it was
             * made (FTAR_REDUNDANCY=1: T), else read where it lies -- the IN of the rank that
             * held vrank vdead at step 0 stays mapped and unwritten after its death (the
             * peers' mappings hold its memory), so the copy need not cross a link in every
             * call to make a recovery possible. */
            void *W = c->ws[WS_W], *IN = ftar_local(c, WS_IN);
            /* Failure model of the elided copy (deviation 6): the dead process's
             * memory outlives it through the peers' mappings (process death), but not a lost
             * or reset device.  The read happens only if the dead rank published that input
             * for this call and our mapping belongs to its current workspace generation;
             * otherwise there is no redundancy to replay from and the job aborts, the
             * reference's rule for an unrecoverable failure (errhandler.c:207-211). */
            const void *D0 = x->keep_recov ? (const void *)c->ws[WS_T]
                                           : ftar_dead_input(c, x->in0_w[vdead], x->count * x->es);
            if (!D0) {
                fprintf(stderr, "ftar: rank %d: the dead rank's step-0 input is not readable: no redundancy\n",
                        c->wrank);
                ftar_abort(c, 1);
            }
            run_reduce(x, at(x, W, dri[0]), at(x, IN, dri[0]), at(x, (void *)D0, dri[0]), drc[0],
                       x->keep_recov ? 0 : FDEV_REMOTE_Y, FDEV_TAG_RECOV);
            for (int s = 1; s <= fs; s++) { /* the step-s partner's send window, as it left step s - 1 */
                int pw = c->order[rb_real(x, vdead ^ (1 << s))];
                void *PW = ftar_buf(c, pw, rb_acc(x, s - 1));
                run_reduce(x, at(x, W, dri[s]), at(x, W, dri[s]), at(x, PW, dri[s]), drc[s], FDEV_REMOTE_Y,
                           FDEV_TAG_RECOV);
            }
            ftar_drain(c);
        }
        ftar_sync_fatal(c); /* the dead rank's state is ready in org's W */
        int cp = rb_real(x, vdead ^ (1 << fs));
        void *OW = ftar_buf(c, org_w, WS_W);
        if (x->rank == cp && x->corr) { /* :170-180: reduce the window the dead rank owed us */
            /* this rank's step-fs window from its (intact) step fs - 1 input: a pull that was
             * skipped, cut short or made from a dying rank's memory is simply not used */
            run_reduce(x, at(x, ftar_local(c, rb_acc(x, fs)), x->rindex[fs]),
                       at(x, ftar_local(c, rb_acc(x, fs - 1)), x->rindex[fs]), at(x, OW, x->rindex[fs]),
                       x->rcount[fs], FDEV_REMOTE_Y, FDEV_TAG_RECOV);
        }
        if (x->rank == new_entry) { /* :213-241: take over the dead rank's role */
            memcpy(x->rindex, dri, sizeof(dri));
            memcpy(x->sindex, dsi, sizeof(dsi));
            memcpy(x->rcount, drc, sizeof(drc));
            memcpy(x->scount, dsc, sizeof(dsc));
            /* the dead rank's whole reduce-scatter state, not only its current window: a
             * later replay (a second failure) pulls this rank's sindex[s] windows of the
             * steps s <= fs, which all lie in the step-0 window (the reference ships the
             * whole buffer, :213-241).  Each part goes where the dead rank held it: the part
             * of window s it sent at step s + 1 in step s's accumulator, the live window
             * fs in step fs's (one launch) */
            fdev_seg seg[MAXSTEPS + 1];
            int nseg = 0;
            for (int s = 0; s <= fs; s++) {
                int64_t off = s < fs ? dsi[s + 1] : dri[fs], n = s < fs ? dsc[s + 1] : drc[fs];
                if (n <= 0) continue;
                seg[nseg++] = (fdev_seg){FDEV_COPY, FDEV_REMOTE_X, at(x, ftar_local(c, rb_acc(x, s)), off),
                                         at(x, OW, off), NULL, (size_t)n, NULL};
            }
            if (nseg) ftar_run(c, x->dtype, x->op, seg, nseg, FDEV_TAG_RECOV);
            x->has_recov = 0;
        }
        ftar_drain(c);
        ftar_sync_fatal(c);
        ftar_regroup(c, dead, new_entry); /* :243-281 */
    }
    x->rem--; /* rabenseifner.c:268-283 */
    rb_vrank(x);
    x->corr = 0;
    c->stats.recoveries++;
}

/* errhandler_allgather (raben/errhandler.c:284-468) in pull form */
static void rb_handler_ag(rb_ctx *x, uint64_t newf, int fs)
{
    ftar_comm *c = x->c;
    int nf = __builtin_popcountll(newf);
    c->acked |= newf; /* MPIX_Comm_failure_ack (:300-301) */
    if (nf > 1 || fs == x->steps - 1) ftar_abort(c, 1); /* :320-323 */
    int dead_w = __builtin_ctzll(newf);
    int dead = ftar_comm_rank_of(c, dead_w);
    int idle_die = (dead < x->rem * 2 && dead % 2 == 1);
    if (idle_die) {
        ftar_regroup(c, dead, x->rem * 2 - 1);
    } else {
        int vdead = (dead < x->rem * 2) ? dead / 2 : dead - x->rem;
        int org = rb_real(x, vdead ^ (x->adjsize >> 1)); /* :372-373 */
        int new_entry = x->rem * 2 - 1;
        if (new_entry == -1) ftar_abort(c, 1); /* :377-378 */
        if (x->rank == new_entry) {
            /* :381-398: the original partner's buffer and index arrays (equal to the dead
             * rank's for every remaining step).  Only the part held after the allgather
             * step fs is live: the reduce-scatter window of step fs-1, or all of it. */
            rb_windows(vdead, x->count, x->steps, x->rindex, x->sindex, x->rcount, x->scount);
            int64_t off = 0, n = (int64_t)x->count;
            if (fs >= 1) {
                off = x->rindex[fs - 1];
                n = x->rcount[fs - 1];
            }
            void *OW = ftar_buf(c, c->order[org], WS_W);
            run_copy(x, at(x, c->ws[WS_W], off), at(x, OW, off), n, FDEV_REMOTE_X, FDEV_TAG_RECOV);
            x->has_recov = 0;
            ftar_drain(c);
        }
        ftar_sync_fatal(c);
        int lp = rb_real(x, vdead ^ (1 << fs)); /* :400-414 */
        if (x->rank == lp) {
            void *NW = ftar_buf(c, c->order[new_entry], WS_W);
            run_copy(x, at(x, c->ws[WS_W], x->sindex[fs]), at(x, NW, x->sindex[fs]), x->scount[fs], FDEV_REMOTE_X,
                     FDEV_TAG_RECOV);
            ftar_drain(c);
        }
        ftar_sync_fatal(c);
        ftar_regroup(c, dead, new_entry);
    }
    x->rem--;
    rb_vrank(x);
    c->stats.recoveries++;
}

/* Push form of the mesh (FTAR_OPT_PUSH): where the pull form's tree kernel reads the p - 1
 * peers' parts of this rank's block over xGMI, here every rank stores its part of each
 * peer's block INTO that peer (the owner's R, one slot per source) and each owner reduces
 * its block from local memory.  Link bytes are the same (S/p per link and direction); the
 * fabric moves remote stores instead of remote loads, which bench.py compares on the node.
 * Slot j of owner u holds x_(u^j) over u's final block -- the tree's src[j] -- starting at
 * the same element offset modulo 16 bytes as the block itself, so the copies and the tree
 * keep their 16-byte vector bodies.  Returns the slot stride in elements, or 0 if the p - 1
 * slots do not fit the workspace (the caller then pulls). */
static int64_t rb_push_slot(const rb_ctx *x)
{
    int64_t e16 = (int64_t)(16 / x->es), bmax = 0;
    for (int u = 0; u < x->adjsize; u++) {
        int64_t ri[MAXSTEPS], si[MAXSTEPS], rc[MAXSTEPS], sc[MAXSTEPS];
        rb_windows(u, x->count, x->steps, ri, si, rc, sc);
        if (rc[x->steps - 1] > bmax) bmax = rc[x->steps - 1];
    }
    int64_t stride = (bmax + e16 + 63) / 64 * 64; /* 256-byte multiples (x 4 or 8 B) */
    if ((size_t)((x->adjsize - 1) * stride) * x->es > x->c->ws_bytes) return 0;
    return stride;
}

static void *rb_push_at(const rb_ctx *x, void *R, int j, int64_t block_off)
{
    int64_t e16 = (int64_t)(16 / x->es);
    return at(x, R, (int64_t)(j - 1) * x->slot + block_off % e16);
}

/* The reduce-scatter of rb_mesh in push form (see rb_push_slot): one launch of p - 1 remote
 * copies, the phase's agree (every slot has landed), the owner's tree over local memory,
 * and one more agree before the allgather reads the owners' blocks.  Kill points and
 * outcomes are rb_mesh's (no idle rank: every failure aborts). */
static void rb_mesh_push_rs(rb_ctx *x, const void *sbuf, void *rbuf)
{
    ftar_comm *c = x->c;
    const int L = x->steps, p = x->adjsize, v = x->vrank;
    void *W = c->ws[WS_W];
    int64_t own0 = x->rindex[L - 1], own_n = x->rcount[L - 1];
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_BEFORE);
    ftar_enter(c);
    fdev_seg segs[FDEV_MAX_SEGS];
    int ns = 0;
    for (int j = 1; j < p; j++) { /* owner u = v ^ j: its tree takes x_v as src[j] */
        int u = v ^ j;
        int64_t ri[MAXSTEPS], si[MAXSTEPS], rc[MAXSTEPS], sc[MAXSTEPS];
        rb_windows(u, x->count, L, ri, si, rc, sc);
        void *R = ftar_buf(c, c->order[rb_real(x, u)], WS_R);
        segs[ns++] = (fdev_seg){FDEV_COPY, FDEV_REMOTE_OUT, rb_push_at(x, R, j, ri[L - 1]),
                                at(x, (void *)sbuf, ri[L - 1]), NULL, (size_t)rc[L - 1], NULL};
    }
    double lb0 = ftar_link_bytes(c);
    ftar_run(c, x->dtype, x->op, segs, ns, FDEV_TAG_STEP0);
    ftar_launched(c, FTAR_PH_LOOP, 0); /* every step's DURING point: the pushes are in flight */
    for (int s = 1; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_DURING);
    ftar_drain(c);
    ftar_exchange_done(c);
    c->stats.step0_link_bytes += ftar_link_bytes(c) - lb0;
    c->stats.steps += L;
    c->stats.mesh_steps++;
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_AFTER);
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_BARRIER);
    uint64_t newf = ftar_step_sync(c, 3); /* every slot landed (:258-265) */
    if (newf) rb_handler_rs(x, newf, L - 1); /* no idle rank: aborts */
    const void *src[FDEV_MAX_TREE];
    src[0] = at(x, (void *)sbuf, own0);
    for (int j = 1; j < p; j++) src[j] = rb_push_at(x, c->ws[WS_R], j, own0);
    /* push == 2: the allgather rides on the tree -- its result goes to this rank's rbuf
     * and straight into every peer's W (the owner's block, remote stores) */
    void *more[FDEV_MAX_TREE];
    int nmore = 0;
    if (x->push == 2) {
        for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_BEFORE);
        ftar_enter(c);
        for (int j = 1; j < p; j++) more[nmore++] = at(x, ftar_buf(c, c->order[rb_real(x, v ^ j)], WS_W), own0);
    }
    void *out = x->push == 2 ? at(x, rbuf, own0) : at(x, W, own0);
    if (x->push == 1) { /* as the pull form: the block into rbuf too, where co-aligned (rb_mesh) */
        more[0] = at(x, rbuf, own0);
        x->own_in_rbuf = x->io_safe && (((uintptr_t)more[0] ^ (uintptr_t)out) & 15) == 0;
        nmore = x->own_in_rbuf;
    }
    if (fdev_tree_out(c->dev, x->dtype, x->op, src, p, 0, out, more, nmore, x->push == 2, (size_t)own_n,
                      FDEV_TAG_STEP)) {
        fprintf(stderr, "ftar: rank %d: launch failed: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    ftar_note_launch(c, x->push == 2 ? more[0] : NULL, 0);
    if (x->push == 2) {
        ftar_launched(c, FTAR_PH_AG, L - 1);
        for (int s = L - 2; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_DURING);
    }
    ftar_drain(c);
    if (x->push == 2) {
        ftar_exchange_done(c);
        c->stats.steps += L;
        c->stats.mesh_steps++;
        for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_AFTER);
        for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_BARRIER);
    }
    /* every owner's block is final (push == 1: before the allgather pulls it; push == 2:
     * every peer's pushed block has landed in this rank's W) */
    newf = ftar_step_sync(c, 3);
    if (newf) rb_handler_rs(x, newf, L - 1);
}

/* push == 2, after rb_mesh_push_rs: the peers' blocks, pushed into this rank's W, to rbuf
 * (one local copy launch), then the ERRORS_ARE_FATAL barrier (:357-360).  The copy comes
 * before this rank arrives at the barrier: no peer's next call can push into W while it
 * is being read. */
static int rb_mesh_push_finish(rb_ctx *x, void *rbuf)
{
    ftar_comm *c = x->c;
    const int L = x->steps, p = x->adjsize, v = x->vrank;
    fdev_seg segs[FDEV_MAX_SEGS];
    int ns = 0;
    for (int j = 1; j < p; j++) {
        int64_t ri[MAXSTEPS], si[MAXSTEPS], rc[MAXSTEPS], sc[MAXSTEPS];
        rb_windows(v ^ j, x->count, L, ri, si, rc, sc);
        segs[ns++] = (fdev_seg){FDEV_COPY, 0, at(x, rbuf, ri[L - 1]), at(x, c->ws[WS_W], ri[L - 1]), NULL,
                                (size_t)rc[L - 1], NULL};
    }
    ftar_run(c, x->dtype, x->op, segs, ns, FDEV_TAG_LOCAL);
    ftar_drain(c);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BEFORE);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_DURING);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_AFTER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BARRIER);
    uint64_t newf = ftar_step_sync(c, 3);
    if (newf) rb_handler_ag(x, newf, 0); /* no idle rank: aborts */
    ftar_stats_end(c);
    return FTAR_SUCCESS;
}

/* The tolerant region at power-of-two p without an idle rank, on the full xGMI mesh.
 *
 * Recursive halving leaves in vrank v's final block the value
 *     T(v, L),  T(v, 0) = x_v,  T(v, s+1) = T(v, s) op T(v ^ 2^s, s)
 * (raben/rabenseifner.c:231-237: own window first, the partner's second; the partner's
 * window was reduced by the same rule).  With the sources listed owner-relative
 * (src[j] = x_{v^j}) that is the left-to-right balanced tree over j, which one tree
 * kernel computes from p - 1 one-hop pulls -- every link of the GPU busy with 1/p of the
 * vector instead of one link per step.  The allgather (:299-355) likewise pulls every
 * peer's final block straight into rbuf.  Per rank and direction each link carries
 * S/p for the reduce-scatter and S/p for the allgather: the mesh lower bound for an
 * allreduce, half of what a 2-hop relay moves.
 *
 * The reference's per-step states are unobservable here: with no idle rank every
 * handler aborts (new_entry = -1, raben/errhandler.c:207-211, 377-378), so a failure
 * anywhere in a phase ends the job exactly as it would at that step's agree.  Every
 * step's kill points are still passed (the injected death lands in the same phase), and
 * each phase ends in the reference's agree + barrier. */
/* The mesh allgather's one launch: this rank's final block W -> rbuf and every peer's final
 * block, pulled out of its W, into rbuf (the operands are known before the reduce-scatter's
 * barrier: the launch can be queued ahead of it, behind a gate). */
static int rb_mesh_ag_segs(rb_ctx *x, void *rbuf, fdev_seg *segs)
{
    ftar_comm *c = x->c;
    const int L = x->steps, p = x->adjsize, v = x->vrank;
    int ns = 0;
    if (!x->own_in_rbuf)
        segs[ns++] = (fdev_seg){FDEV_COPY, 0, at(x, rbuf, x->rindex[L - 1]), at(x, c->ws[WS_W], x->rindex[L - 1]),
                                NULL, (size_t)x->rcount[L - 1], NULL};
    for (int j = 1; j < p; j++) {
        int u = v ^ j;
        int64_t ri[MAXSTEPS], si[MAXSTEPS], rc[MAXSTEPS], sc[MAXSTEPS];
        rb_windows(u, x->count, L, ri, si, rc, sc);
        void *PW = ftar_buf(c, c->order[rb_real(x, u)], WS_W);
        segs[ns++] = (fdev_seg){FDEV_COPY, FDEV_REMOTE_X, at(x, rbuf, ri[L - 1]), at(x, PW, ri[L - 1]), NULL,
                                (size_t)rc[L - 1], NULL};
    }
    return ns;
}

/* The mesh with its allgather ordered on the device (FTAR_OPT_MESH_WAIT), continuing
 * rb_mesh after the tree launch.  The reduce-scatter's agree only ever served to say "every
 * owner's block is final" -- with no idle rank every failure aborts the job at whichever
 * agree sees it (new_entry = -1, raben/errhandler.c:207-211, 377-378) -- so that fact moves
 * to the device: each rank releases its tree (a fenced marker) and publishes the call's token
 * in its line of the control block's flag page (host memory every GPU maps); the allgather,
 * queued right behind, runs once every peer's flag holds the token.  Per call this saves one
 * host agree round, one drain and the allgather's launch latency; the call keeps its first
 * and last agree.  A peer that dies before publishing: the drain's failure detector gives
 * the wait up (the allgather returns untouched), and the last agree sees the death -- the
 * handler aborts, as at the agree this form leaves out.  A wait the device gave up with
 * every member alive (its timeout): each rank publishes its verdict in the last agree round,
 * so all of them learn it alike; by then every tree is released (each rank drained its own
 * before arriving), the ranks whose allgather returned untouched launch it again (it never
 * writes what it reads), and one more round keeps the peers' next call off their W until it
 * is done.  Every step's kill points are passed, in the order both launches are queued: RS
 * BEFORE, DURING; AG BEFORE, DURING; then, once drained, RS AFTER / BARRIER and AG AFTER /
 * BARRIER. */
static int rb_mesh_devwait(rb_ctx *x, void *rbuf, double lb0)
{
    ftar_comm *c = x->c;
    const int L = x->steps, p = x->adjsize, v = x->vrank;
    fdev_seg segs[FDEV_MAX_SEGS];
    ftar_launched(c, FTAR_PH_LOOP, 0);
    for (int s = 1; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_DURING);
    for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_BEFORE);
    /* the call's token: the agree sequence number, uniform over the members and only growing */
    const uint64_t token = c->job.seq;
#ifdef FTAR_TEST_HOOKS
    /* TEST-ONLY: this rank's flag published late (its peers' waits time out) */
    if (getenv("FTAR_PEER_WAIT_DELAY_US")) {
        ftar_drain(c); /* the tree done first: the delay is in the host, not on the device */
        usleep((useconds_t)atoll(getenv("FTAR_PEER_WAIT_DELAY_US")));
    }
#endif
    void *pf[FDEV_MAX_PEERS];
    int np = 0;
    for (int j = 1; j < p; j++) pf[np++] = ftar_flag(c, c->order[rb_real(x, v ^ j)]);
    for (int i = 0; i < c->size; i++) /* FTAR_TRACE: each flag line is its owner's */
        fdev_trace_region(c->dev, ftar_flag(c, c->order[i]), sizeof(c->job.shm->pwflag[0]), c->order[i], "PF");
    if (fdev_peer_wait(c->dev, ftar_flag(c, c->wrank), pf, np, token, ftar_watch_peers, c)) {
        fprintf(stderr, "ftar: rank %d: peer wait failed: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    int ns = rb_mesh_ag_segs(x, rbuf, segs);
    ftar_run(c, x->dtype, x->op, segs, ns, FDEV_TAG_STEP);
    ftar_launched(c, FTAR_PH_AG, L - 1);
    for (int s = L - 2; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_DURING);
    ftar_drain_watch(c);
    const int ran = fdev_peer_wait_verdict(c->dev);
    if (!ran) c->stats.peer_wait_skips++;
    ftar_exchange_done(c);
    c->stats.step0_link_bytes += ftar_link_bytes(c) - lb0;
    c->stats.steps += 2 * L;
    c->stats.mesh_steps += 2;
    c->stats.peer_waits++;
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_AFTER);
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_BARRIER);
    for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_AFTER);
    for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_BARRIER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BEFORE);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_DURING);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_AFTER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BARRIER);
    /* the reduce-scatter's and the allgather's agree and the ERRORS_ARE_FATAL barrier: one
     * round, which also carries every rank's verdict */
    c->pubval = ran ? 0 : 1;
    uint64_t newf = ftar_step_sync(c, 1);
    c->pubval = 0;
    if (newf) rb_handler_ag(x, newf, 0); /* no idle rank: aborts */
    int any_skipped = 0;
    for (int i = 0; i < c->size; i++) any_skipped |= ftar_peer_pub(c, c->order[i]) != 0;
    if (any_skipped) {
        if (!ran) {
            ftar_run(c, x->dtype, x->op, segs, ns, FDEV_TAG_STEP);
            ftar_drain(c);
        }
        newf = ftar_step_sync(c, 1);
        if (newf) rb_handler_ag(x, newf, 0);
    }
    ftar_stats_end(c);
    return FTAR_SUCCESS;
}

static int rb_mesh(rb_ctx *x, const void *sbuf, void *rbuf)
{
    ftar_comm *c = x->c;
    const int L = x->steps, p = x->adjsize, v = x->vrank;
    void *W = c->ws[WS_W];
    int64_t own0 = x->rindex[L - 1], own_n = x->rcount[L - 1];
    fdev_seg segs[FDEV_MAX_SEGS];
    int ns = 0;

    uint64_t newf;
    if (x->push) {
        rb_mesh_push_rs(x, sbuf, rbuf);
        if (x->push == 2) return rb_mesh_push_finish(x, rbuf);
        goto allgather;
    }
    /* reduce-scatter: T(v, L) over this rank's final block */
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_BEFORE);
    ftar_enter(c);
    const void *src[FDEV_MAX_TREE];
    unsigned remote = 0;
    for (int j = 0; j < p; j++) {
        int u = v ^ j;
        /* a peer's input: its sbuf in place, or its staged IN */
        src[j] = j == 0 ? at(x, (void *)sbuf, own0) : at(x, ftar_buf(c, c->order[rb_real(x, u)], WS_IN), own0);
        if (j) remote |= 1u << j;
    }
    double lb0 = ftar_link_bytes(c);
    ftar_note_launch(c, src[1], (size_t)own_n * x->es);
    /* the block goes to W, where the peers' allgather pulls it, and in the same pass to its
     * place in rbuf (a second destination of the tree: one more local store of S/p), so the
     * allgather only pulls the peers' blocks -- no local copy of this rank's own block, S/p
     * fewer HBM reads per call (in place, rbuf's block is sbuf's, read by this lane only) */
    void *own_out = at(x, rbuf, own0);
    /* only where rbuf is co-aligned with W (a 16-byte vector body needs every operand at the
     * same offset mod 16; otherwise the tree would fall back to scalar accesses): else the
     * allgather copies the block out of W as before */
    x->own_in_rbuf = x->io_safe && (((uintptr_t)own_out ^ (uintptr_t)at(x, W, own0)) & 15) == 0;
    if (fdev_tree_out(c->dev, x->dtype, x->op, src, p, remote, at(x, W, own0), &own_out, x->own_in_rbuf, 0,
                      (size_t)own_n, FDEV_TAG_STEP0)) {
        fprintf(stderr, "ftar: rank %d: launch failed: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    if (x->devwait) return rb_mesh_devwait(x, rbuf, lb0);
    /* FTAR_OPT_MESH_WAIT=0: the allgather launched after the reduce-scatter's agree round.
     * (Round 4's form with the allgather queued behind the tree behind a host-opened gate,
     * FTAR_GATE_MAX >= S, was slower in every rehearsal and is superseded by the device wait:
     * removed in round 6.) */
    ftar_launched(c, FTAR_PH_LOOP, 0); /* every step's DURING point: the one launch is in flight */
    for (int s = 1; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_DURING);
    ftar_drain(c);
    ftar_exchange_done(c);
    c->stats.step0_link_bytes += ftar_link_bytes(c) - lb0;
    c->stats.steps += L;
    c->stats.mesh_steps++;
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_AFTER);
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_BARRIER);
    newf = ftar_step_sync(c, 2); /* agree + barrier (:258-265) */
    if (newf) rb_handler_rs(x, newf, L - 1); /* no idle rank: aborts */

allgather:
    /* allgather: every peer's final block into rbuf, this rank's own out of W */
    for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_BEFORE);
    ftar_enter(c);
    ns = rb_mesh_ag_segs(x, rbuf, segs);
    ftar_run(c, x->dtype, x->op, segs, ns, FDEV_TAG_STEP);
    ftar_launched(c, FTAR_PH_AG, L - 1);
    for (int s = L - 2; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_DURING);
    ftar_drain(c);
    ftar_exchange_done(c);
    c->stats.steps += L;
    c->stats.mesh_steps++;
    for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_AFTER);
    for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_BARRIER);
    /* The allgather's agree (:330-335) and the ERRORS_ARE_FATAL barrier (:357-360; no
     * post-step at rem = 0) are one round: a failure seen at either ends the job the same
     * way (no idle rank: errhandler_allgather aborts, new_entry = -1, :377-378), so the
     * outcome of every kill point is unchanged. */
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BEFORE);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_DURING);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_AFTER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BARRIER);
    newf = ftar_step_sync(c, 2);
    if (newf) rb_handler_ag(x, newf, 0); /* no idle rank: aborts */
    ftar_stats_end(c);
    return FTAR_SUCCESS;
}

/* One-shot mesh for small vectors: the allgather's data movement folded into the
 * reduce-scatter launch.  Each rank evaluates EVERY block in its owner's tree,
 * T(u, L) = tree over x_(u^j) (the same operands and order as rb_mesh's reduce-scatter,
 * so the same bits), straight into rbuf: one launch instead of two, (p-1) S link bytes
 * per rank instead of 2 (p-1) S / p -- cheaper below the size where a launch + drain
 * (~11 us) outweighs the extra link time.  Kill points and the two agree rounds are
 * rb_mesh's; with no idle rank a failure anywhere aborts. */
/* The one-shot launch's operands as the peers' inputs stand now (ftar_buf: a peer's
 * exported sbuf once ftar_resolve_inputs mapped it, else its staged IN). */
static void rb_oneshot_plan(rb_ctx *x, const void *sbuf, void *rbuf, struct rb_batch *B)
{
    ftar_comm *c = x->c;
    const int L = x->steps, p = x->adjsize, v = x->vrank;
    memset(B, 0, sizeof(*B));
    for (int u = 0; u < p; u++) { /* block owned by vrank u */
        int64_t ri[MAXSTEPS], si[MAXSTEPS], rc[MAXSTEPS], sc[MAXSTEPS];
        rb_windows(u, x->count, L, ri, si, rc, sc);
        const int64_t off = ri[L - 1];
        B->out[u] = at(x, rbuf, off);
        B->n[u] = (size_t)rc[L - 1];
        for (int j = 0; j < p; j++) {
            const int w = u ^ j;
            if (w == v) {
                B->src[u * p + j] = at(x, (void *)sbuf, off);
            } else {
                B->src[u * p + j] = at(x, ftar_buf(c, c->order[rb_real(x, w)], WS_IN), off);
                B->remote[u] |= 1u << j;
            }
        }
    }
}

/* Queue the one-shot launch right behind this rank's staging copy, before the barrier
 * after which the peers' staged inputs may be read: its workgroups wait on a gate that
 * rb_oneshot opens at the point where it would otherwise launch, so the launch latency
 * overlaps the staging drain and the barrier.  The plan assumes every peer stages its
 * input (this rank did, so the size is the same everywhere); rb_oneshot re-plans after
 * the inputs are resolved and skips the gated launch if anything differs. */
static void rb_oneshot_prelaunch(rb_ctx *x, const void *sbuf, void *rbuf, void *stage_dst)
{
    ftar_comm *c = x->c;
    x->gated = 0;
    if (!c->gate) return;
    rb_oneshot_plan(x, sbuf, rbuf, &x->gplan);
    /* stage_dst: this rank's staging copy (sbuf -> IN) rides in the same launch, ahead of
     * the gate -- one launch per call instead of two */
    if (fdev_tree_batch_staged_gated(c->dev, x->dtype, x->op, x->gplan.src, x->adjsize, x->gplan.remote,
                                     x->gplan.out, x->gplan.n, x->adjsize, FDEV_TAG_STEP0, stage_dst, sbuf,
                                     stage_dst ? x->count : 0, &x->gated)) {
        fprintf(stderr, "ftar: rank %d: launch failed: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    if (x->gated) c->stats.gated_launches++;
}

static int rb_oneshot(rb_ctx *x, const void *sbuf, void *rbuf)
{
    ftar_comm *c = x->c;
    const int L = x->steps, p = x->adjsize;
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_BEFORE);
    ftar_enter(c);
    struct rb_batch B;
    rb_oneshot_plan(x, sbuf, rbuf, &B);
    const void *const *src = B.src;
    double lb0 = ftar_link_bytes(c);
    for (int k = 0; k < p * p; k++) /* the first peer operand: the padding's re-pull source */
        if (B.remote[k / p] & (1u << (k % p))) {
            ftar_note_launch(c, src[k], B.n[k / p] * x->es);
            break;
        }
    /* the queued launch runs now, or returns untouched and is replaced (also when another
     * launch has given it up meanwhile) */
    int pending = x->gated && fdev_gate_pending(c->dev);
    int go = pending && memcmp(&B, &x->gplan, sizeof(B)) == 0;
    if (x->gated && !go) c->stats.gated_skips++;
    if (pending) fdev_gate_open(c->dev, !go);
    x->gated = 0;
    if (!go && fdev_tree_batch(c->dev, x->dtype, x->op, src, p, B.remote, B.out, B.n, p, FDEV_TAG_STEP0)) {
        fprintf(stderr, "ftar: rank %d: launch failed: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    ftar_launched(c, FTAR_PH_LOOP, 0);
    for (int s = 1; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_DURING);
    ftar_drain(c);
    ftar_exchange_done(c);
    c->stats.step0_link_bytes += ftar_link_bytes(c) - lb0;
    c->stats.steps += 2 * L;
    c->stats.mesh_steps++;
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_AFTER);
    for (int s = 0; s < L; s++) ftar_maybe_die(c, FTAR_PH_LOOP, s, FTAR_PT_BARRIER);
    /* The reduce-scatter's agree (:258-265), the allgather's (:330-335) and the
     * ERRORS_ARE_FATAL barrier (:357-360) are one round here: the allgather's data moved in
     * the same launch, and with no idle rank a failure seen at any of them ends the job the
     * same way (both handlers abort, new_entry = -1, errhandler.c:207-211, 377-378) -- the
     * kill points of every phase are passed before it, so each one's outcome is unchanged. */
    for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_BEFORE);
    ftar_enter(c); /* the allgather's data already moved in the one launch */
    ftar_launched(c, FTAR_PH_AG, L - 1);
    for (int s = L - 2; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_DURING);
    ftar_exchange_done(c);
    for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_AFTER);
    for (int s = L - 1; s >= 0; s--) ftar_maybe_die(c, FTAR_PH_AG, s, FTAR_PT_BARRIER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BEFORE);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_DURING);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_AFTER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BARRIER);
    uint64_t newf = ftar_step_sync(c, 1);
    if (newf) rb_handler_rs(x, newf, L - 1); /* no idle rank: aborts */
    ftar_stats_end(c);
    return FTAR_SUCCESS;
}

int ftar_allreduce_rabenseifner(const void *sbuf, void *rbuf, size_t count, ftar_dtype dtype, ftar_op op,
                                ftar_comm *c)
{
    if (!c) return FTAR_ERR_ARG;
    rb_ctx X;
    memset(&X, 0, sizeof(X));
    rb_ctx *x = &X;
    x->c = c;
    x->dtype = (int)dtype;
    x->op = (int)op;
    x->es = ftar_esize(dtype);
    x->count = count;
    int orc = ftar_check_op((int)dtype, (int)op);
    if (orc) return orc;
    x->steps = ftar_hibit(c->size, (int)(sizeof(int) * 8) - 1); /* :16-21 */
    if (x->steps == -1) return FTAR_ERR_ARG;
    if (count == 0) return FTAR_ERR_UNKNOWN; /* copy_buffer(count <= 0), util.c:40-43 */
    if (count > (size_t)INT64_MAX / 16 || !sbuf || !rbuf) return FTAR_ERR_ARG;
    /* device pointers: pageable host memory or a short allocation is refused, not faulted on */
    if (fdev_check_ptr(c->dev, sbuf, count * x->es) || fdev_check_ptr(c->dev, rbuf, count * x->es))
        return FTAR_ERR_ARG;
    x->adjsize = 1 << x->steps;
    x->rem = c->size - x->adjsize;
    x->alt = x->rem > 0; /* uniform; fixed for the call (rem only decreases) */
    /* The step-0 copy of the partner's other half (tmp, :191-197) is only ever read by
     * an RS error handler's replay, and every handler aborts before replaying when
     * there is no idle spare (new_entry = 2 rem - 1 = -1, errhandler.c:207-211,377-378).
     * rem only decreases during a call, so with rem = 0 at the start the copy can never
     * be consumed: skip it (FTAR_REDUNDANCY=1 keeps it, the reference's shape).
     * With a spare, the copy is what lets the replay survive the loss of the dead rank's
     * memory (the reference copies at step 0 precisely because that memory is gone,
     * :206-211).  A peer's mapping keeps a killed process's memory readable on one device
     * (tested), but across GPUs that premise is unverified, so by default (auto, 2) the
     * copy moves whenever the comm spans more than one GPU; FTAR_REDUNDANCY=0 elides it on
     * any layout (the replay then reads the dead rank's input in place, deviation 6).
     * Uniform: the members' devices are the same on every rank. */
    x->keep_recov = c->redundancy == 1 || (c->redundancy == 2 && x->rem > 0 && ftar_spans_devices(c));
    /* The reference's recovery data: every rank holds its step-0 partner's other half (in
     * tmp) while a spare can use it, except a replacement rank (errhandler.c:213-241 ships
     * it the dead rank's state, not its redundancy: a replay by it aborts, as the oracle's
     * restatement does).  Without the physical copy (keep_recov = 0) the replay reads that
     * half where it lies: the IN of the rank that held the vrank at step 0. */
    x->has_recov = x->keep_recov || x->rem > 0;
    /* Without an idle rank every failure aborts (new_entry = -1, errhandler.c:207-211,
     * 377-378), so nothing outside the schedule has to stay recoverable: step 0 reads
     * this rank's reduce half straight from sbuf (only the half peers pull is staged in
     * IN), the last allgather step writes rbuf directly and copies this rank's own final
     * half out of W in the same launch, and the prologue's three barriers (no pre-step
     * exchange at rem = 0) collapse into one.  Same operands, same bits. */
    x->fast_io = !x->keep_recov && x->rem == 0 && x->steps >= 1;
    x->mesh = x->fast_io && c->mesh && c->size <= FDEV_MAX_TREE;
    /* Uniform: count, p and the options are the same on every rank.  At p = 2 the
     * one-shot form moves the same link bytes as the two-launch mesh (S per direction)
     * in one launch, so it runs at every size; at p > 2 it reads (p - 2) S / p more per
     * link and pays off only below oneshot_max. */
    x->oneshot = x->mesh && c->size <= FDEV_MAX_BATCH && c->oneshot_max > 0 &&
                 (c->size == 2 || count * (size_t)x->es <= c->oneshot_max);
    /* push 2 (both phases) needs every peer as an extra destination of one tree: p <= 8 */
    x->push = (x->mesh && !x->oneshot && c->push) ? (c->push == 2 && c->size <= 8 ? 2 : 1) : 0;
    /* uniform too; every block non-empty (count >= p: the allgather launch always exists); not
     * with FTAR_OPT_FLAG_SYNC off, the conservative mode of fenced-marker drains only (whose
     * pinned flag words the wait also uses) */
    x->devwait = x->mesh && !x->oneshot && !x->push && c->mesh_wait && count >= (size_t)c->size &&
                 c->size - 1 <= FDEV_MAX_PEERS && fdev_get_knob(c->dev, FDEV_KNOB_FLAG_SYNC) == 1 && ftar_flag(c, c->wrank);
    c->uin = sbuf;
    c->uout = rbuf;
    ftar_stats_begin(c);
    c->stats.step0_copy = x->keep_recov && c->size > 1;
    if (c->size == 1) return ftar_single_rank(c, sbuf, rbuf, count * x->es);

    size_t bytes = count * x->es;
    ftar_ensure_workspace(c, bytes);
    if (x->push) { /* uniform: the same geometry on every rank */
        x->slot = rb_push_slot(x);
        x->push = x->slot > 0;
    }
    void *IN = c->ws[WS_IN], *W = c->ws[WS_W], *T = c->ws[WS_T];
    fdev_order_after(c->dev, c->user_stream); /* sbuf may still be in flight on the caller's stream */
    rb_vrank(x);
    /* Where nothing writes this rank's IN -- every rank but the pre-step pairs; the
     * handlers only read it -- the peers read sbuf in place; otherwise, or when its
     * memory cannot be shared, it is staged in IN.  With a spare, the partner's step-0
     * redundancy copy may still be reading sbuf while the last allgather step writes
     * rbuf, so there sbuf and rbuf must not overlap. */
    const char *s0 = (const char *)sbuf, *d0 = (const char *)rbuf;
    int disjoint = s0 + bytes <= d0 || d0 + bytes <= s0;
    /* partly overlapping sbuf / rbuf (neither the same buffer nor disjoint): rbuf is written
     * only after every peer is done reading sbuf */
    x->io_safe = disjoint || s0 == d0;
    /* The one-shot launch writes rbuf while peers still read this rank's input: in place,
     * that input must be staged (whole: peers read every block of it). */
    /* push: no peer ever reads this rank's input (it stores its parts into the owners) */
    int aliased = x->push ? 0 :
                  ftar_stage_input(c, sbuf, bytes,
                                   x->oneshot ? disjoint : (x->fast_io || (x->rank >= 2 * x->rem && disjoint)));
    if (x->push) {
        ftar_inputs_done(c);
        rb_windows(x->vrank, count, x->steps, x->rindex, x->sindex, x->rcount, x->scount);
    } else if (aliased) {
        IN = (void *)sbuf;
        rb_windows(x->vrank, count, x->steps, x->rindex, x->sindex, x->rcount, x->scount);
    } else if (x->oneshot) {
        rb_windows(x->vrank, count, x->steps, x->rindex, x->sindex, x->rcount, x->scount);
        /* small inputs are staged by every rank (ftar_stage_input): the launch's operands
         * are known before the barrier, and the staging copy can ride in it */
        if (bytes <= c->stage_max) {
            rb_oneshot_prelaunch(x, sbuf, rbuf, IN);
            if (x->gated) ftar_note_launch(c, NULL, 0); /* the staging phase is in flight */
        }
        if (!x->gated) {
            run_copy(x, IN, sbuf, (int64_t)count, 0, FDEV_TAG_LOCAL);
            if (bytes <= c->stage_max) rb_oneshot_prelaunch(x, sbuf, rbuf, NULL);
        }
    } else if (x->mesh) { /* peers pull every block of sbuf but this rank's own final one */
        rb_windows(x->vrank, count, x->steps, x->rindex, x->sindex, x->rcount, x->scount);
        int64_t b0 = x->rindex[x->steps - 1], b1 = b0 + x->rcount[x->steps - 1];
        fdev_seg cp[2] = {{FDEV_COPY, 0, IN, sbuf, NULL, (size_t)b0, NULL},
                          {FDEV_COPY, 0, at(x, IN, b1), at(x, (void *)sbuf, b1), NULL, (size_t)((int64_t)count - b1),
                           NULL}};
        ftar_run(c, x->dtype, x->op, cp, 2, FDEV_TAG_LOCAL);
    } else if (x->fast_io) { /* the half of sbuf peers pull at step 0 */
        rb_windows(x->vrank, count, x->steps, x->rindex, x->sindex, x->rcount, x->scount);
        run_copy(x, at(x, IN, x->sindex[0]), at(x, (void *)sbuf, x->sindex[0]), x->scount[0], 0, FDEV_TAG_LOCAL);
    } else {
        run_copy(x, IN, sbuf, (int64_t)count, 0, FDEV_TAG_LOCAL); /* rbuf = sbuf, :35-42 */
    }
    ftar_drain(c);

    /* ---- pre-step (:61-139): failures are fatal here ---- */
    ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_BEFORE);
    if (x->fast_io) {
        ftar_enter(c);
        ftar_launched(c, FTAR_PH_PRE, 0);
        ftar_exchange_done(c);
        ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_AFTER);
        ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_BARRIER);
        ftar_sync_fatal(c); /* every IN is ready; the barrier before the tolerant region (:166) */
        ftar_resolve_inputs(c);
    } else {
        ftar_sync_fatal(c); /* every IN is ready */
        ftar_resolve_inputs(c);
        ftar_enter(c);
        int64_t lh = (int64_t)count / 2, rh = (int64_t)count - lh;
        int pair = x->rank < 2 * x->rem;
        if (pair) {
            if (x->rank % 2 != 0) { /* odd: reduce the right half with the even's right half */
                void *P = ftar_buf(c, c->order[x->rank - 1], WS_IN);
                run_reduce(x, at(x, IN, lh), at(x, IN, lh), at(x, P, lh), rh, FDEV_REMOTE_Y, FDEV_TAG_STEP);
            } else { /* even: reduce the left half with the odd's left half */
                void *P = ftar_buf(c, c->order[x->rank + 1], WS_IN);
                run_reduce(x, IN, IN, P, lh, FDEV_REMOTE_Y, FDEV_TAG_STEP);
            }
        }
        ftar_launched(c, FTAR_PH_PRE, 0);
        if (pair) {
            ftar_drain(c);
            c->stats.steps++;
        }
        ftar_exchange_done(c);
        ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_AFTER);
        ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_BARRIER);
        ftar_sync_fatal(c);
        if (x->rank < 2 * x->rem && x->rank % 2 == 0) { /* even: receive the reduced right half (:120) */
            void *P = ftar_buf(c, c->order[x->rank + 1], WS_IN);
            run_copy(x, at(x, IN, lh), at(x, P, lh), rh, FDEV_REMOTE_X, FDEV_TAG_STEP);
            ftar_drain(c);
        }
        if (x->vrank != -1)
            rb_windows(x->vrank, count, x->steps, x->rindex, x->sindex, x->rcount, x->scount);
        ftar_sync_fatal(c); /* MPI_Barrier before the tolerant region (:166) */
    }

    if (x->oneshot) return rb_oneshot(x, sbuf, rbuf);
    if (x->mesh) return rb_mesh(x, sbuf, rbuf);

    /* ---- reduce-scatter (:170-284) ---- */
    for (int v = 0; v < x->adjsize; v++) x->in0_w[v] = c->order[rb_real(x, v)];
    int step = 0;
    for (int mask = 1; mask < x->adjsize; mask <<= 1, step++) {
        ftar_plan P;
        ftar_xstate xs;
        memset(&xs, 0, sizeof(xs));
        rb_plan(x, step, mask, 0, &P);
        ftar_maybe_die(c, FTAR_PH_LOOP, step, FTAR_PT_BEFORE);
        ftar_enter(c);
        int skip = 0, pw = -1;
        if (x->vrank != -1) {
            pw = c->order[rb_real(x, x->vrank ^ mask)];
            if (!ftar_peer_entered(c, pw)) skip = x->corr = 1; /* the exchange failed (:238-241) */
            c->stats.steps++;
        }
        /* A partner that dies mid-exchange (after entering, before its side completed) fails
         * the Sendrecv too: the reference then discards the received window (corr, :238-241)
         * and the RS handler rebuilds it from the impersonator's replay.  With a spare the
         * step reduced out of place (rb_acc): its input window is intact, so discarding is
         * just not using the result -- the handler's corr reduce recomputes the window from
         * the step's input and the replayed state.  (At step 0 the handler aborts.)  If a
         * relay died the window may be partly unreduced, but then a second rank died with
         * the partner and the handler aborts (nf > 1, errhandler.c:37-38). */
        int guard = x->rem > 0 && step >= 1 && pw >= 0 && !skip;
        double lb0 = ftar_link_bytes(c);
        int tag = step == 0 ? FDEV_TAG_STEP0 : FDEV_TAG_STEP;
        if (step == 0 && c->overlap && !ftar_xfer_would_relay(c, &P, x->es)) {
            /* :206-211 full exchange + :231-237 reduce, direct.  The reduce half is on the
             * critical path; the redundancy half (kept in T for recovery, :191-197) is only
             * needed by a later error handler, so it runs on the background stream and
             * overlaps steps 1.. (joined before any replay and before the final barrier).
             * (With relays both halves are striped in the step itself.) */
            if (x->vrank != -1 && !skip) {
                const ftar_pull *pl = P.pull[x->rank];
                void *PIN = ftar_buf(c, pl[0].src, WS_IN);
                fdev_seg red = {FDEV_REDUCE, FDEV_REMOTE_Y, at(x, ftar_local(c, pl[0].dst_buf), pl[0].off),
                                at(x, ftar_local(c, pl[0].x_buf), pl[0].off), at(x, PIN, pl[0].off), (size_t)pl[0].n,
                                NULL};
                fdev_seg cpy = {FDEV_COPY, FDEV_REMOTE_X, at(x, T, pl[1].off), at(x, PIN, pl[1].off), NULL,
                                (size_t)pl[1].n, NULL};
                ftar_run_pulls(c, x->dtype, x->op, &red, 1, FDEV_TAG_STEP0, 0);
                if (x->keep_recov) {
                    ftar_run_pulls(c, x->dtype, x->op, &cpy, 1, FDEV_TAG_BG, 1);
                    x->bg_pending = 1;
                }
            }
            ftar_launched(c, FTAR_PH_LOOP, step);
            if (x->vrank != -1 && !skip) ftar_drain(c);
            ftar_exchange_done(c);
            ftar_maybe_die(c, FTAR_PH_LOOP, step, FTAR_PT_AFTER);
        } else {
            ftar_xfer_step(c, &P, x->dtype, x->op, tag, skip, FTAR_PH_LOOP, step, NULL, 0, &xs);
        }
        if (guard && !ftar_peer_done(c, pw)) { /* partner died mid-exchange: corr */
            x->corr = 1;
            xs.skipped = 1; /* nothing of this window is re-pulled after the agree */
            if (c->verbose)
                fprintf(stderr, "ftar: rank %d: partner %d died mid-exchange at RS step %d: window discarded\n",
                        c->wrank, pw, step);
        }
        if (step == 0) c->stats.step0_link_bytes += ftar_link_bytes(c) - lb0;
        ftar_maybe_die(c, FTAR_PH_LOOP, step, FTAR_PT_BARRIER);
        uint64_t newf = ftar_step_sync(c, 2 * x->steps); /* agree + barrier (:258-265) */
        if (newf) {
            ftar_xfer_repair(c, &P, x->dtype, x->op, &xs, newf);
            rb_handler_rs(x, newf, step);
        }
    }

    /* ---- allgather (:299-355) ---- */
    step = x->steps - 1;
    for (int mask = x->adjsize >> 1; mask > 0; mask >>= 1, step--) {
        ftar_plan P;
        ftar_xstate xs;
        rb_plan(x, step, mask, 1, &P);
        ftar_maybe_die(c, FTAR_PH_AG, step, FTAR_PT_BEFORE);
        ftar_enter(c);
        int skip = 0;
        if (x->vrank != -1) {
            skip = !ftar_peer_entered(c, c->order[rb_real(x, x->vrank ^ mask)]);
            c->stats.steps++;
        }
        /* last step: this rank's own final half W -> rbuf rides in the same launch */
        fdev_seg own = {FDEV_COPY, 0, NULL, NULL, NULL, 0, NULL};
        int nown = 0;
        if (step == 0 && x->vrank != -1) {
            own.out = at(x, rbuf, x->rindex[0]);
            own.x = at(x, W, x->rindex[0]);
            own.n = (size_t)x->rcount[0];
            nown = 1;
        }
        ftar_xfer_step(c, &P, x->dtype, x->op, FDEV_TAG_STEP, skip, FTAR_PH_AG, step, &own, nown, &xs);
        ftar_maybe_die(c, FTAR_PH_AG, step, FTAR_PT_BARRIER);
        uint64_t newf = ftar_step_sync(c, 2 * x->steps); /* (:330-335) */
        x->out_done = nown && !skip && !newf; /* a recovery here re-homes windows: copy W at the end */
        if (newf) {
            ftar_xfer_repair(c, &P, x->dtype, x->op, &xs, newf);
            rb_handler_ag(x, newf, step);
        }
    }

    if (x->bg_pending) { /* peers read our IN until their copies are done: join before the barrier */
        ftar_drain_bg(c);
        x->bg_pending = 0;
    }

    /* ---- ERRORS_ARE_FATAL barrier + post-step (:357-381) ---- */
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BEFORE);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_DURING);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_AFTER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BARRIER);
    ftar_sync_fatal(c);
    if (x->fast_io) { /* rbuf is complete; no idle rank reads W, every peer is done with it */
        ftar_stats_end(c);
        return FTAR_SUCCESS;
    }
    if (x->rank < 2 * x->rem && x->rank % 2 != 0) {
        void *P = ftar_buf(c, c->order[x->rank - 1], WS_W); /* odd: result from rank-1 */
        run_copy(x, rbuf, P, (int64_t)count, FDEV_REMOTE_X, FDEV_TAG_STEP);
        c->stats.steps++;
    } else if (!x->out_done) { /* with one rank there is no exchange and rbuf = sbuf (:35-42) */
        run_copy(x, rbuf, x->steps == 0 ? IN : W, (int64_t)count, 0, FDEV_TAG_LOCAL);
    }
    ftar_drain(c);
    ftar_sync_fatal(c); /* peers are done reading our W before it is reused */
    ftar_stats_end(c);
    return FTAR_SUCCESS;
}

int ftar_allreduce_rabenseifner_host(const void *sbuf, void *rbuf, size_t count, ftar_dtype dtype, ftar_op op,
                                     ftar_comm *c)
{
    if (!c) return FTAR_ERR_ARG;
    int orc = ftar_check_op((int)dtype, (int)op); /* before anything is copied */
    if (orc) return orc;
    size_t es = ftar_esize(dtype);
    size_t bytes = count * es;
    /* Power of two without a spare (every failure aborts, so nothing is recovered across
     * calls): the vector goes through as a pipeline of chunk Allreduces -- chunk k's
     * H2D, chunk k-1's Allreduce and chunk k-2's D2H in flight at once (copy engines both
     * ways, xGMI) -- instead of H2D, Allreduce, D2H in turn.  Each chunk is a complete
     * fault-tolerant call (barriers, agree, abort).
     * Chunks move the block boundaries, and an element's tree takes its operands in its
     * owner's order (src[j] = x_(owner ^ j)): the unordered tree is the same for every
     * owner, so the bits are too wherever the op commutes exactly -- integers, float
     * SUM/PROD -- but not float MAX/MIN (NaN, signed zeros), which stay one call. */
    int p = c->size;
    int nchunk = 1;
    int commutes = dtype == FTAR_INT32 || dtype == FTAR_INT64 || op == FTAR_SUM || op == FTAR_PROD;
    if (c->host_pipe && commutes && c->redundancy != 1 && c->loop_seconds <= 0 && p >= 2 && (p & (p - 1)) == 0 &&
        bytes >= HOST_PIPE_MIN) {
        nchunk = (int)(bytes / HOST_PIPE_CHUNK);
        if (nchunk > HOST_PIPE_MAX) nchunk = HOST_PIPE_MAX;
    }
    /* Not pipelined and the caller's buffers pinned: the device entry point reads sbuf and
     * writes rbuf in place over PCIe, no staging copies */
    if (nchunk <= 1 && fdev_host_pinned(sbuf) && fdev_host_pinned(rbuf))
        return ftar_allreduce_rabenseifner(sbuf, rbuf, count, dtype, op, c);
    ftar_ensure_staging(c, bytes);
    if (nchunk <= 1) {
        if (bytes && fdev_h2d(c->dev, c->hsend, sbuf, bytes)) ftar_host_copy_failed(c, "H2D copy");
        int rc = ftar_allreduce_rabenseifner(c->hsend, c->hrecv, count, dtype, op, c);
        if (rc) return rc;
        if (bytes && fdev_d2h(c->dev, rbuf, c->hrecv, bytes)) ftar_host_copy_failed(c, "D2H copy");
        return FTAR_SUCCESS;
    }
    size_t per = (count + (size_t)nchunk - 1) / (size_t)nchunk;
    per = (per + 63) / 64 * 64; /* chunk boundaries on 256-byte multiples */
    int n = 0;
    for (size_t off = 0; off < count; off += per, n++) {
        size_t m = count - off < per ? count - off : per;
        if (fdev_h2d_async(c->dev, (char *)c->hsend + off * es, (const char *)sbuf + off * es, m * es, n))
            ftar_host_copy_failed(c, "H2D copy");
    }
    n = 0;
    for (size_t off = 0; off < count; off += per, n++) {
        size_t m = count - off < per ? count - off : per;
        if (fdev_wait_h2d(c->dev, n, ftar_ctrl_poll, &c->job)) ftar_host_copy_failed(c, "H2D copy");
        c->chunk_cont = n > 0;
        int rc = ftar_allreduce_rabenseifner((char *)c->hsend + off * es, (char *)c->hrecv + off * es, m, dtype, op,
                                             c);
        c->chunk_cont = 0;
        if (rc) return rc;
        if (fdev_d2h_async(c->dev, (char *)rbuf + off * es, (char *)c->hrecv + off * es, m * es))
            ftar_host_copy_failed(c, "D2H copy");
    }
    if (fdev_sync_d2h(c->dev, ftar_ctrl_poll, &c->job)) ftar_host_copy_failed(c, "D2H copy");
    return FTAR_SUCCESS;
}
