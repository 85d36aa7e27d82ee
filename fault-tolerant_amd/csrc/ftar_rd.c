/*
 * ftar_rd.c -- fault-tolerant recursive-doubling Allreduce on MI355X (per rank, host C).
 *
 * Restates src/rd/recursive_doubling.c:6-90, src/rd/util.c:3-95 and
 * src/rd/errhandler.c:6-302.  Each MPI_Sendrecv + MPI_Reduce_local of a step becomes
 * one kernel that reads the partner's accumulator over xGMI and writes the sum into
 * this rank's other ping-pong buffer:
 *
 *   middle steps (:42-49, Reduce_local(dst, src)):  A' = A + peer.A
 *   last step    (:42-44, Reduce_local(src, dst)):  A' = peer.A + A   (operand roles kept)
 *
 * The reference accumulates in src (clobbering it) and receives into dst; here src is
 * never written: the accumulator ping-pongs between the exported buffers W and T and
 * each rank publishes which one holds its value at every barrier, so a peer never
 * reads a buffer that is being written.
 *
 * Data (rd/header.h:16-26) is call-local: active/inactive lists of original ranks,
 * identical on every rank because every rank applies the same decisions to the same
 * agreed failure set.
 *
 * Deviation: the master search of the spare branch (errhandler.c:96-111)
 * never advances `j` and loops forever; the build implements its evident intent (the
 * master of each block of distance/2 ranks is its first rank that is alive and whose
 * partner of the failed step is alive).  Cases where the reference reads
 * uninitialised ranks or waits forever in the fan-out abort instead.
 */
#include "ftar_internal.h"

#include <stdio.h>
#include <string.h>

typedef struct {
    ftar_comm *c;
    int dtype, op;
    size_t es, count;
    int active[FTAR_MAX_RANKS], nactive;
    int inactive[FTAR_MAX_RANKS], ninactive;
    int cur; /* WS_* buffer holding this rank's accumulator */
} rd_ctx;

static int index_of(const int *a, int n, int w)
{
    for (int i = 0; i < n; i++)
        if (a[i] == w) return i;
    return -1;
}

static int in_set(uint64_t set, int w) { return (int)((set >> w) & 1u); }

/* the accumulator's buffer id is published at every sync (ftar_sync) and read back
 * for the round that just completed, so a fast rank's next value never races a slow
 * reader */
static void publish_cur(rd_ctx *x) { x->c->pubval = x->cur; }

static int peer_cur(rd_ctx *x, int w) { return (int)ftar_peer_pub(x->c, w); }

/* A pull's source buffer when planning a step: a rank that died before the last agree left no
 * entry for it -- its death surfaces at the step's own agree and reaches the handler there, as
 * the reference's first Sendrecv with it would (rd/recursive_doubling.c:35-56); the pull from
 * it is never made (its partner skips the exchange), so any buffer will do. */
static int peer_cur_plan(rd_ctx *x, int w)
{
    int64_t v;
    return ftar_peer_pub_try(x->c, w, &v) ? (int)v : x->cur;
}

static void run1(rd_ctx *x, int kind, void *out, const void *a, const void *b, int remote, int tag)
{
    fdev_seg s = {kind, remote, out, a, b, x->count, NULL};
    ftar_run(x->c, x->dtype, x->op, &s, 1, tag);
}

/* Every active rank's pull at the step of `distance` (recursive_doubling.c:35-49): middle
 * steps src = dst + src (Reduce_local(dst, src)), the last step dst = src + dst
 * (Reduce_local(src, dst)) -- the pulled operand first.  This rank reads its accumulator
 * from buffer `cur` and writes the other ping-pong buffer (returned); a partner's
 * accumulator is where it published it, or in buffer `pred` (>= 0) when the plan is made
 * ahead of the barrier that publishes it (every rank's buffers alternate alike). */
static int rd_plan(rd_ctx *x, int distance, int cur, int pred, ftar_plan *P)
{
    ftar_comm *c = x->c;
    int last = (distance * 2 >= x->nactive);
    int i = index_of(x->active, x->nactive, c->wrank);
    int out = (cur == WS_W) ? WS_T : WS_W;
    ftar_plan_clear(P);
    for (int a = 0; a < x->nactive; a++) {
        int cr = ftar_comm_rank_of(c, x->active[a]);
        int pw = x->active[a ^ distance];
        ftar_pull *pl = &P->pull[cr][0];
        *pl = (ftar_pull){FDEV_REDUCE, last, pw, pred >= 0 ? pred : peer_cur_plan(x, pw), 0, 0, 0, (int64_t)x->count, 0};
        if (a == i) {
            pl->dst_buf = out;
            pl->x_buf = cur;
            pl->to_uout = last; /* the result also lands in dst (no final copy) */
        }
        P->npull[cr] = 1;
    }
    return out;
}

/* The segments of this rank's step at `distance` planned ahead (rd_plan with `pred`), into
 * g; 0 if that step would be relayed (never queued ahead) or this rank pulls nothing. */
static int rd_plan_ahead(rd_ctx *x, int distance, int cur, int pred, int tag, struct ftar_gplan *g)
{
    ftar_plan P;
    rd_plan(x, distance, cur, pred, &P);
    g->valid = 0;
    if (ftar_xfer_would_relay(x->c, &P, x->es)) return 0;
    g->nseg = ftar_xfer_direct_segs(x->c, &P, x->es, g->segs, 0);
    g->dtype = x->dtype;
    g->op = x->op;
    g->tag = tag;
    g->valid = g->nseg > 0;
    return g->valid;
}

/* pull the accumulator of original rank `from` into a free buffer of this rank */
static void restore_from(rd_ctx *x, int from)
{
    ftar_comm *c = x->c;
    int dst = (x->cur == WS_IN) ? WS_W : x->cur;
    run1(x, FDEV_COPY, c->ws[dst], ftar_buf(c, from, peer_cur(x, from)), NULL, FDEV_REMOTE_X, FDEV_TAG_RECOV);
    x->cur = dst;
}

/* errhandler (rd/errhandler.c:6-302); `distance` is the caller's doubled distance.
 * Returns the possibly reduced distance. */
static int rd_handler(rd_ctx *x, uint64_t F, int distance)
{
    ftar_comm *c = x->c;
    int d = distance / 2;
    int nf = __builtin_popcountll(F);
    int me = c->wrank;

    /* shift out failed inactive ranks (:47-65) */
    int inactive_nf = 0, k = 0;
    for (int i = 0; i < x->ninactive; i++) {
        if (in_set(F, x->inactive[i])) inactive_nf++;
        else x->inactive[k++] = x->inactive[i];
    }
    x->ninactive = k;

    int active_failed = 0;
    for (int i = 0; i < x->nactive; i++)
        if (in_set(F, x->active[i])) active_failed = 1;

    if (active_failed) {
        int nfa = nf - inactive_nf;
        if (nfa >= d) { /* check_abort (util.c:49-78) */
            int cnt = 0;
            for (int i = 0; i < x->nactive; i++) {
                if (i % distance == 0) cnt = 0;
                if (in_set(F, x->active[i]) || in_set(F, x->active[i ^ d])) cnt++;
                if (cnt == distance) ftar_abort(c, FTAR_ERR_OTHER);
            }
        }
        if (nfa <= x->ninactive) {
            /* spare branch (:78-177): wake spares, restore corrupted partners */
            int master[FTAR_MAX_RANKS];
            for (int b = 0; b * d < x->nactive; b++) {
                master[b] = -1;
                for (int i = b * d; i < (b + 1) * d && i < x->nactive; i++)
                    if (!in_set(F, x->active[i]) && !in_set(F, x->active[i ^ d])) {
                        master[b] = i;
                        break;
                    }
            }
            int j = x->ninactive - 1;
            for (int i = 0; i < x->nactive; i++) {
                if (!in_set(F, x->active[i])) continue;
                int m = master[i / d];
                if (m < 0) ftar_abort(c, FTAR_ERR_OTHER); /* no healthy rank to restore from */
                int spare = x->inactive[j];
                if (me == spare) restore_from(x, x->active[m]); /* woken (:240-244) */
                int corr = i ^ d;
                if (!in_set(F, x->active[corr])) { /* corrupted partner (:147-162, :245-249) */
                    int mc = master[corr / d];
                    if (mc < 0) ftar_abort(c, FTAR_ERR_OTHER);
                    if (me == x->active[corr]) restore_from(x, x->active[mc]);
                }
                x->active[i] = spare;
                j--;
            }
            x->ninactive = j + 1;
            ftar_drain(c);
            publish_cur(x);
        } else {
            /* shrink to the next lower power of two (:178-217) */
            int p = ftar_floor_pow2(x->nactive - nfa);
            int kk = x->nactive / p;
            int newdist = distance / kk;
            int blk = newdist * kk;
            int newarr[FTAR_MAX_RANKS], total = 0, bc = 0;
            int extra[FTAR_MAX_RANKS], nextra = 0;
            for (int i = 0; i < x->nactive; i++) {
                if (i % blk == 0) bc = 0;
                if (in_set(F, x->active[i])) continue;
                if (bc < newdist && !in_set(F, x->active[i ^ (blk / 2)])) {
                    newarr[total++] = x->active[i];
                    bc++;
                } else {
                    extra[nextra++] = x->active[i];
                }
            }
            if (total < p) ftar_abort(c, FTAR_ERR_OTHER); /* reference: uninitialised ranks */
            for (int i = 0; i < nextra; i++) x->inactive[x->ninactive++] = extra[i];
            memcpy(x->active, newarr, sizeof(int) * (size_t)p);
            x->nactive = p;
            distance = newdist;
        }
    }
    c->acked |= F;
    ftar_shrink(c, F); /* MPIX_Comm_shrink of the world (:43-45) */
    ftar_sync_fatal(c); /* errhandler's closing barrier (:299) */
    c->stats.recoveries++;
    return distance;
}

int ftar_recursive_doubling(const void *src, void *dst, size_t count, ftar_dtype dtype, ftar_op op, ftar_comm *c)
{
    if (!c) return FTAR_ERR_ARG;
    rd_ctx X;
    memset(&X, 0, sizeof(X));
    rd_ctx *x = &X;
    x->c = c;
    x->dtype = (int)dtype;
    x->op = (int)op;
    x->es = ftar_esize(dtype);
    x->count = count;
    int orc = ftar_check_op((int)dtype, (int)op);
    if (orc) return orc;
    if (count && (!src || !dst)) return FTAR_ERR_ARG;
    if (count == 0) return FTAR_SUCCESS;
    /* device pointers: pageable host memory or a short allocation is refused, not faulted on */
    if (fdev_check_ptr(c->dev, src, count * x->es) || fdev_check_ptr(c->dev, dst, count * x->es))
        return FTAR_ERR_ARG;
    c->uin = src;
    c->uout = dst;
    ftar_stats_begin(c);
    if (c->size == 1) return ftar_single_rank(c, src, dst, count * x->es);
    int me = c->wrank;

    size_t bytes = count * x->es;
    ftar_ensure_workspace(c, bytes);
    fdev_order_after(c->dev, c->user_stream);
    /* Nothing writes IN after this: the peers read src in place when its memory can be
     * shared -- unless it overlaps dst, which the last step writes while (with a single
     * step) the partner may still be reading IN. */
    const char *s0 = (const char *)src, *d0 = (const char *)dst;
    int disjoint = s0 + bytes <= d0 || d0 + bytes <= s0;
    int staged = !ftar_stage_input(c, src, bytes, disjoint);
    x->cur = WS_IN;

    /* Data + reduce_pow2 (recursive_doubling.c:118-130, util.c:3-34) */
    int size = c->size;
    int pp = ftar_floor_pow2(size);
    x->nactive = pp;
    for (int i = 0; i < pp; i++) x->active[i] = c->order[i];
    x->ninactive = size - pp;
    for (int i = pp; i < size; i++) x->inactive[i - pp] = c->order[i];
    /* Small and mid-size calls at a power of two (no pre-step): each step's launch is queued
     * ahead of the barrier that readies its operands, behind a gate (ftar_prelaunch) -- step
     * 0's right behind the staging copy (every rank stages a small input, so the partners'
     * inputs will be in their IN), step s + 1's behind step s's (the accumulators alternate
     * W, T, W, ... on every rank).  The step then runs it only if its own plan, made after
     * the barrier, is the same (ftar_xfer_step); a recovery in between makes it a plain launch. */
    /* Mid-size vectors (up to FTAR_GATE_MAX) queue steps 1.. ahead too -- their operands are
     * the peers' accumulators, predictable -- while step 0 reads the peers' inputs, which
     * only small staged calls can predict (a larger input is read in place, where the
     * peer's mapping is known after the barrier only). */
    int ahead = c->gate && x->ninactive == 0 && pp >= 2 && bytes <= c->gate_max && !c->copy_engine;
    int folded = 0; /* the staging copy rides in step 0's gated launch, ahead of its gate */
    if (ahead && staged && bytes <= c->stage_max && rd_plan_ahead(x, 1, WS_IN, WS_IN, FDEV_TAG_STEP0, &c->gnext)) {
        c->gnext.valid = 0;
        folded = ftar_prelaunch(c, c->gnext.dtype, c->gnext.op, c->gnext.segs, c->gnext.nseg, c->gnext.tag,
                                c->ws[WS_IN], src, count);
        if (folded) ftar_note_launch(c, NULL, 0); /* the staging phase is in flight */
    }
    if (staged && !folded) run1(x, FDEV_COPY, c->ws[WS_IN], src, NULL, 0, FDEV_TAG_LOCAL);
    ftar_drain(c);
    publish_cur(x);
    uint64_t involved = 0; /* ranks with a pre-step exchange (errors there are fatal) */
    for (int r = 0; r < x->ninactive; r++) involved |= (1ull << x->active[r]) | (1ull << x->inactive[r]);

    ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_BEFORE);
    uint64_t newf = ftar_sync(c); /* every IN is ready */
    if (newf & involved) ftar_abort(c, FTAR_ERR_PROC_FAILED);
    ftar_resolve_inputs(c);
    ftar_enter(c);
    int ia = index_of(x->active, x->nactive, me);
    int pre = ia >= 0 && ia < x->ninactive;
    if (pre) {
        const void *P = ftar_buf(c, x->inactive[ia], WS_IN);
        run1(x, FDEV_REDUCE, c->ws[WS_W], ftar_local(c, WS_IN), P, FDEV_REMOTE_Y, FDEV_TAG_STEP); /* src = dst + src */
    }
    ftar_launched(c, FTAR_PH_PRE, 0);
    if (pre) {
        ftar_drain(c);
        x->cur = WS_W;
        publish_cur(x);
        c->stats.steps++;
    }
    ftar_exchange_done(c);
    ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_AFTER);
    ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_BARRIER);
    newf = ftar_sync(c); /* MPI_Barrier after switching to ERRORS_RETURN (:16-18) */
    if (newf & involved) ftar_abort(c, FTAR_ERR_PROC_FAILED);

    /* recursive doubling body (:21-71) */
    int iter = 0, dst_done = 0;
    for (int distance = 1; distance < x->nactive; distance *= 2, iter++) {
        int last = (distance * 2 >= x->nactive);
        int i = index_of(x->active, x->nactive, me);
        /* every active rank's pull (ftar_xfer stripes it over relays when large) */
        ftar_plan P;
        ftar_xstate xs;
        int out = rd_plan(x, distance, x->cur, -1, &P);
        /* the next step's launch, queued gated behind this one's (see `ahead`) */
        if (ahead && i >= 0 && !last) rd_plan_ahead(x, distance * 2, out, out, FDEV_TAG_STEP, &c->gnext);
        ftar_maybe_die(c, FTAR_PH_LOOP, iter, FTAR_PT_BEFORE);
        ftar_enter(c);
        int skip = 0;
        if (i >= 0) {
            skip = !ftar_peer_entered(c, x->active[i ^ distance]); /* corrupted (:35-49 ignore the error) */
            c->stats.steps++;
        }
        double lb0 = ftar_link_bytes(c);
        ftar_xfer_step(c, &P, x->dtype, x->op, iter == 0 ? FDEV_TAG_STEP0 : FDEV_TAG_STEP, skip, FTAR_PH_LOOP, iter,
                       NULL, 0, &xs);
        if (iter == 0) c->stats.step0_link_bytes += ftar_link_bytes(c) - lb0;
        if (i >= 0 && !skip) {
            x->cur = out;
            publish_cur(x);
        }
        ftar_maybe_die(c, FTAR_PH_LOOP, iter, FTAR_PT_BARRIER);
        newf = ftar_step_sync(c, ftar_hibit(x->nactive, 31) > 0 ? ftar_hibit(x->nactive, 31) : 1); /* (:51-53) */
        dst_done = last && i >= 0 && !skip && !newf; /* a recovery may move on: copy at the end */
        if (newf) {
            ftar_xfer_repair(c, &P, x->dtype, x->op, &xs, newf);
            int dd = rd_handler(x, newf, distance * 2);
            distance = dd / 2;
        }
    }

    /* ERRORS_ARE_FATAL barrier (:73-75), then the fan-out to inactive ranks (:78-89) */
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BEFORE);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_DURING);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_AFTER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BARRIER);
    ftar_sync_fatal(c);
    if (x->ninactive > x->nactive) ftar_abort(c, 1); /* reference: inactive ranks wait forever */
    int ii = index_of(x->inactive, x->ninactive, me);
    if (ii >= 0) {
        int from = x->active[ii];
        run1(x, FDEV_COPY, dst, ftar_buf(c, from, peer_cur(x, from)), NULL, FDEV_REMOTE_X, FDEV_TAG_STEP);
        c->stats.steps++;
    } else if (!dst_done) {
        run1(x, FDEV_COPY, dst, ftar_local(c, x->cur), NULL, 0, FDEV_TAG_LOCAL);
    }
    ftar_drain(c);
    ftar_sync_fatal(c); /* main's MPI_Barrier (:134); peers are done reading */
    ftar_stats_end(c);
    return FTAR_SUCCESS;
}

int ftar_recursive_doubling_host(const void *src, void *dst, size_t count, ftar_dtype dtype, ftar_op op,
                                 ftar_comm *c)
{
    if (!c) return FTAR_ERR_ARG;
    int orc = ftar_check_op((int)dtype, (int)op); /* before anything is copied */
    if (orc) return orc;
    size_t es = ftar_esize(dtype);
    size_t bytes = count * es;
    /* pinned caller buffers: the device entry point reads src and writes dst in place over
     * PCIe (the last step's result goes straight to dst), no staging copies */
    if (fdev_host_pinned(src) && fdev_host_pinned(dst)) return ftar_recursive_doubling(src, dst, count, dtype, op, c);
    ftar_ensure_staging(c, bytes);
    if (bytes && fdev_h2d(c->dev, c->hsend, src, bytes)) ftar_host_copy_failed(c, "H2D copy");
    int rc = ftar_recursive_doubling(c->hsend, c->hrecv, count, dtype, op, c);
    if (rc) return rc;
    if (bytes && fdev_d2h(c->dev, dst, c->hrecv, bytes)) ftar_host_copy_failed(c, "D2H copy");
    return FTAR_SUCCESS;
}
