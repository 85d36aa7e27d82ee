/*
 * ftar_xfer.c -- the exchange transport of one schedule step.
 *
 * Both schedules are pairwise: at every step each receiving rank pulls one window (or
 * two, Raben step 0) from ONE partner, so only one of the 7 xGMI links of an MI355X
 * is busy per step.  For large windows the pull is striped over 2-hop paths through
 * the other receivers of the step:
 *
 *   phase 1  (one kernel per rank)  rank X pulls stripe 0 of its own window directly
 *            from its partner, and, for every other receiver Y, copies Y's stripe j
 *            (X being Y's j-th relay) out of Y's partner's HBM into X's relay buffer R;
 *   barrier  (agree round: a relay that died before it is known to every rank);
 *   phase 2  Y pulls its relayed stripes from the relays' R buffers and reduces (or
 *            copies) them into its window, and its last stripe directly from its
 *            partner (that link is otherwise idle in phase 2).
 *
 * A window is cut into r stripes (r receivers): two direct ones (one per phase) and
 * r - 2 relayed ones.  Every link of a rank then carries 1/r of a window per phase
 * instead of the whole window on one link: for r = 8 a step costs about 2/8 of the
 * direct exchange.  Results are bit-identical to the direct pull: every element is still
 * combined once, with the same operands in the same roles.
 *
 * Faults: the pulled data is always the partner's window, stable since the previous
 * barrier, so any stripe can be re-pulled.  Stripes of relays that died before the
 * mid-step barrier are skipped in phase 2 and re-pulled directly after the step's agree
 * (ftar_xfer_repair), so the state the reference's error handlers see is exactly the
 * state of a direct exchange.  A receiver whose partner was dead at the start of the
 * step skips all of its stripes (the reference's `corr`).
 */
#include "ftar_internal.h"

#include <stdio.h>
#include <string.h>

#define STRIPE_ALIGN 256 /* elements; interior stripe boundaries are multiples of this */
#define SLOT_PAD 64      /* elements; a relay slot keeps its source's offset modulo this */
#define MAX_RELAY_RECEIVERS 8

void ftar_plan_clear(ftar_plan *p) { memset(p->npull, 0, sizeof(p->npull)); }

static int receivers(const ftar_comm *c, const ftar_plan *p, int *R)
{
    int n = 0;
    for (int y = 0; y < c->size; y++)
        if (p->npull[y] > 0) R[n++] = y;
    return n;
}

/* relays of receiver y (comm ranks): every other receiver but y's partner */
static int relays_of(const ftar_comm *c, const ftar_plan *p, const int *R, int nr, int y, int *out)
{
    int src = ftar_comm_rank_of(c, p->pull[y][0].src);
    int k = 0;
    for (int i = 0; i < nr; i++)
        if (R[i] != y && R[i] != src) out[k++] = R[i];
    return k;
}

/* stripes of a window with k relays: 0 = direct in phase 1, 1..k relayed (relay j-1),
 * k + 1 = direct in phase 2 */
static int nstripes(int k) { return k + 2; }

static void stripe(const ftar_pull *pl, int nst, int j, int64_t *start, int64_t *len)
{
    int64_t base = (pl->n / nst) / STRIPE_ALIGN * STRIPE_ALIGN;
    *start = pl->off + (int64_t)j * base;
    *len = (j < nst - 1) ? base : pl->n - (int64_t)(nst - 1) * base;
}

static int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

/* Element offset in X's relay buffer of (receiver y, pull u); also returns X's total
 * relay footprint in *total.  Every rank evaluates the same enumeration. */
static int64_t slot_of(const ftar_comm *c, const ftar_plan *p, const int *R, int nr, int X, int y, int u,
                       int64_t *total)
{
    int64_t off = 0, found = -1;
    int rel[FTAR_MAX_RANKS];
    for (int i = 0; i < nr; i++) {
        int yy = R[i];
        if (yy == X) continue;
        int k = relays_of(c, p, R, nr, yy, rel);
        int idx = -1;
        for (int t = 0; t < k; t++)
            if (rel[t] == X) idx = t;
        if (idx < 0) continue;
        for (int uu = 0; uu < p->npull[yy]; uu++) {
            int64_t st, len;
            stripe(&p->pull[yy][uu], nstripes(k), idx + 1, &st, &len);
            int64_t slot = round_up(off, SLOT_PAD) + (st % SLOT_PAD);
            if (yy == y && uu == u) found = slot;
            off = slot + len;
        }
    }
    if (total) *total = off;
    return found;
}

int ftar_xfer_would_relay(ftar_comm *c, const ftar_plan *p, size_t es)
{
    if (!c->relay) return 0;
    int R[FTAR_MAX_RANKS];
    int nr = receivers(c, p, R);
    if (nr < 3 || nr > MAX_RELAY_RECEIVERS) return 0;
    for (int i = 0; i < nr; i++)
        for (int u = 0; u < p->npull[R[i]]; u++)
            if ((size_t)p->pull[R[i]][u].n * es < c->relay_min) return 0;
    for (int i = 0; i < nr; i++) { /* every relay's staging fits its R buffer */
        int64_t total = 0;
        slot_of(c, p, R, nr, R[i], -1, -1, &total);
        if ((size_t)total * es > c->ws_bytes) return 0;
    }
    return 1;
}

static char *at(void *base, int64_t idx, size_t es) { return (char *)base + (size_t)idx * es; }

/* segment for [st, st+len) of pull pl at this rank, pulled operand at `pulled` (already
 * offset to the stripe start) */
static fdev_seg own_seg(ftar_comm *c, const ftar_pull *pl, int64_t st, int64_t len, const void *pulled,
                        size_t es)
{
    fdev_seg s;
    memset(&s, 0, sizeof(s));
    s.kind = pl->kind;
    s.out = at(ftar_local(c, pl->dst_buf), st, es);
    if (pl->to_uout) s.out2 = at(c->uout, st, es);
    s.n = (size_t)len;
    if (pl->kind == FDEV_COPY) {
        s.x = pulled;
        s.remote = FDEV_REMOTE_X;
    } else if (pl->swap) {
        s.x = pulled;
        s.y = at(ftar_local(c, pl->x_buf), st, es);
        s.remote = FDEV_REMOTE_X;
    } else {
        s.x = at(ftar_local(c, pl->x_buf), st, es);
        s.y = pulled;
        s.remote = FDEV_REMOTE_Y;
    }
    return s;
}

/* staging slot in R for a segment whose output lies in IN, W or T (same offset) */
static void *staging_of(ftar_comm *c, const void *out)
{
    const char *o = (const char *)out;
    for (int b = WS_IN; b <= WS_T; b++) {
        const char *base = (const char *)c->ws[b];
        if (base && o >= base && o < base + c->ws_bytes) return (char *)c->ws[WS_R] + (o - base);
    }
    return NULL;
}

void ftar_run_pulls(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag, int bg)
{
    if (!c->copy_engine) {
        if (bg) ftar_run_bg(c, dtype, op, segs, nseg, tag);
        else ftar_run(c, dtype, op, segs, nseg, tag);
        return;
    }
    /* The reference's shape: the exchange is a copy (hipMemcpyAsync over xGMI, SDMA or
     * blit engine) and the reduce a separate local kernel over the received window. */
    size_t es = ftar_esize(dtype);
    fdev_seg local[FDEV_MAX_SEGS];
    int nl = 0;
    for (int i = 0; i < nseg; i++) {
        fdev_seg t = segs[i];
        int rc = 0;
        if (!t.remote) {
            local[nl++] = t;
        } else if (t.kind == FDEV_COPY) {
            ftar_note_launch(c, t.x, t.n * es);
            rc = fdev_copy(c->dev, bg, t.out, t.x, t.n * es, 1, tag);
            if (t.out2) /* the second destination from the landed copy (same stream) */
                local[nl++] = (fdev_seg){FDEV_COPY, 0, t.out2, t.out, NULL, t.n, NULL};
        } else {
            void *stage = staging_of(c, t.out);
            if (!stage) {
                local[nl++] = t;
                continue;
            }
            const void *src = (t.remote & FDEV_REMOTE_X) ? t.x : t.y;
            ftar_note_launch(c, src, t.n * es);
            rc = fdev_copy(c->dev, bg, stage, src, t.n * es, 1, tag);
            if (t.remote & FDEV_REMOTE_X) t.x = stage;
            else t.y = stage;
            t.remote = 0;
            local[nl++] = t;
        }
        if (rc) {
            fprintf(stderr, "ftar: rank %d: copy failed: %s\n", c->wrank, fdev_last_error());
            ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
        }
    }
    if (nl) {
        if (bg) ftar_run_bg(c, dtype, op, local, nl, tag);
        else ftar_run(c, dtype, op, local, nl, tag);
    }
}

int ftar_xfer_direct_segs(ftar_comm *c, const ftar_plan *p, size_t es, fdev_seg *segs, int ns)
{
    int me = ftar_my_comm_rank(c);
    for (int u = 0; u < p->npull[me]; u++) {
        const ftar_pull *pl = &p->pull[me][u];
        segs[ns++] = own_seg(c, pl, pl->off, pl->n, at(ftar_buf(c, pl->src, pl->src_buf), pl->off, es), es);
    }
    return ns;
}

void ftar_xfer_step(ftar_comm *c, const ftar_plan *p, int dtype, int op, int tag, int skip, int kphase, int kstep,
                    const fdev_seg *extra, int nextra, ftar_xstate *xs)
{
    size_t es = ftar_esize(dtype);
    int me = ftar_my_comm_rank(c);
    memset(xs, 0, sizeof(*xs));
    xs->skipped = skip;
    fdev_seg segs[FDEV_MAX_SEGS];
    int ns = 0;
    for (int i = 0; i < nextra; i++) segs[ns++] = extra[i];
    if (!ftar_xfer_would_relay(c, p, es)) { /* direct pull of the whole window */
        if (!skip) ns = ftar_xfer_direct_segs(c, p, es, segs, ns);
        /* a launch queued for this step ahead of its barrier runs if it was planned with
         * these very segments (ftar_run_gated_or), else it is replaced */
        if (!c->copy_engine && (c->gplan.valid || fdev_gate_pending(c->dev))) ftar_run_gated_or(c, dtype, op, segs, ns, tag);
        else if (ns) ftar_run_pulls(c, dtype, op, segs, ns, tag, 0);
        if (c->gnext.valid) { /* the next step's launch, queued gated behind this one */
            c->gnext.valid = 0;
            ftar_prelaunch(c, c->gnext.dtype, c->gnext.op, c->gnext.segs, c->gnext.nseg, c->gnext.tag, NULL, NULL, 0);
        }
        ftar_launched(c, kphase, kstep); /* FTAR_PT_DURING: our pulls and the partner's in flight */
        if (ns) ftar_drain(c);
        ftar_exchange_done(c);
        ftar_maybe_die(c, kphase, kstep, FTAR_PT_AFTER);
        return;
    }
    xs->relayed = 1;
    c->stats.relayed_steps++;
    c->gnext.valid = 0; /* relayed steps are never queued ahead (their first launch gives up any gate) */
    if (c->gplan.valid) {
        c->gplan.valid = 0;
        c->stats.gated_skips++;
    }
    int R[FTAR_MAX_RANKS], rel[FTAR_MAX_RANKS];
    int nr = receivers(c, p, R);
    /* phase 1: own stripe 0 + relay duties */
    if (!skip && p->npull[me] > 0) {
        int k = relays_of(c, p, R, nr, me, rel);
        for (int u = 0; u < p->npull[me]; u++) {
            const ftar_pull *pl = &p->pull[me][u];
            int64_t st, len;
            stripe(pl, nstripes(k), 0, &st, &len);
            if (len > 0) segs[ns++] = own_seg(c, pl, st, len, at(ftar_buf(c, pl->src, pl->src_buf), st, es), es);
        }
    }
    for (int i = 0; i < nr; i++) {
        int y = R[i];
        if (y == me) continue;
        int k = relays_of(c, p, R, nr, y, rel);
        int idx = -1;
        for (int t = 0; t < k; t++)
            if (rel[t] == me) idx = t;
        if (idx < 0) continue;
        for (int u = 0; u < p->npull[y]; u++) {
            const ftar_pull *pl = &p->pull[y][u];
            int64_t st, len;
            stripe(pl, nstripes(k), idx + 1, &st, &len);
            if (len <= 0) continue;
            int64_t slot = slot_of(c, p, R, nr, me, y, u, NULL);
            fdev_seg s;
            memset(&s, 0, sizeof(s));
            s.kind = FDEV_COPY;
            s.remote = FDEV_REMOTE_X;
            s.out = at(c->ws[WS_R], slot, es);
            s.x = at(ftar_buf(c, pl->src, pl->src_buf), st, es);
            s.n = (size_t)len;
            segs[ns++] = s;
        }
    }
    if (ns) ftar_run(c, dtype, op, segs, ns, tag);
    ftar_launched(c, kphase, kstep); /* FTAR_PT_DURING: phase-1 pulls (ours and the relays') in flight */
    if (ns) ftar_drain(c);
    /* this rank's side of the exchange is complete once its phase 1 drained: a death
     * after this point (AFTER) leaves the partner's exchange intact, as in the direct form */
    ftar_exchange_done(c);
    ftar_maybe_die(c, kphase, kstep, FTAR_PT_AFTER);
    /* mid-step barrier: relays that died before finishing phase 1 are known to all */
    xs->mid_dead = ftar_sync(c);
    /* phase 2: gather the relayed stripes */
    ns = 0;
    if (!skip && p->npull[me] > 0) {
        int k = relays_of(c, p, R, nr, me, rel);
        for (int u = 0; u < p->npull[me]; u++) {
            const ftar_pull *pl = &p->pull[me][u];
            for (int t = 0; t < k; t++) {
                int64_t st, len;
                stripe(pl, nstripes(k), t + 1, &st, &len);
                if (len <= 0) continue;
                int xw = c->order[rel[t]];
                if (xs->mid_dead & (1ull << xw)) {
                    xs->missing = 1;
                    continue;
                }
                int64_t slot = slot_of(c, p, R, nr, rel[t], me, u, NULL);
                segs[ns++] = own_seg(c, pl, st, len, at(ftar_buf(c, xw, WS_R), slot, es), es);
            }
            int64_t st, len; /* the phase-2 direct stripe (the partner's window is stable) */
            stripe(pl, nstripes(k), k + 1, &st, &len);
            if (len > 0) segs[ns++] = own_seg(c, pl, st, len, at(ftar_buf(c, pl->src, pl->src_buf), st, es), es);
        }
    }
    if (ns) {
        ftar_run(c, dtype, op, segs, ns, tag);
        ftar_drain(c);
    }
}

void ftar_xfer_repair(ftar_comm *c, const ftar_plan *p, int dtype, int op, ftar_xstate *xs, uint64_t known)
{
    if (!xs->relayed || !xs->mid_dead) return; /* uniform: every rank saw the same mid_dead */
    size_t es = ftar_esize(dtype);
    int me = ftar_my_comm_rank(c);
    if (xs->missing && !xs->skipped) {
        int R[FTAR_MAX_RANKS], rel[FTAR_MAX_RANKS];
        int nr = receivers(c, p, R);
        int k = relays_of(c, p, R, nr, me, rel);
        fdev_seg segs[FDEV_MAX_SEGS];
        int ns = 0;
        for (int u = 0; u < p->npull[me]; u++) {
            const ftar_pull *pl = &p->pull[me][u];
            for (int t = 0; t < k; t++) {
                if (!(xs->mid_dead & (1ull << c->order[rel[t]]))) continue;
                int64_t st, len;
                stripe(pl, nstripes(k), t + 1, &st, &len);
                if (len > 0)
                    segs[ns++] = own_seg(c, pl, st, len, at(ftar_buf(c, pl->src, pl->src_buf), st, es), es);
            }
        }
        if (ns) {
            ftar_run(c, dtype, op, segs, ns, FDEV_TAG_RECOV);
            ftar_drain(c);
        }
    }
    uint64_t f = ftar_sync(c); /* windows are whole again on every rank */
    if (f & ~known) ftar_abort(c, FTAR_ERR_PROC_FAILED);
}
