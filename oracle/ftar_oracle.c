/*
 * ftar_oracle.c -- CPU restatement (test infrastructure only, see ftar_oracle.h).
 *
 * The reference runs one MPI process per rank and synchronises with
 * MPIX_Comm_agree + MPI_Barrier after every exchange step.  Because every step is
 * bracketed by that barrier, the whole job can be replayed as a lockstep global
 * simulation: per step, every rank first "sends" (snapshot of the sender's buffer
 * taken before anyone reduces, as MPI_Sendrecv does), then every rank reduces, then
 * the barrier decides whether an error handler runs.  Error handlers are restated as
 * the global effect of their point-to-point messages.
 *
 * Compile with -ffp-contract=off and without fast-math: each element is reduced with
 * exactly one IEEE operation per tree node, which is what makes the GPU build
 * bit-exact to this file.
 */
#include "ftar_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* element operations                                                         */
/* ------------------------------------------------------------------------- */

size_t ftar_oracle_esize(int dtype)
{
    switch (dtype) {
    case FTAR_INT32: return 4;
    case FTAR_FLOAT32: return 4;
    case FTAR_INT64: return 8;
    case FTAR_FLOAT64: return 8;
    default: return 0;
    }
}

/* OpenMPI's 2-buffer ops compute out = out <op> in, and for MAX/MIN
 * out = (out > in) ? out : in  (ompi/mca/op/base/op_base_functions.c).  The
 * reference only ever uses MPI_SUM; the other ops follow the same operand roles.
 * MPI's logical ops (LAND, LOR, LXOR) yield 0 / 1, the bitwise ones (BAND, BOR, BXOR)
 * act on the two's-complement bits; both exist for the integer types only
 * (MPI 4.1 section 6.9.2), which ftar_oracle_reduce_local enforces. */
#define ARITH_CASES(T, UT)                                                        \
    case FTAR_SUM:                                                                \
        for (i = 0; i < n; i++) inout[i] = (T)((UT)inout[i] + (UT)in[i]);         \
        break;                                                                    \
    case FTAR_PROD:                                                               \
        for (i = 0; i < n; i++) inout[i] = (T)((UT)inout[i] * (UT)in[i]);         \
        break;                                                                    \
    case FTAR_MAX:                                                                \
        for (i = 0; i < n; i++) inout[i] = (inout[i] > in[i]) ? inout[i] : in[i]; \
        break;                                                                    \
    case FTAR_MIN:                                                                \
        for (i = 0; i < n; i++) inout[i] = (inout[i] < in[i]) ? inout[i] : in[i]; \
        break;
#define BIT_CASES(T)                                                              \
    case FTAR_LAND:                                                               \
        for (i = 0; i < n; i++) inout[i] = (T)(inout[i] != 0 && in[i] != 0);      \
        break;                                                                    \
    case FTAR_BAND:                                                               \
        for (i = 0; i < n; i++) inout[i] = (T)(inout[i] & in[i]);                 \
        break;                                                                    \
    case FTAR_LOR:                                                                \
        for (i = 0; i < n; i++) inout[i] = (T)(inout[i] != 0 || in[i] != 0);      \
        break;                                                                    \
    case FTAR_BOR:                                                                \
        for (i = 0; i < n; i++) inout[i] = (T)(inout[i] | in[i]);                 \
        break;                                                                    \
    case FTAR_LXOR:                                                               \
        for (i = 0; i < n; i++) inout[i] = (T)((inout[i] != 0) != (in[i] != 0)); \
        break;                                                                    \
    case FTAR_BXOR:                                                               \
        for (i = 0; i < n; i++) inout[i] = (T)(inout[i] ^ in[i]);                 \
        break;
#define DEF_REDUCE_INT(NAME, T, UT)                                               \
    static void NAME(int op, const T *in, T *inout, size_t n)                     \
    {                                                                             \
        size_t i;                                                                 \
        switch (op) { ARITH_CASES(T, UT) BIT_CASES(T) }                           \
    }
#define DEF_REDUCE_FLOAT(NAME, T)                                                 \
    static void NAME(int op, const T *in, T *inout, size_t n)                     \
    {                                                                             \
        size_t i;                                                                 \
        switch (op) { ARITH_CASES(T, T) }                                         \
    }

DEF_REDUCE_INT(reduce_i32, int32_t, uint32_t)
DEF_REDUCE_INT(reduce_i64, int64_t, uint64_t)
DEF_REDUCE_FLOAT(reduce_f32, float)
DEF_REDUCE_FLOAT(reduce_f64, double)

/* type/op check of MPI_Reduce_local: unknown -> MPI_ERR_ARG, logical or bitwise op on a
 * floating-point type -> MPI_ERR_OP */
static int check_op(int dtype, int op)
{
    if (ftar_oracle_esize(dtype) == 0 || op < FTAR_SUM || op >= FTAR_NOPS) return FTAR_ERR_ARG;
    if (op >= FTAR_LAND && (dtype == FTAR_FLOAT32 || dtype == FTAR_FLOAT64)) return FTAR_ERR_OP;
    return FTAR_SUCCESS;
}

int ftar_oracle_reduce_local(int dtype, int op, const void *in, void *inout, size_t n)
{
    int rc = check_op(dtype, op);
    if (rc) return rc;
    switch (dtype) {
    case FTAR_INT32: reduce_i32(op, (const int32_t *)in, (int32_t *)inout, n); break;
    case FTAR_INT64: reduce_i64(op, (const int64_t *)in, (int64_t *)inout, n); break;
    case FTAR_FLOAT32: reduce_f32(op, (const float *)in, (float *)inout, n); break;
    case FTAR_FLOAT64: reduce_f64(op, (const double *)in, (double *)inout, n); break;
    default: return FTAR_ERR_ARG;
    }
    return FTAR_SUCCESS;
}

int32_t ftar_oracle_checksum17(const int32_t *buf, size_t n)
{
    uint32_t res = 0; /* int accumulator of the reference, with defined wrap-around */
    for (size_t i = 0; i < n; i++) res += (uint32_t)(buf[i] % 17);
    return (int32_t)res;
}

int32_t ftar_oracle_checksum17_f32(const float *buf, size_t n)
{
    uint32_t res = 0;
    for (size_t i = 0; i < n; i++) res += (uint32_t)(((int32_t)buf[i]) % 17);
    return (int32_t)res;
}

/* ------------------------------------------------------------------------- */
/* simulation helpers                                                         */
/* ------------------------------------------------------------------------- */

typedef struct {
    int p;
    size_t count;
    int dtype, op;
    size_t es;
    const ftar_kill *kills;
    int nkills;
    ftar_oracle_result *res;
    int aborted;
} sim_t;

static unsigned char *ELEM(void *base, size_t idx, size_t es)
{
    return (unsigned char *)base + idx * es;
}

static void reduce_into(sim_t *s, void *inout, const void *in, size_t n)
{
    ftar_oracle_reduce_local(s->dtype, s->op, in, inout, n);
}

/* Poison a window whose receive failed: a corrupted partner's buffer must never
 * reach a survivor's result (float: quiet NaN, int: 0x5A5A...). */
static void poison(sim_t *s, void *buf, size_t n)
{
    if (s->dtype == FTAR_FLOAT32) {
        uint32_t v = 0x7fc0dead;
        for (size_t i = 0; i < n; i++) memcpy(ELEM(buf, i, 4), &v, 4);
    } else if (s->dtype == FTAR_FLOAT64) {
        uint64_t v = 0x7ff800000000deadull;
        for (size_t i = 0; i < n; i++) memcpy(ELEM(buf, i, 8), &v, 8);
    } else {
        memset(buf, 0x5A, n * s->es);
    }
}

/* A partner's Sendrecv with a rank that dies at kill point `kp` of the step failed: the
 * rank died before its exchange (BEFORE) or in the middle of it (DURING, a transfer cut
 * short: raben/rabenseifner.c:209-211 return an error, :238-241 mark corr).  A rank that
 * dies after its Sendrecv returned (AFTER, BARRIER) had delivered its data. */
static int failed_xchg(int kp) { return kp == FTAR_PT_BEFORE || kp == FTAR_PT_DURING; }

/* Does original rank w die at (phase, step)?  Returns the point or -1. */
static int kill_point(const sim_t *s, int w, int phase, int step)
{
    for (int k = 0; k < s->nkills; k++)
        if (s->kills[k].rank == w && s->kills[k].phase == phase && s->kills[k].step == step)
            return s->kills[k].point;
    return -1;
}

/* A failure in a region under MPI_ERRORS_ARE_FATAL (pre-step, post-step, the fatal barriers):
 * OpenMPI's fatal handler aborts the job with the failure's error class, MPIX_ERR_PROC_FAILED
 * (75; rd/recursive_doubling.c:56 hard-codes the same value for its own abort).  The handlers'
 * explicit aborts keep their codes: MPI_Abort(comm, 1) (raben/errhandler.c:38,211,322,378) and
 * 16 (rd/util.c:75). */
#define FATAL_CODE 75

static void do_abort(sim_t *s, int code)
{
    s->aborted = 1;
    s->res->aborted = 1;
    s->res->abort_code = code;
}

/* hibit(value, start) of raben/util.c:22-37 */
static int hibit(int value, int start)
{
    unsigned int mask = (unsigned int)value & ((1u << start) - 1u);
    if (mask == 0) return -1;
    return (int)(8 * sizeof(int) - 1) - __builtin_clz(mask);
}

/* ------------------------------------------------------------------------- */
/* Rabenseifner  (src/raben/rabenseifner.c:3-395, errhandler.c:3-468)          */
/* ------------------------------------------------------------------------- */

#define MAXSTEPS 32

typedef struct {
    int alive;
    unsigned char *sbuf; /* the rank's input after the pre-step (reference aligns sbuf=rbuf, :128) */
    unsigned char *rbuf;
    unsigned char *tmp;
    int vrank, corr;
    int rindex[MAXSTEPS], sindex[MAXSTEPS], rcount[MAXSTEPS], scount[MAXSTEPS];
    int wsize;
    /* 1 while the rank still plays the vrank it held at reduce-scatter step 0 and
     * therefore owns a valid step-0 copy of its partner's vector in tmp. */
    int has_recov;
} rb_rank;

typedef struct {
    sim_t *s;
    rb_rank *rk;    /* indexed by original rank */
    int order[FTAR_MAX_RANKS]; /* comm rank -> original rank */
    int size, steps, adjsize, rem;
} rb_t;

static int rb_real(const rb_t *b, int v) /* raben/rabenseifner.c:179-181 */
{
    return (v < b->rem) ? v * 2 : v + b->rem;
}

static void rb_vranks(rb_t *b) /* raben/rabenseifner.c:268-281 */
{
    for (int c = 0; c < b->size; c++) {
        rb_rank *r = &b->rk[b->order[c]];
        if (c < 2 * b->rem) r->vrank = (c % 2 == 0) ? c / 2 : -1;
        else r->vrank = c - b->rem;
    }
}

static int rb_comm_rank_of(const rb_t *b, int w)
{
    for (int c = 0; c < b->size; c++)
        if (b->order[c] == w) return c;
    return -1;
}

/* Window of comm rank `rank` at a step, given the partner comm rank `dest`
 * (raben/rabenseifner.c:182-203).  Arrays hold the window start on entry. */
static void rb_window(int rank, int dest, int step, int wsize, int *rindex, int *sindex,
                      int *rcount, int *scount)
{
    if (rank < dest) {
        rcount[step] = wsize / 2;
        scount[step] = wsize - rcount[step];
        sindex[step] = rindex[step] + rcount[step];
    } else {
        scount[step] = wsize / 2;
        rcount[step] = wsize - scount[step];
        rindex[step] = sindex[step] + scount[step];
    }
}

/* Group re-ordering of both error handlers (raben/errhandler.c:50-76, 243-268, 425-441):
 * drop the entry at comm rank `repl`, and put it where `dead` was. */
static void rb_regroup(rb_t *b, int dead, int repl)
{
    int neworder[FTAR_MAX_RANKS];
    int k = 0;
    for (int c = 0; c < b->size; c++)
        if (c != repl) neworder[k++] = b->order[c];
    if (repl != dead) {
        int pos = (dead < repl) ? dead : dead - 1;
        neworder[pos] = b->order[repl];
    }
    memcpy(b->order, neworder, sizeof(int) * (size_t)k);
    b->size = k;
}

/* errhandler_reduce_scatter, raben/errhandler.c:3-282 */
static void rb_handler_rs(rb_t *b, const int *dead_w, int nf, int failed_step)
{
    sim_t *s = b->s;
    size_t es = s->es;
    if (nf > 1 || failed_step == 0) { /* :37-38 */
        do_abort(s, 1);
        return;
    }
    int dead = rb_comm_rank_of(b, dead_w[0]);
    int idle_die = (dead < b->rem * 2 && dead % 2 == 1);
    if (idle_die) { /* :50-76 */
        rb_regroup(b, dead, b->rem * 2 - 1);
    } else {
        int vdead = (dead < b->rem * 2) ? dead / 2 : dead - b->rem; /* :80-88 */
        int org = rb_real(b, vdead ^ 1);                           /* :89-90 */
        int new_entry = b->rem * 2 - 1;                            /* :207 */
        rb_rank *imp = &b->rk[b->order[org]];
        if (!imp->has_recov) {
            /* deviation: the impersonator holds no step-0 copy of the dead rank's vector
             * (it is itself a replacement); the reference replays garbage here. */
            s->res->deviations |= FTAR_DEV_RABEN_NO_RECOV;
            do_abort(s, 1);
            return;
        }
        /* The impersonator replays the dead rank's reduce-scatter steps 0..failed_step
         * (:106-200).  Intent restated: it accumulates into a scratch copy of its own
         * input (the reference accumulates into sbuf and receives into tmp, which
         * destroys the redundancy for a second recovery by the same rank). */
        unsigned char *acc = (unsigned char *)malloc(s->count * es + 1);
        unsigned char *rx = (unsigned char *)malloc(s->count * es + 1);
        memcpy(acc, imp->sbuf, s->count * es);
        int d_rindex[MAXSTEPS], d_sindex[MAXSTEPS], d_rcount[MAXSTEPS], d_scount[MAXSTEPS];
        int adj = 1 << (failed_step + 1);
        int step = 0, wsize = (int)s->count;
        d_sindex[0] = d_rindex[0] = 0;
        for (int mask = 1; mask < adj; mask <<= 1) {
            int dest = rb_real(b, vdead ^ mask);
            rb_window(dead, dest, step, wsize, d_rindex, d_sindex, d_rcount, d_scount);
            if (step != 0) {
                /* partner of the dead rank at this step re-sends its unchanged sindex
                 * window (:159-169); the impersonator reduces it (:143-152) */
                rb_rank *pr = &b->rk[b->order[dest]];
                memcpy(ELEM(rx, (size_t)d_rindex[step], es), ELEM(pr->rbuf, (size_t)pr->sindex[step], es),
                       (size_t)d_rcount[step] * es);
                reduce_into(s, ELEM(acc, (size_t)d_rindex[step], es), ELEM(rx, (size_t)d_rindex[step], es),
                            (size_t)d_rcount[step]);
                if (step == failed_step) {
                    /* :153-157 and :170-180: the dead rank's outgoing window reaches the
                     * partner, which reduces it only if its own receive had failed */
                    memcpy(ELEM(pr->tmp, (size_t)pr->rindex[step], es), ELEM(acc, (size_t)d_sindex[step], es),
                           (size_t)d_scount[step] * es);
                    if (pr->corr)
                        reduce_into(s, ELEM(pr->rbuf, (size_t)pr->rindex[step], es),
                                    ELEM(pr->tmp, (size_t)pr->rindex[step], es), (size_t)pr->rcount[step]);
                }
            }
            if (step + 1 < b->steps) { /* :183-189 */
                d_rindex[step + 1] = d_rindex[step];
                d_sindex[step + 1] = d_rindex[step];
                wsize = d_rcount[step];
            }
            if (step == 0) /* :191-197 -- tmp holds the dead rank's vector from step 0 */
                reduce_into(s, ELEM(acc, (size_t)d_rindex[0], es), ELEM(imp->tmp, (size_t)d_rindex[0], es),
                            (size_t)d_rcount[0]);
            if ((mask << 1) < adj) step++;
        }
        if (new_entry == -1) { /* :210-211 */
            free(acc);
            free(rx);
            do_abort(s, 1);
            return;
        }
        /* state hand-off to new_entry (:213-241) */
        rb_rank *ne = &b->rk[b->order[new_entry]];
        memcpy(ne->rbuf, acc, s->count * es);
        memcpy(ne->rindex, d_rindex, sizeof(d_rindex));
        memcpy(ne->sindex, d_sindex, sizeof(d_sindex));
        memcpy(ne->rcount, d_rcount, sizeof(d_rcount));
        memcpy(ne->scount, d_scount, sizeof(d_scount));
        ne->wsize = wsize;
        ne->has_recov = 0; /* it has the dead rank's state, not its redundancy */
        free(acc);
        free(rx);
        rb_regroup(b, dead, new_entry); /* :252-268 */
    }
    b->rem--; /* caller, rabenseifner.c:268-283 */
    rb_vranks(b);
    for (int c = 0; c < b->size; c++) b->rk[b->order[c]].corr = 0;
    s->res->recoveries++;
}

/* errhandler_allgather, raben/errhandler.c:284-468 */
static void rb_handler_ag(rb_t *b, const int *dead_w, int nf, int failed_step)
{
    sim_t *s = b->s;
    size_t es = s->es;
    if (nf > 1 || failed_step == b->steps - 1) { /* :320-323 */
        do_abort(s, 1);
        return;
    }
    int dead = rb_comm_rank_of(b, dead_w[0]);
    int idle_die = (dead < b->rem * 2 && dead % 2 == 1);
    if (idle_die) {
        rb_regroup(b, dead, b->rem * 2 - 1);
    } else {
        int vdead = (dead < b->rem * 2) ? dead / 2 : dead - b->rem;
        int org = rb_real(b, vdead ^ (b->adjsize >> 1)); /* :372-373 */
        int new_entry = b->rem * 2 - 1;
        if (new_entry == -1) {
            do_abort(s, 1);
            return;
        }
        rb_rank *o = &b->rk[b->order[org]];
        rb_rank *ne = &b->rk[b->order[new_entry]];
        /* :381-398: full buffer + index arrays of the original partner */
        memcpy(ne->rbuf, o->rbuf, s->count * es);
        memcpy(ne->rindex, o->rindex, sizeof(o->rindex));
        memcpy(ne->sindex, o->sindex, sizeof(o->sindex));
        memcpy(ne->rcount, o->rcount, sizeof(o->rcount));
        memcpy(ne->scount, o->scount, sizeof(o->scount));
        ne->has_recov = 0;
        /* :400-414: repair the block the dead rank owed its last partner */
        int lp = rb_real(b, vdead ^ (1 << failed_step));
        rb_rank *l = &b->rk[b->order[lp]];
        memcpy(ELEM(l->rbuf, (size_t)l->sindex[failed_step], es),
               ELEM(ne->rbuf, (size_t)ne->rindex[failed_step], es), (size_t)ne->rcount[failed_step] * es);
        rb_regroup(b, dead, new_entry);
    }
    b->rem--;
    rb_vranks(b);
    s->res->recoveries++;
}

int ftar_oracle_rabenseifner(int p, size_t count, int dtype, int op, const void *const *inputs,
                             void *const *outputs, const ftar_kill *kills, int nkills,
                             ftar_oracle_result *res)
{
    sim_t S;
    memset(res, 0, sizeof(*res));
    memset(&S, 0, sizeof(S));
    S.p = p; S.count = count; S.dtype = dtype; S.op = op; S.kills = kills; S.nkills = nkills;
    S.res = res; S.es = ftar_oracle_esize(dtype);
    if (p < 1 || p > FTAR_MAX_RANKS || check_op(dtype, op)) {
        res->ret = p < 1 || p > FTAR_MAX_RANKS ? FTAR_ERR_ARG : check_op(dtype, op);
        return res->ret;
    }
    size_t es = S.es;
    rb_t B;
    memset(&B, 0, sizeof(B));
    B.s = &S;
    B.size = p;
    for (int c = 0; c < p; c++) B.order[c] = c;
    B.steps = hibit(p, (int)(sizeof(int) * 8) - 1); /* :16-21 */
    if (B.steps == -1) {
        res->ret = FTAR_ERR_ARG;
        return res->ret;
    }
    B.adjsize = 1 << B.steps;
    B.rem = p - B.adjsize;
    for (int w = 0; w < p; w++) res->status[w] = FTAR_ORACLE_OK;
    if (count == 0) { /* copy_buffer(count<=0) -> MPI_ERR_UNKNOWN, util.c:40-43 */
        res->ret = FTAR_ERR_UNKNOWN;
        res->size_after = p;
        for (int c = 0; c < p; c++) res->order_after[c] = c;
        return res->ret;
    }
    B.rk = (rb_rank *)calloc((size_t)p, sizeof(rb_rank));
    for (int w = 0; w < p; w++) {
        rb_rank *r = &B.rk[w];
        r->alive = 1;
        r->has_recov = 1;
        r->sbuf = (unsigned char *)malloc(count * es);
        r->rbuf = (unsigned char *)malloc(count * es);
        r->tmp = (unsigned char *)malloc(count * es);
        memcpy(r->sbuf, inputs[w], count * es);
        memcpy(r->rbuf, inputs[w], count * es); /* :35-42 */
        poison(&S, r->tmp, count);
    }

    /* ---- pre-step (:61-139), errors fatal ---- */
    for (int w = 0; w < p; w++)
        if (kill_point(&S, w, FTAR_PH_PRE, 0) >= 0) {
            /* a death before the tolerant region is fatal: the partner's Sendrecv or the
             * ERRORS_ARE_FATAL barrier at :166 aborts the job */
            B.rk[w].alive = 0;
            res->status[w] = FTAR_ORACLE_DEAD;
            do_abort(&S, FATAL_CODE);
        }
    if (!S.aborted) {
        size_t lh = count / 2, rh = count - count / 2;
        for (int c = 0; c + 1 < 2 * B.rem; c += 2) {
            rb_rank *e = &B.rk[B.order[c]], *o = &B.rk[B.order[c + 1]];
            /* Sendrecv: odd gets even's right half, even gets odd's left half */
            memcpy(ELEM(o->tmp, lh, es), ELEM(e->rbuf, lh, es), rh * es);
            memcpy(e->tmp, o->rbuf, lh * es);
            reduce_into(&S, ELEM(o->rbuf, lh, es), ELEM(o->tmp, lh, es), rh); /* :86-87 */
            reduce_into(&S, e->rbuf, e->tmp, lh);                            /* :117 */
            memcpy(ELEM(e->rbuf, lh, es), ELEM(o->rbuf, lh, es), rh * es);   /* :90, :120 */
            memcpy(e->sbuf, e->rbuf, count * es);                            /* :128 */
        }
        rb_vranks(&B);
    }

    /* ---- reduce-scatter (:153-284) ---- */
    for (int w = 0; w < p; w++) {
        B.rk[w].wsize = (int)count;
        B.rk[w].sindex[0] = B.rk[w].rindex[0] = 0;
        B.rk[w].corr = 0;
    }
    int step = 0;
    for (int mask = 1; mask < B.adjsize && !S.aborted; mask <<= 1) {
        int kp[FTAR_MAX_RANKS];
        for (int w = 0; w < p; w++) kp[w] = B.rk[w].alive ? kill_point(&S, w, FTAR_PH_LOOP, step) : -1;
        int dest_of[FTAR_MAX_RANKS];
        /* windows */
        for (int c = 0; c < B.size; c++) {
            int w = B.order[c];
            rb_rank *r = &B.rk[w];
            dest_of[c] = -1;
            if (r->vrank == -1) continue;
            int dest = rb_real(&B, r->vrank ^ mask);
            dest_of[c] = dest;
            rb_window(c, dest, step, r->wsize, r->rindex, r->sindex, r->rcount, r->scount);
        }
        /* exchange: receivers snapshot the sender's buffer before any reduce */
        int got[FTAR_MAX_RANKS];
        for (int c = 0; c < B.size; c++) {
            int w = B.order[c];
            rb_rank *r = &B.rk[w];
            got[c] = 0;
            if (dest_of[c] < 0 || kp[w] == FTAR_PT_BEFORE) continue;
            int dw = B.order[dest_of[c]];
            rb_rank *d = &B.rk[dw];
            if (failed_xchg(kp[dw])) { /* partner died before or during its Sendrecv: :238-241 */
                r->corr = 1;
                poison(&S, ELEM(r->tmp, (size_t)r->rindex[step], es), (size_t)r->rcount[step]);
                continue;
            }
            if (step == 0) /* :206-211 whole buffer */
                memcpy(r->tmp, d->rbuf, count * es);
            else           /* :219-222 */
                memcpy(ELEM(r->tmp, (size_t)r->rindex[step], es), ELEM(d->rbuf, (size_t)d->sindex[step], es),
                       (size_t)r->rcount[step] * es);
            got[c] = 1;
        }
        for (int c = 0; c < B.size; c++) {
            int w = B.order[c];
            rb_rank *r = &B.rk[w];
            if (dest_of[c] < 0) continue;
            if (got[c] && kp[w] != FTAR_PT_AFTER && kp[w] != FTAR_PT_BEFORE && kp[w] != FTAR_PT_DURING)
                reduce_into(&S, ELEM(r->rbuf, (size_t)r->rindex[step], es), ELEM(r->tmp, (size_t)r->rindex[step], es),
                            (size_t)r->rcount[step]);
            if (step + 1 < B.steps) { /* :244-249 */
                r->rindex[step + 1] = r->rindex[step];
                r->sindex[step + 1] = r->rindex[step];
                r->wsize = r->rcount[step];
            }
        }
        /* barrier (:258-265): deaths of this step are detected uniformly */
        int dead_w[FTAR_MAX_RANKS], nf = 0;
        for (int w = 0; w < p; w++)
            if (kp[w] >= 0) {
                B.rk[w].alive = 0;
                res->status[w] = FTAR_ORACLE_DEAD;
                dead_w[nf++] = w;
            }
        if (nf > 0) rb_handler_rs(&B, dead_w, nf, step);
        step++;
    }

    /* ---- allgather (:299-355) ---- */
    step = B.steps - 1;
    for (int mask = B.adjsize >> 1; mask > 0 && !S.aborted; mask >>= 1) {
        int kp[FTAR_MAX_RANKS];
        for (int w = 0; w < p; w++) kp[w] = B.rk[w].alive ? kill_point(&S, w, FTAR_PH_AG, step) : -1;
        /* receives go into disjoint windows of rbuf; stage them to model simultaneity */
        unsigned char *stage[FTAR_MAX_RANKS];
        for (int c = 0; c < B.size; c++) {
            int w = B.order[c];
            rb_rank *r = &B.rk[w];
            stage[c] = NULL;
            if (r->vrank == -1 || kp[w] == FTAR_PT_BEFORE) continue;
            int dest = rb_real(&B, r->vrank ^ mask);
            int dw = B.order[dest];
            rb_rank *d = &B.rk[dw];
            stage[c] = (unsigned char *)malloc((size_t)r->scount[step] * es + 1);
            if (failed_xchg(kp[dw])) {
                poison(&S, stage[c], (size_t)r->scount[step]);
            } else {
                memcpy(stage[c], ELEM(d->rbuf, (size_t)d->rindex[step], es), (size_t)r->scount[step] * es);
            }
        }
        for (int c = 0; c < B.size; c++) {
            if (!stage[c]) continue;
            rb_rank *r = &B.rk[B.order[c]];
            memcpy(ELEM(r->rbuf, (size_t)r->sindex[step], es), stage[c], (size_t)r->scount[step] * es);
            free(stage[c]);
        }
        int dead_w[FTAR_MAX_RANKS], nf = 0;
        for (int w = 0; w < p; w++)
            if (kp[w] >= 0) {
                B.rk[w].alive = 0;
                res->status[w] = FTAR_ORACLE_DEAD;
                dead_w[nf++] = w;
            }
        if (nf > 0) rb_handler_ag(&B, dead_w, nf, step);
        step--;
    }

    /* ---- fatal barrier + post-step (:357-381) ---- */
    if (!S.aborted) {
        for (int c = 0; c < B.size; c++) {
            int w = B.order[c];
            if (kill_point(&S, w, FTAR_PH_POST, 0) >= 0) {
                B.rk[w].alive = 0;
                res->status[w] = FTAR_ORACLE_DEAD;
                do_abort(&S, FATAL_CODE);
            }
        }
    }
    if (!S.aborted) {
        for (int c = 0; c + 1 < 2 * B.rem; c += 2) {
            rb_rank *e = &B.rk[B.order[c]], *o = &B.rk[B.order[c + 1]];
            memcpy(o->rbuf, e->rbuf, count * es);
        }
    }

    if (S.aborted) {
        for (int w = 0; w < p; w++)
            if (res->status[w] == FTAR_ORACLE_OK) res->status[w] = FTAR_ORACLE_ABORTED;
    } else {
        for (int w = 0; w < p; w++)
            if (res->status[w] == FTAR_ORACLE_OK) memcpy(outputs[w], B.rk[w].rbuf, count * es);
    }
    res->size_after = B.size;
    memcpy(res->order_after, B.order, sizeof(int) * (size_t)B.size);
    for (int w = 0; w < p; w++) {
        free(B.rk[w].sbuf);
        free(B.rk[w].rbuf);
        free(B.rk[w].tmp);
    }
    free(B.rk);
    res->ret = FTAR_SUCCESS;
    return res->ret;
}

/* ------------------------------------------------------------------------- */
/* Recursive doubling (src/rd/recursive_doubling.c:6-90, util.c, errhandler.c) */
/* ------------------------------------------------------------------------- */

typedef struct {
    int alive;
    unsigned char *src, *dst;
} rd_rank;

typedef struct {
    sim_t *s;
    rd_rank *rk;
    /* Data (rd/header.h:16-26): identical on every rank, ids are original ranks */
    int active[FTAR_MAX_RANKS], nactive;
    int inactive[FTAR_MAX_RANKS], ninactive;
} rd_t;

static int contains(const int *a, int target, int n) /* rd/util.c:36-47 */
{
    for (int i = 0; i < n; i++)
        if (a[i] == target) return 1;
    return 0;
}

static int floor_pow2(int n)
{
    int p = 1;
    while (p * 2 <= n) p *= 2;
    return p;
}

/* rd/errhandler.c:6-302, global effect.  `distance` is the caller's doubled distance
 * (recursive_doubling.c:58); returns the possibly reduced distance.  `last` selects the
 * accumulator buffer (dst on the last step, :59-66). */
static int rd_handler(rd_t *b, const int *F, int nf, int distance, int last)
{
    sim_t *s = b->s;
    size_t es = s->es;
    int d = distance / 2;
    int inactive_nf = 0;
    /* compact failed inactive ranks (:47-65) */
    {
        int k = 0;
        for (int i = 0; i < b->ninactive; i++) {
            if (contains(F, b->inactive[i], nf)) inactive_nf++;
            else b->inactive[k++] = b->inactive[i];
        }
        b->ninactive = k;
    }
    int active_failed = 0;
    for (int i = 0; i < b->nactive; i++)
        if (contains(F, b->active[i], nf)) active_failed = 1;
    if (!active_failed) return distance; /* :219-222 */

    int nfa = nf - inactive_nf;
    if (nfa >= d) { /* check_abort, util.c:49-78: a block of 2d ranks all dead or corrupted */
        int k = 0;
        for (int i = 0; i < b->nactive; i++) {
            if (i % distance == 0) k = 0;
            if (contains(F, b->active[i], nf) || contains(F, b->active[i ^ d], nf)) k++;
            if (k == distance) {
                do_abort(s, FTAR_ERR_OTHER);
                return distance;
            }
        }
    }
    if (nfa <= b->ninactive) {
        /* spare branch (:78-177).  Deviation: the master search loop at :100-111 never
         * advances j and spins forever; restated with its evident intent -- the master of
         * each block of d ranks is its first rank that is alive and whose partner at the
         * failed step is alive. */
        s->res->deviations |= FTAR_DEV_RD_MASTER_LOOP;
        int master_of_block[FTAR_MAX_RANKS];
        for (int blk = 0; blk * d < b->nactive; blk++) {
            master_of_block[blk] = -1;
            for (int i = blk * d; i < (blk + 1) * d && i < b->nactive; i++)
                if (!contains(F, b->active[i], nf) && !contains(F, b->active[i ^ d], nf)) {
                    master_of_block[blk] = i;
                    break;
                }
        }
        int killed[FTAR_MAX_RANKS], nk = 0;
        for (int i = 0; i < b->nactive; i++)
            if (contains(F, b->active[i], nf)) killed[nk++] = i;
        int j = b->ninactive - 1;
        for (int i = 0; i < b->nactive; i++) {
            if (!contains(F, b->active[i], nf)) continue;
            int m = master_of_block[i / d];
            int spare = b->inactive[j];
            if (m < 0) { /* no healthy rank left to restore from */
                do_abort(s, FTAR_ERR_OTHER);
                return distance;
            }
            unsigned char *mbuf = last ? b->rk[b->active[m]].dst : b->rk[b->active[m]].src;
            /* woken spare receives the master's accumulator (:232-244) */
            memcpy(last ? b->rk[spare].dst : b->rk[spare].src, mbuf, s->count * es);
            int corr = i ^ d; /* corrupted partner (:147-168) */
            if (!contains(killed, corr, nk)) {
                int mc = master_of_block[corr / d];
                if (mc < 0) {
                    do_abort(s, FTAR_ERR_OTHER);
                    return distance;
                }
                unsigned char *cb = last ? b->rk[b->active[corr]].dst : b->rk[b->active[corr]].src;
                unsigned char *mcb = last ? b->rk[b->active[mc]].dst : b->rk[b->active[mc]].src;
                memcpy(cb, mcb, s->count * es);
            }
            b->active[i] = spare;
            j--;
        }
        b->ninactive = j + 1;
        return distance;
    }
    /* not enough spares: shrink to the next lower power of two (:178-217) */
    int p = floor_pow2(b->nactive - nfa);
    int k = b->nactive / p;
    int newdist = distance / k;
    int blk2 = newdist * k; /* = distance, the block of 2d ranks holding equal sums */
    int newarr[FTAR_MAX_RANKS], total = 0, block_count = 0;
    int extra[FTAR_MAX_RANKS], nextra = 0;
    for (int i = 0; i < b->nactive; i++) {
        if (i % blk2 == 0) block_count = 0;
        if (!contains(F, b->active[i], nf)) {
            if (block_count < newdist && !contains(F, b->active[i ^ (blk2 / 2)], nf)) {
                newarr[total++] = b->active[i];
                block_count++;
            } else {
                extra[nextra++] = b->active[i];
            }
        }
    }
    if (total < p) { /* deviation: the reference reads uninitialised new_array entries */
        s->res->deviations |= FTAR_DEV_RD_SHORT_SHRINK;
        do_abort(s, FTAR_ERR_OTHER);
        return distance;
    }
    for (int i = 0; i < nextra; i++) b->inactive[b->ninactive++] = extra[i];
    memcpy(b->active, newarr, sizeof(int) * (size_t)p);
    b->nactive = p;
    return newdist;
}

int ftar_oracle_recursive_doubling(int p, size_t count, int dtype, int op, const void *const *inputs,
                                   void *const *outputs, const ftar_kill *kills, int nkills,
                                   ftar_oracle_result *res)
{
    sim_t S;
    memset(res, 0, sizeof(*res));
    memset(&S, 0, sizeof(S));
    S.p = p; S.count = count; S.dtype = dtype; S.op = op; S.kills = kills; S.nkills = nkills;
    S.res = res; S.es = ftar_oracle_esize(dtype);
    if (p < 1 || p > FTAR_MAX_RANKS || check_op(dtype, op)) {
        res->ret = p < 1 || p > FTAR_MAX_RANKS ? FTAR_ERR_ARG : check_op(dtype, op);
        return res->ret;
    }
    size_t es = S.es;
    rd_t B;
    memset(&B, 0, sizeof(B));
    B.s = &S;
    B.rk = (rd_rank *)calloc((size_t)p, sizeof(rd_rank));
    for (int w = 0; w < p; w++) {
        B.rk[w].alive = 1;
        B.rk[w].src = (unsigned char *)malloc(count * es + 1);
        B.rk[w].dst = (unsigned char *)malloc(count * es + 1);
        memcpy(B.rk[w].src, inputs[w], count * es);
        poison(&S, B.rk[w].dst, count);
        res->status[w] = FTAR_ORACLE_OK;
    }
    /* Data init (recursive_doubling.c:118-130) */
    B.nactive = p;
    for (int w = 0; w < p; w++) B.active[w] = w;
    B.ninactive = 0;

    /* reduce_pow2 (util.c:3-34) */
    int pp = floor_pow2(p);
    if (pp < p) {
        B.nactive = pp;
        B.ninactive = p - pp;
        for (int i = pp; i < p; i++) B.inactive[i - pp] = i;
    }
    int pre_dead[FTAR_MAX_RANKS], npre = 0;
    for (int w = 0; w < p; w++)
        if (kill_point(&S, w, FTAR_PH_PRE, 0) >= 0) {
            int involved = (w >= pp) || (w < B.ninactive);
            B.rk[w].alive = 0;
            res->status[w] = FTAR_ORACLE_DEAD;
            if (involved) do_abort(&S, FATAL_CODE); /* Send/Recv under ERRORS_ARE_FATAL */
            else pre_dead[npre++] = w;     /* surfaces at the first step's barrier */
        }
    if (!S.aborted) {
        for (int r = 0; r < B.ninactive; r++) {
            int a = B.active[r], in = B.inactive[r];
            memcpy(B.rk[a].dst, B.rk[in].src, count * es);              /* util.c:31 */
            reduce_into(&S, B.rk[a].src, B.rk[a].dst, count);           /* util.c:32 */
        }
    }

    /* distance loop (recursive_doubling.c:21-71) */
    int iter = 0;
    for (int distance = 1; !S.aborted && distance < B.nactive; distance *= 2, iter++) {
        int kp[FTAR_MAX_RANKS];
        for (int w = 0; w < p; w++) {
            kp[w] = B.rk[w].alive ? kill_point(&S, w, FTAR_PH_LOOP, iter) : -1;
            if (iter == 0 && contains(pre_dead, w, npre)) kp[w] = FTAR_PT_BEFORE;
        }
        int last = (distance * 2 >= B.nactive);
        int n = B.nactive;
        unsigned char *stage[FTAR_MAX_RANKS];
        for (int i = 0; i < n; i++) {
            int w = B.active[i];
            stage[i] = NULL;
            if (kp[w] == FTAR_PT_BEFORE || (!B.rk[w].alive && kp[w] < 0)) continue;
            int pw = B.active[i ^ distance];
            stage[i] = (unsigned char *)malloc(count * es + 1);
            if (failed_xchg(kp[pw]) || (!B.rk[pw].alive && kp[pw] < 0))
                poison(&S, stage[i], count); /* Sendrecv error ignored (:35-37): corrupted */
            else
                memcpy(stage[i], B.rk[pw].src, count * es);
        }
        for (int i = 0; i < n; i++) {
            if (!stage[i]) continue;
            rd_rank *r = &B.rk[B.active[i]];
            memcpy(r->dst, stage[i], count * es);
            free(stage[i]);
            if (kp[B.active[i]] == FTAR_PT_AFTER || kp[B.active[i]] == FTAR_PT_DURING) continue;
            if (last) reduce_into(&S, r->dst, r->src, count); /* :44 Reduce_local(src, dst) */
            else reduce_into(&S, r->src, r->dst, count);      /* :48 Reduce_local(dst, src) */
        }
        int F[FTAR_MAX_RANKS], nf = 0;
        for (int w = 0; w < p; w++)
            if (kp[w] >= 0) {
                B.rk[w].alive = 0;
                res->status[w] = FTAR_ORACLE_DEAD;
                F[nf++] = w;
            }
        if (nf > 0) {
            int dd = distance * 2;
            dd = rd_handler(&B, F, nf, dd, dd >= B.nactive ? 1 : last);
            if (!S.aborted) res->recoveries++;
            distance = dd / 2;
        }
    }
    if (!S.aborted) {
        for (int w = 0; w < p; w++)
            if (B.rk[w].alive && kill_point(&S, w, FTAR_PH_POST, 0) >= 0) {
                B.rk[w].alive = 0;
                res->status[w] = FTAR_ORACLE_DEAD;
                do_abort(&S, FATAL_CODE);
            }
    }
    if (!S.aborted && B.nactive == 1 && p == 1) {
        /* deviation: with one rank the reference never writes dst */
        memcpy(B.rk[0].dst, B.rk[0].src, count * es);
        res->deviations |= FTAR_DEV_RD_SINGLE;
    }
    if (!S.aborted) {
        /* result fan-out to inactive ranks (:78-89) */
        if (B.ninactive > B.nactive) {
            res->deviations |= FTAR_DEV_RD_FANOUT;
            do_abort(&S, 1);
        } else {
            for (int r = 0; r < B.ninactive; r++)
                memcpy(B.rk[B.inactive[r]].dst, B.rk[B.active[r]].dst, count * es);
        }
    }
    if (S.aborted) {
        for (int w = 0; w < p; w++)
            if (res->status[w] == FTAR_ORACLE_OK) res->status[w] = FTAR_ORACLE_ABORTED;
    } else {
        for (int w = 0; w < p; w++)
            if (res->status[w] == FTAR_ORACLE_OK) memcpy(outputs[w], B.rk[w].dst, count * es);
    }
    /* comm after the call: active ranks in their comm order (the survivor world for the
     * next call is every alive rank in original order) */
    res->size_after = 0;
    for (int w = 0; w < p; w++)
        if (res->status[w] == FTAR_ORACLE_OK) res->order_after[res->size_after++] = w;
    for (int w = 0; w < p; w++) {
        free(B.rk[w].src);
        free(B.rk[w].dst);
    }
    free(B.rk);
    res->ret = FTAR_SUCCESS;
    return res->ret;
}
