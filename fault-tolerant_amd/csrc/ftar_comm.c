/*
 * ftar_comm.c -- communicator bootstrap, workspace exchange, synchronisation and the
 * small C-ABI entry points (rank queries, barrier, abort, local reduce, statistics).
 *
 * Bootstrap replaces MPI_Init + MPI_Comm_dup(MPI_COMM_WORLD)
 * (raben/rabenseifner.c:439-454, rd/recursive_doubling.c:100-103).
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include "ftar_internal.h"

#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#define WS_ALIGN (2u << 20)

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

size_t ftar_esize(int dtype)
{
    switch (dtype) {
    case FTAR_INT32:
    case FTAR_FLOAT32: return 4;
    case FTAR_INT64:
    case FTAR_FLOAT64: return 8;
    default: return 0;
    }
}

/* MPI_Reduce_local's type/op check: an unknown type or op is an argument error, a
 * logical or bitwise op on a floating-point type is MPI_ERR_OP (MPI 4.1, 6.9.2). */
int ftar_check_op(int dtype, int op)
{
    if (ftar_esize(dtype) == 0 || op < FTAR_SUM || op >= FTAR_NOPS) return FTAR_ERR_ARG;
    if (op >= FTAR_LAND && (dtype == FTAR_FLOAT32 || dtype == FTAR_FLOAT64)) return FTAR_ERR_OP;
    return FTAR_SUCCESS;
}

int ftar_hibit(int value, int start) /* raben/util.c:22-37 */
{
    unsigned int mask = (unsigned int)value & ((1u << start) - 1u);
    if (mask == 0) return -1;
    return (int)(8 * sizeof(int) - 1) - __builtin_clz(mask);
}

int ftar_floor_pow2(int n) /* (int)pow(2, floor(log2(n))), rd/util.c:5 */
{
    int p = 1;
    while (p * 2 <= n) p *= 2;
    return p;
}

int ftar_my_comm_rank(const ftar_comm *c) { return ftar_comm_rank_of(c, c->wrank); }

int ftar_comm_rank_of(const ftar_comm *c, int w)
{
    for (int i = 0; i < c->size; i++)
        if (c->order[i] == w) return i;
    return -1;
}

static void recompute_members(ftar_comm *c)
{
    c->members = 0;
    for (int i = 0; i < c->size; i++) c->members |= 1ull << c->order[i];
}

/* ---- fault injection ---------------------------------------------------- */

/* "rank:phase:step:point[:call]" entries separated by ',' (call = 0-based index of the
 * allreduce call on that rank; omitted = every call) */
static int parse_kills(const char *s, ftar_kill *out, int *call, int max)
{
    int n = 0;
    while (s && *s && n < max) {
        ftar_kill k;
        int used = 0, cl = -1, used2 = 0;
        if (sscanf(s, "%d:%d:%d:%d%n", &k.rank, &k.phase, &k.step, &k.point, &used) != 4) break;
        s += used;
        if (*s == ':' && sscanf(s, ":%d%n", &cl, &used2) == 1) s += used2;
        call[n] = cl;
        out[n++] = k;
        while (*s == ',' || *s == ' ' || *s == ';') s++;
    }
    return n;
}

void ftar_maybe_die(ftar_comm *c, int phase, int step, int point)
{
    for (int i = 0; i < c->nkills; i++) {
        const ftar_kill *k = &c->kills[i];
        if (k->rank != c->wrank || k->phase != phase || k->step != step || k->point != point) continue;
        if (c->kill_call[i] >= 0 && c->kill_call[i] != c->ncalls - 1) continue;
        if (point == FTAR_PT_BARRIER) /* let every peer finish the step first */
            ftar_ctrl_wait_peers_before_dying(&c->job, c->members, c->job.seq + 1);
        if (point == FTAR_PT_DURING) {
            /* mid-exchange: this rank's own pulls are queued, and once every peer has
             * launched its pulls of the step the partners' kernels read our HBM while
             * this process (and its queues) is torn down */
            int peers = ftar_ctrl_wait_peers_launched(&c->job, c->members);
            int busy = fdev_busy(c->dev);
            fprintf(stderr, "ftar: rank %d dies mid-exchange (phase %d step %d): own kernel %s, %d peers launched\n",
                    c->wrank, phase, step, busy ? "in flight" : "complete", peers);
        }
#ifdef FTAR_TEST_HOOKS
        if (getenv("FTAR_KILL_WITHDRAW")) {
            /* TEST-ONLY (the hooks build, lib/libftar_hooks.so and host-sim): the victim's
             * input is gone with it (as after the loss of its device): its workspace
             * generation moves on and its published sbuf is withdrawn, so no peer may read
             * either (ftar_dead_input) */
            ftar_slot *me = &c->job.shm->slot[c->wrank];
            atomic_fetch_add(&me->ws_gen, 1);
            me->uid = 0;
            me->useq = 0;
            fprintf(stderr, "ftar: rank %d withdraws its input before dying\n", c->wrank);
        }
#endif
        if (c->verbose) fprintf(stderr, "ftar: rank %d dies at phase %d step %d point %d\n", c->wrank, phase, step, point);
        fflush(stdout);
        fflush(stderr);
        raise(SIGKILL);
    }
}

int ftar_set_kills(ftar_comm *c, const ftar_kill *kills, int nkills)
{
    if (!c || nkills < 0 || nkills > FTAR_MAX_KILLS) return FTAR_ERR_ARG;
    memcpy(c->kills, kills, sizeof(ftar_kill) * (size_t)nkills);
    for (int i = 0; i < nkills; i++) c->kill_call[i] = -1;
    c->nkills = nkills;
    return FTAR_SUCCESS;
}

/* ---- bootstrap ------------------------------------------------------------ */

/* The comm's environment defaults: every value must be a whole number (or a decimal where
 * `real`) inside [lo, hi] -- "auto", "on", "" or "1x" are refused with FTAR_ERR_ARG and a
 * message naming the variable, never read as 0 the way atoi would.  The same
 * ranges ftar_comm_set_option accepts. */
struct env_knob {
    const char *name;
    double lo, hi, dflt;
    int real;
};

static int env_value(int rank, const struct env_knob *k, double *out)
{
    const char *e = getenv(k->name);
    *out = k->dflt;
    if (!e) return 0;
    char *end = NULL;
    double v = k->real ? strtod(e, &end) : (double)strtoll(e, &end, 10);
    if (end == e || *end != 0 || !(v >= k->lo && v <= k->hi)) {
        fprintf(stderr, "ftar: rank %d: %s=%s is not a %s in [%g, %g]: refused\n", rank, k->name, e,
                k->real ? "number" : "whole number", k->lo, k->hi);
        return FTAR_ERR_ARG;
    }
    *out = v;
    return 0;
}

int ftar_init_rank(ftar_comm **out, const char *job, int rank, int size, int device)
{
    *out = NULL;
    if (!job || rank < 0 || size < 1 || rank >= size || size > FTAR_MAX_RANKS) return FTAR_ERR_ARG;
    ftar_comm *c = (ftar_comm *)calloc(1, sizeof(ftar_comm));
    if (!c) return FTAR_ERR_NOMEM;
    c->wrank = rank;
    c->wsize = size;
    c->device = device;
    const double MiB = (double)(1 << 20), SZ = 4611686018427387904.0; /* sizes up to 2^62 */
    const struct env_knob knobs[] = {
        {"FTAR_VERBOSE", 0, 9, 0, 0},         {"FTAR_LOOP_SECONDS", 0, 1e6, 0, 1},
        {"FTAR_OVERLAP", 0, 1, 1, 0},         {"FTAR_RELAY", 0, 1, 1, 0},
        {"FTAR_REDUNDANCY", 0, 2, 2, 0},      {"FTAR_COPY_ENGINE", 0, 1, 0, 0},
        {"FTAR_MESH", 0, 1, 1, 0},            {"FTAR_PUSH", 0, 2, 0, 0},
        {"FTAR_MESH_WAIT", 0, 1, 1, 0},       {"FTAR_GATE", 0, 1, 1, 0},
        {"FTAR_GATE_HOLD_US", 0, 1e12, 2000, 1}, {"FTAR_GATE_MAX", 0, SZ, MiB, 0},
        {"FTAR_ONESHOT_MAX", 0, SZ, MiB, 0},  {"FTAR_EXPORT", 0, 1, 1, 0},
        {"FTAR_STAGE_MAX", 0, SZ, MiB, 0},    {"FTAR_HOST_PIPE", 0, 1, 1, 0},
        {"FTAR_RELAY_MIN", 0, SZ, 4 * MiB, 0},
    };
    double v[sizeof(knobs) / sizeof(knobs[0])];
    for (size_t i = 0; i < sizeof(knobs) / sizeof(knobs[0]); i++)
        if (env_value(rank, &knobs[i], &v[i])) {
            free(c);
            return FTAR_ERR_ARG;
        }
    c->verbose = (int)v[0];
    c->loop_seconds = v[1];
    c->overlap = (int)v[2];
    c->relay = (int)v[3];
    c->redundancy = (int)v[4];
    c->copy_engine = (int)v[5];
    c->mesh = (int)v[6];
    c->push = (int)v[7];
    c->mesh_wait = (int)v[8];
    c->gate = (int)v[9];
    c->gate_hold_s = v[10] * 1e-6;
    c->gate_max = (size_t)v[11];
    c->oneshot_max = (size_t)v[12];
    c->export_user = (int)v[13];
    c->stage_max = (size_t)v[14];
    c->host_pipe = (int)v[15];
    c->relay_min = (size_t)v[16];
    int create = getenv("FTAR_LAUNCHER") == NULL;
    int rc = ftar_ctrl_attach(&c->job, job, rank, size, create);
    if (rc) {
        free(c);
        return rc;
    }
    rc = fdev_open(device, &c->dev);
    if (rc) {
        fprintf(stderr, "ftar: rank %d: device %d: %s\n", rank, device, fdev_last_error());
        ftar_ctrl_detach(&c->job);
        free(c);
        return rc;
    }
    char phys[32];
    if (fdev_physical_id(c->dev, phys, sizeof(phys))) phys[0] = 0;
    rc = ftar_ctrl_join(&c->job, device, phys);
    if (rc) {
        fdev_close(c->dev);
        ftar_ctrl_detach(&c->job);
        free(c);
        return rc;
    }
    /* the device-wait flags (ftar_flag): the control block's flag page, mapped for this GPU */
    if (fdev_host_map(c->dev, (void *)c->job.shm->pwflag, sizeof(c->job.shm->pwflag), &c->pwflag_dev)) {
        fprintf(stderr, "ftar: rank %d: flag page not mapped (%s): the mesh orders its allgather on the host\n", rank,
                fdev_last_error());
        c->pwflag_dev = NULL;
    }
    const char *tp = getenv("FTAR_TRACE"); /* test instrumentation: tests/fence_check.py */
    if (tp && *tp) {
        char path[512];
        snprintf(path, sizeof(path), "%s.%d", tp, rank);
        if (fdev_trace_open(c->dev, path)) fprintf(stderr, "ftar: rank %d: %s\n", rank, fdev_last_error());
    }
    c->size = size;
    for (int i = 0; i < size; i++) c->order[i] = i;
    recompute_members(c);
    c->acked = 0;
    const char *ks = getenv("FTAR_KILL");
    if (ks) c->nkills = parse_kills(ks, c->kills, c->kill_call, FTAR_MAX_KILLS);
    /* every rank has mapped the control block once this round completes */
    ftar_sync_fatal(c);
    if (rank == 0) shm_unlink(job);
    *out = c;
    return FTAR_SUCCESS;
}

int ftar_init(ftar_comm **out)
{
    char name[128];
    int rank, size, device = -1;
    const char *e;
    if ((e = getenv("FTAR_JOB")) && getenv("FTAR_RANK") && getenv("FTAR_SIZE")) {
        snprintf(name, sizeof(name), "%s", e);
        rank = atoi(getenv("FTAR_RANK"));
        size = atoi(getenv("FTAR_SIZE"));
    } else if (getenv("RANK") && getenv("WORLD_SIZE")) { /* torchrun */
        rank = atoi(getenv("RANK"));
        size = atoi(getenv("WORLD_SIZE"));
        const char *port = getenv("MASTER_PORT");
        snprintf(name, sizeof(name), "/ftar-%s-%d", port ? port : "0", (int)getppid());
        if (getenv("LOCAL_RANK")) device = atoi(getenv("LOCAL_RANK"));
    } else {
        rank = 0;
        size = 1;
        snprintf(name, sizeof(name), "/ftar-solo-%d", (int)getpid());
    }
    if ((e = getenv("FTAR_DEVICE"))) device = atoi(e);
    int ndev = 0;
    int rc = fdev_device_count(&ndev);
    if (rc || ndev < 1) {
        fprintf(stderr, "ftar: rank %d: no HIP device visible (%s)\n", rank, fdev_last_error());
        return FTAR_ERR_DEVICE;
    }
    if (device < 0) device = rank;
    device %= ndev;
    return ftar_init_rank(out, name, rank, size, device);
}

static const char *const ws_name[FTAR_NBUF] = {"IN", "W", "T", "R"};

static void release_peers(ftar_comm *c)
{
    for (int w = 0; w < c->wsize; w++)
        for (int b = 0; b < FTAR_NBUF; b++)
            if (c->peer[w][b]) {
                fdev_trace_unregion(c->dev, c->peer[w][b]);
                fdev_unimport(c->dev, c->peer[w][b]);
                c->peer[w][b] = NULL;
            }
}

static void drop_mapping(ftar_comm *c, int w, int k)
{
    if (c->ucache[w][k].base) {
        fdev_trace_unregion(c->dev, c->ucache[w][k].base);
        fdev_unimport(c->dev, c->ucache[w][k].base);
    }
    c->ucache[w][k].base = NULL;
    c->ucache[w][k].id = 0;
}

static void release_user_peers(ftar_comm *c)
{
    for (int w = 0; w < c->wsize; w++)
        for (int k = 0; k < FTAR_UCACHE; k++) drop_mapping(c, w, k);
}

/* The exporter's side of the send-buffer caches (ftar_internal.h): this call's allocation is
 * a hit (1), enters a free entry (1, *fresh: the peers map it now), or finds the cache full
 * (0: staged).  The peers' peer_sbuf applies the same rule to the same sequence of ids, so its
 * cache of this rank holds exactly these ids. */
static int xcache_admit(ftar_comm *c, uint64_t id, int *fresh)
{
    const uint64_t now = (uint64_t)c->ncalls;
    *fresh = 0;
    int free_k = -1;
    for (int k = 0; k < FTAR_UCACHE; k++) {
        if (c->xcache[k].id == id) {
            c->xcache[k].last = now;
            return 1;
        }
        if (!c->xcache[k].id && free_k < 0) free_k = k;
    }
    if (free_k < 0) return 0;
    c->xcache[free_k].id = id;
    c->xcache[free_k].last = now;
    *fresh = 1;
    return 1;
}

static void xcache_forget(ftar_comm *c, uint64_t id)
{
    for (int k = 0; k < FTAR_UCACHE; k++)
        if (c->xcache[k].id == id) c->xcache[k].id = 0;
}

int ftar_stage_input(ftar_comm *c, const void *sbuf, size_t bytes, int alias_ok)
{
    ftar_slot *me = &c->job.shm->slot[c->wrank];
    uint64_t id = 0;
    size_t off = 0;
    int fresh = 0;
    ftar_inputs_done(c);
    /* a small input is cheaper staged than read in place: the staging copy signals its own
     * completion, where peers reading the caller's memory need a fenced marker */
    if (bytes <= c->stage_max) alias_ok = 0;
    int ok = alias_ok && c->export_user && bytes && fdev_export_range(c->dev, sbuf, bytes, NULL, &id, &off) == 0 &&
             xcache_admit(c, id, &fresh);
    /* a new entry: export its handle now (the peers map it after the call's first barrier) */
    if (ok && fresh && fdev_export_range(c->dev, sbuf, bytes, me->uhandle, &id, &off) != 0) {
        xcache_forget(c, id);
        ok = 0;
    }
    me->uid = ok ? id : 0;
    me->uoff = off;
    me->unew = ok && fresh;
    me->useq = (uint64_t)c->ncalls; /* a rank that dies before this point leaves an older tag */
    if (ok) {
        char nm[32];
        snprintf(nm, sizeof(nm), "U%llu", (unsigned long long)id);
        fdev_trace_region(c->dev, (const char *)sbuf - off, off + bytes, c->wrank, nm);
        fdev_trace_external_write(c->dev, sbuf, bytes); /* the caller wrote it: needs the fenced drain */
        c->in_alias = sbuf;
        /* peers read the caller's memory in place: the drain before the call's first barrier
         * must write it back device-wide (a fenced marker), whatever this rank launched */
        fdev_fence_next_drain(c->dev);
    }
    c->in_bytes = bytes;
    if (c->verbose >= 2)
        fprintf(stderr, "ftar[%d] call %d: input %s (allocation %llu, offset %zu%s)\n", c->wrank, c->ncalls,
                ok ? "in place" : "staged", (unsigned long long)me->uid, (size_t)me->uoff, fresh ? ", new" : "");
    return ok;
}

/* Rank w's exported send buffer as this rank maps it: the importer's side of xcache_admit. */
static void *peer_sbuf(ftar_comm *c, int w, int *failed)
{
    ftar_slot *s = &c->job.shm->slot[w];
    const uint64_t id = s->uid, now = (uint64_t)c->ncalls;
    if (s->useq != now || !id) return NULL; /* staged in IN, or not published (dead) */
    int k = -1;
    for (int j = 0; j < FTAR_UCACHE; j++) {
        if (c->ucache[w][j].base && c->ucache[w][j].id == id) {
            c->ucache[w][j].last = now;
            char nm[32];
            snprintf(nm, sizeof(nm), "U%llu", (unsigned long long)id);
            fdev_trace_region(c->dev, c->ucache[w][j].base, s->uoff + c->in_bytes, w, nm);
            return (char *)c->ucache[w][j].base + s->uoff;
        }
        if (!c->ucache[w][j].base && k < 0) k = j;
    }
    if (!s->unew || k < 0) {
        /* the exporter holds an entry this cache lacks (never expected: both apply one rule
         * to one sequence): make room, and report it */
        fprintf(stderr, "ftar: rank %d: call %d: rank %d's allocation %llu is not in this rank's cache (%s)\n", c->wrank,
                c->ncalls, w, (unsigned long long)id, s->unew ? "full" : "exported earlier");
        if (k < 0) {
            k = 0;
            for (int j = 1; j < FTAR_UCACHE; j++)
                if (c->ucache[w][j].last < c->ucache[w][k].last) k = j;
            drop_mapping(c, w, k);
        }
    }
    void *base = NULL;
    if (fdev_import(c->dev, s->uhandle, &base)) {
        fprintf(stderr, "ftar: rank %d: call %d: mapping rank %d's allocation %llu failed: %s\n", c->wrank, c->ncalls, w,
                (unsigned long long)id, fdev_last_error());
        *failed = !ftar_is_dead(c, w); /* a dead rank's data is never used */
        return NULL;
    }
    if (c->verbose >= 2)
        fprintf(stderr, "ftar[%d] call %d: mapped rank %d's allocation %llu\n", c->wrank, c->ncalls, w,
                (unsigned long long)id);
    c->ucache[w][k].id = id;
    c->ucache[w][k].base = base;
    c->ucache[w][k].last = now;
    char nm[32];
    snprintf(nm, sizeof(nm), "U%llu", (unsigned long long)id);
    fdev_trace_region(c->dev, base, s->uoff + c->in_bytes, w, nm);
    return (char *)base + s->uoff;
}

/* Map the peers' exported inputs.  A mapping is made only where an exporter published a new
 * cache entry (unew), and every rank reads the same words: then an extra agree round makes
 * sure every rank managed before anyone reads through a mapping -- if one did not, the job
 * stops exporting for good: the exporters stage their inputs in IN and the call goes on.
 * A call whose buffers the peers all hold already (any number of alternating buffers up to
 * FTAR_UCACHE) needs no extra round. */
void ftar_resolve_inputs(ftar_comm *c)
{
    int changed = 0, failed = 0;
    unsigned char member[FTAR_MAX_RANKS];
    memset(member, 0, sizeof(member));
    for (int i = 0; i < c->size; i++) { /* every member, this rank included: uniform */
        int w = c->order[i];
        const ftar_slot *s = &c->job.shm->slot[w];
        member[w] = 1;
        if (s->useq == (uint64_t)c->ncalls && s->uid && s->unew) changed = 1;
    }
    /* a rank no longer in the comm: its inputs are never read again, and a mapping would keep
     * its memory alive */
    for (int w = 0; w < c->wsize; w++)
        if (!member[w])
            for (int k = 0; k < FTAR_UCACHE; k++) drop_mapping(c, w, k);
    for (int i = 0; i < c->size; i++) {
        int w = c->order[i];
        if (w != c->wrank) c->peer_in[w] = peer_sbuf(c, w, &failed);
    }
    if (changed) {
        ftar_slot *me = &c->job.shm->slot[c->wrank];
        if (failed) {
            fprintf(stderr, "ftar: rank %d: cannot map a peer's send buffer (%s): inputs are staged from now on\n",
                    c->wrank, fdev_last_error());
            me->ufail = (uint64_t)c->ncalls;
        }
        (void)ftar_sync(c); /* new failures are reported again by the schedule's next agree */
        int any = 0;
        for (int i = 0; i < c->size; i++) any |= c->job.shm->slot[c->order[i]].ufail == (uint64_t)c->ncalls;
        if (any) {
            c->export_user = 0;
            me->uid = 0; /* this call's input is the staged IN from here on (ftar_dead_input) */
            if (c->in_alias) { /* stage the whole vector: what every schedule reads from IN */
                fdev_seg s = {FDEV_COPY, 0, c->ws[WS_IN], c->in_alias, NULL, c->in_bytes / 4, NULL};
                ftar_run(c, FTAR_INT32, FTAR_SUM, &s, 1, FDEV_TAG_LOCAL);
                ftar_drain(c);
            }
            ftar_inputs_done(c);
            (void)ftar_sync(c); /* every staged copy is ready */
        }
    } else if (failed) {
        /* a mapping outside the agreed ones failed (the caches disagreed): no uniform fallback */
        fprintf(stderr, "ftar: rank %d: cannot map a peer's send buffer: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
}

const void *ftar_dead_input(ftar_comm *c, int w, size_t bytes)
{
    ftar_slot *s = &c->job.shm->slot[w];
    if (s->useq != (uint64_t)c->ncalls) return NULL; /* not this call's input */
    if (c->peer_in[w]) return s->uid ? c->peer_in[w] : NULL; /* its sbuf, exported for this call */
    if (s->uid || !c->peer[w][WS_IN]) return NULL;
    if (c->peer_gen[w] != atomic_load(&s->ws_gen) || c->peer_bytes[w] < bytes) return NULL;
    return c->peer[w][WS_IN];
}

void ftar_inputs_done(ftar_comm *c)
{
    c->in_alias = NULL;
    memset(c->peer_in, 0, sizeof(c->peer_in));
}

int ftar_finalize(ftar_comm *c)
{
    if (!c) return FTAR_ERR_ARG;
    ftar_sync_fatal(c);
    release_peers(c);
    release_user_peers(c);
    ftar_sync_fatal(c); /* nobody maps our workspace any more */
    for (int b = 0; b < FTAR_NBUF; b++) fdev_free(c->dev, c->ws[b]);
    fdev_free(c->dev, c->hsend);
    fdev_free(c->dev, c->hrecv);
    fdev_free(c->dev, c->pad);
    ftar_ctrl_leave(&c->job);
    if (c->pwflag_dev) fdev_host_unmap(c->dev, (void *)c->job.shm->pwflag);
    fdev_close(c->dev);
    ftar_ctrl_detach(&c->job);
    free(c);
    return FTAR_SUCCESS;
}

int ftar_comm_rank(const ftar_comm *c, int *r)
{
    if (!c || !r) return FTAR_ERR_ARG;
    *r = ftar_my_comm_rank(c);
    return FTAR_SUCCESS;
}
int ftar_comm_size(const ftar_comm *c, int *s)
{
    if (!c || !s) return FTAR_ERR_ARG;
    *s = c->size;
    return FTAR_SUCCESS;
}
int ftar_world_rank(const ftar_comm *c, int *r)
{
    if (!c || !r) return FTAR_ERR_ARG;
    *r = c->wrank;
    return FTAR_SUCCESS;
}
int ftar_world_size(const ftar_comm *c, int *s)
{
    if (!c || !s) return FTAR_ERR_ARG;
    *s = c->wsize;
    return FTAR_SUCCESS;
}
int ftar_comm_device(const ftar_comm *c, int *d)
{
    if (!c || !d) return FTAR_ERR_ARG;
    *d = c->device;
    return FTAR_SUCCESS;
}

int ftar_comm_set_stream(ftar_comm *c, void *stream)
{
    if (!c) return FTAR_ERR_ARG;
    c->user_stream = stream;
    return FTAR_SUCCESS;
}

int ftar_comm_set_option(ftar_comm *c, ftar_option opt, double v)
{
    if (!c || v < 0) return FTAR_ERR_ARG;
    switch (opt) {
    case FTAR_OPT_OVERLAP: c->overlap = v != 0; break;
    case FTAR_OPT_RELAY: c->relay = v != 0; break;
    case FTAR_OPT_RELAY_MIN: c->relay_min = (size_t)v; break;
    case FTAR_OPT_LOOP_SECONDS: c->loop_seconds = v; break;
    case FTAR_OPT_COPY_ENGINE: c->copy_engine = v != 0; break;
    case FTAR_OPT_REDUNDANCY:
        if (v != 0 && v != 1 && v != 2) return FTAR_ERR_ARG;
        c->redundancy = (int)v;
        break;
    case FTAR_OPT_MESH: c->mesh = v != 0; break;
    case FTAR_OPT_ONESHOT_MAX: c->oneshot_max = (size_t)v; break;
    case FTAR_OPT_PUSH: c->push = v >= 2 ? 2 : v != 0; break;
    case FTAR_OPT_MESH_WAIT: c->mesh_wait = v != 0; break;
    case FTAR_OPT_GATE: c->gate = v != 0; break;
    case FTAR_OPT_GATE_MAX: c->gate_max = (size_t)v; break;
    case FTAR_OPT_FLAG_SYNC:
        if (fdev_set_knob(c->dev, FDEV_KNOB_FLAG_SYNC, v != 0)) return FTAR_ERR_ARG;
        break;
    case FTAR_OPT_TREE_UNROLL:
        if (v != (int)v || fdev_set_knob(c->dev, FDEV_KNOB_TREE_UNROLL, (int)v)) return FTAR_ERR_ARG;
        break;
    default: return FTAR_ERR_ARG;
    }
    return FTAR_SUCCESS;
}

int ftar_comm_get_option(const ftar_comm *c, ftar_option opt, double *v)
{
    if (!c || !v) return FTAR_ERR_ARG;
    switch (opt) {
    case FTAR_OPT_OVERLAP: *v = c->overlap; break;
    case FTAR_OPT_RELAY: *v = c->relay; break;
    case FTAR_OPT_RELAY_MIN: *v = (double)c->relay_min; break;
    case FTAR_OPT_LOOP_SECONDS: *v = c->loop_seconds; break;
    case FTAR_OPT_COPY_ENGINE: *v = c->copy_engine; break;
    case FTAR_OPT_REDUNDANCY: *v = c->redundancy; break;
    case FTAR_OPT_MESH: *v = c->mesh; break;
    case FTAR_OPT_ONESHOT_MAX: *v = (double)c->oneshot_max; break;
    case FTAR_OPT_PUSH: *v = c->push; break;
    case FTAR_OPT_MESH_WAIT: *v = c->mesh_wait; break;
    case FTAR_OPT_GATE: *v = c->gate; break;
    case FTAR_OPT_GATE_MAX: *v = (double)c->gate_max; break;
    case FTAR_OPT_FLAG_SYNC: *v = fdev_get_knob(c->dev, FDEV_KNOB_FLAG_SYNC); break;
    case FTAR_OPT_TREE_UNROLL: *v = fdev_get_knob(c->dev, FDEV_KNOB_TREE_UNROLL); break;
    default: return FTAR_ERR_ARG;
    }
    return FTAR_SUCCESS;
}

void ftar_abort(ftar_comm *c, int code) { ftar_ctrl_abort(&c->job, code); }

int ftar_barrier(ftar_comm *c)
{
    if (!c) return FTAR_ERR_ARG;
    ftar_sync_fatal(c);
    return FTAR_SUCCESS;
}

/* ---- synchronisation ------------------------------------------------------ */

/* FTAR_LOOP_SECONDS (the harness's stretch of the schedule, run/run_mpi.sh): the reference's
 * CPU exchanges take seconds, so its random kills land in data movement; a GPU step takes
 * milliseconds.  Instead of idling, the step re-pulls its last peer window (up to
 * FTAR_PAD_BYTES of it) into local scratch again and again until its share of the stretch
 * is used up: a kill then meets pull kernels in flight.  The re-pulls are idempotent reads
 * of a window that is stable until the next barrier (or of a dead peer's still-mapped
 * memory) into a buffer nothing else reads, so results and decisions do not change. */
uint64_t ftar_step_sync(ftar_comm *c, int nsteps)
{
    if (c->loop_seconds > 0 && nsteps > 0) { /* busy (R state), like a rank inside its exchange */
        double t0 = now_s(), d = c->loop_seconds / nsteps;
        if (c->pad_src && !c->pad && fdev_alloc_plain(c->dev, FTAR_PAD_BYTES, &c->pad)) c->pad = NULL;
        while (now_s() - t0 < d) {
            if (c->pad_src && c->pad) {
                size_t n = c->pad_bytes < FTAR_PAD_BYTES ? c->pad_bytes : FTAR_PAD_BYTES;
                fdev_seg s = {FDEV_COPY, FDEV_REMOTE_X, c->pad, c->pad_src, NULL, n / 4, NULL};
                const void *src = c->pad_src;
                if (n / 4 == 0 || ftar_run(c, FTAR_INT32, FTAR_SUM, &s, 1, FDEV_TAG_LOCAL)) break;
                ftar_drain(c);
                c->pad_src = src; /* ftar_run noted it again; keep it for the next round */
            } else {
                ftar_ctrl_poll(&c->job);
            }
        }
    }
    c->pad_src = NULL; /* the next step re-pulls what it reads itself */
    return ftar_sync(c);
}

/* A launch queued behind a gate spins at the head of this rank's stream -- and of any
 * other stream of the process sharing its hardware queue -- until the barrier after which
 * the host opens it.  When that barrier waits long (a late peer), the launch is given up
 * (skip: its workgroups return untouched) and the step launches after the barrier instead:
 * the stall stays bounded by FTAR_GATE_HOLD_US, and the device's own gate timeout is never
 * reached while this process runs. */
static void gate_hold(void *arg)
{
    ftar_comm *c = (ftar_comm *)arg;
    if (!fdev_gate_pending(c->dev)) return;
    fdev_gate_open(c->dev, 1);
    c->stats.gate_holds++;
    if (c->verbose)
        fprintf(stderr, "ftar: rank %d: barrier waited past %.0f us: gated launch given up\n", c->wrank,
                c->gate_hold_s * 1e6);
}

uint64_t ftar_sync(ftar_comm *c)
{
    double t0 = now_s();
    uint64_t next = c->job.seq + 1;
    atomic_store_explicit(&c->job.shm->slot[c->wrank].pubv[next % 2], (next << 16) | ((uint64_t)c->pubval & 0xffff),
                          memory_order_release);
    if (c->gate_hold_s > 0 && fdev_gate_pending(c->dev)) {
        c->job.wait_hook = gate_hold;
        c->job.wait_arg = c;
        c->job.wait_after_s = c->gate_hold_s;
    }
    fdev_trace_note(c->dev, "A %llu", (unsigned long long)next);
    uint64_t snap = ftar_ctrl_agree(&c->job, c->members);
    fdev_trace_note(c->dev, "P %llu", (unsigned long long)c->job.seq);
    c->job.wait_hook = NULL;
    double dt = now_s() - t0;
    c->stats.sync_wait_s += dt;
    c->stats.syncs++;
    if (c->verbose >= 2)
        fprintf(stderr, "ftar[%d] sync %llu waited %.3f ms\n", c->wrank, (unsigned long long)c->job.seq, dt * 1e3);
    return snap & ~c->acked;
}

void ftar_sync_fatal(ftar_comm *c)
{
    uint64_t f = ftar_sync(c);
    if (f) {
        /* a failure outside the tolerant region: MPI_ERRORS_ARE_FATAL */
        ftar_ctrl_abort(&c->job, FTAR_ERR_PROC_FAILED);
    }
}

static void stale_publication(ftar_comm *c, int w, uint64_t s, uint64_t u) __attribute__((noreturn));
static void stale_publication(ftar_comm *c, int w, uint64_t s, uint64_t u)
{
    fprintf(stderr, "ftar: rank %d: stale publication of rank %d (round %llu, tag %llu)\n", c->wrank, w,
            (unsigned long long)s, (unsigned long long)(u >> 16));
    ftar_ctrl_abort(&c->job, FTAR_ERR_STATE);
}

int64_t ftar_peer_pub(ftar_comm *c, int w)
{
    uint64_t s = c->job.seq;
    uint64_t v = atomic_load_explicit(&c->job.shm->slot[w].pubv[s % 2], memory_order_acquire);
    if ((v >> 16) != s) stale_publication(c, w, s, v);
    return (int64_t)(v & 0xffff);
}

int ftar_peer_pub_try(ftar_comm *c, int w, int64_t *v)
{
    uint64_t s = c->job.seq;
    uint64_t u = atomic_load_explicit(&c->job.shm->slot[w].pubv[s % 2], memory_order_acquire);
    if ((u >> 16) == s) {
        *v = (int64_t)(u & 0xffff);
        return 1;
    }
    if (ftar_is_dead(c, w)) return 0; /* died before arriving: no entry for this round */
    stale_publication(c, w, s, u);     /* a live member's entry is always there */
}

int ftar_is_dead(ftar_comm *c, int w) { return ftar_ctrl_is_dead(&c->job, w); }

/* Physical identities, not HIP ordinals: under per-rank HIP_VISIBLE_DEVICES /
 * ROCR_VISIBLE_DEVICES masks every rank may see its own GPU as device 0.  A
 * slot without an identity falls back to the ordinal. */
int ftar_spans_devices(const ftar_comm *c)
{
    const ftar_slot *a = &c->job.shm->slot[c->order[0]];
    for (int i = 1; i < c->size; i++) {
        const ftar_slot *b = &c->job.shm->slot[c->order[i]];
        if (a->phys[0] && b->phys[0] ? strncmp(a->phys, b->phys, sizeof(a->phys)) != 0 : a->device != b->device)
            return 1;
    }
    return 0;
}
void ftar_enter(ftar_comm *c) { ftar_ctrl_enter(&c->job); }
int ftar_peer_entered(ftar_comm *c, int w) { return ftar_ctrl_peer_entered(&c->job, w); }
int ftar_peer_done(ftar_comm *c, int w) { return ftar_ctrl_peer_done(&c->job, w); }

void ftar_launched(ftar_comm *c, int phase, int step)
{
    ftar_ctrl_launched(&c->job);
    ftar_maybe_die(c, phase, step, FTAR_PT_DURING);
}

void ftar_exchange_done(ftar_comm *c) { ftar_ctrl_done(&c->job); }

void ftar_note_launch(ftar_comm *c, const void *remote, size_t bytes)
{
    _Atomic int *w = &c->job.shm->slot[c->wrank].inflight;
    if (remote) {
        atomic_store_explicit(w, FTAR_INFLIGHT_PULL, memory_order_release);
        c->pad_src = remote;
        c->pad_bytes = bytes;
    } else if (atomic_load_explicit(w, memory_order_relaxed) == 0) {
        atomic_store_explicit(w, FTAR_INFLIGHT_LOCAL, memory_order_release);
    }
}

static void note_segs(ftar_comm *c, int dtype, const fdev_seg *segs, int nseg)
{
    const void *remote = NULL;
    size_t bytes = 0;
    int push = 0;
    for (int i = 0; i < nseg && !remote; i++) {
        if (segs[i].remote & FDEV_REMOTE_X) remote = segs[i].x;
        else if (segs[i].kind != FDEV_COPY && (segs[i].remote & FDEV_REMOTE_Y)) remote = segs[i].y;
        push |= (segs[i].remote & FDEV_REMOTE_OUT) != 0;
        bytes = segs[i].n * ftar_esize(dtype);
    }
    ftar_note_launch(c, remote, bytes);
    if (push && !remote) /* stores into peers' HBM: an exchange in flight too (nothing to re-pull) */
        atomic_store_explicit(&c->job.shm->slot[c->wrank].inflight, FTAR_INFLIGHT_PULL, memory_order_release);
}

int ftar_prelaunch(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag, void *stage_dst,
                   const void *stage_src, size_t stage_n)
{
    int gated = 0;
    c->gplan.valid = 0;
    if (!c->gate || nseg <= 0 || nseg > FDEV_MAX_SEGS) return 0;
    if (fdev_run_gated(c->dev, dtype, op, segs, nseg, tag, stage_dst, stage_src, stage_n, &gated)) {
        fprintf(stderr, "ftar: rank %d: launch failed: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    if (!gated) return 0;
    c->gplan = (struct ftar_gplan){1, dtype, op, tag, nseg, {{0}}};
    memcpy(c->gplan.segs, segs, sizeof(fdev_seg) * (size_t)nseg);
    c->stats.gated_launches++;
    return 1;
}

static int seg_eq(const fdev_seg *a, const fdev_seg *b)
{
    return a->kind == b->kind && a->remote == b->remote && a->out == b->out && a->x == b->x &&
           (a->kind == FDEV_COPY || a->y == b->y) && a->n == b->n && a->out2 == b->out2;
}

void ftar_run_gated_or(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    int pending = fdev_gate_pending(c->dev);
    int go = pending && c->gplan.valid && c->gplan.dtype == dtype && c->gplan.op == op && c->gplan.tag == tag &&
             c->gplan.nseg == nseg;
    for (int i = 0; go && i < nseg; i++) go = seg_eq(&segs[i], &c->gplan.segs[i]);
    if (c->gplan.valid && !go) c->stats.gated_skips++; /* given up here, or already by another launch */
    c->gplan.valid = 0;
    if (pending) fdev_gate_open(c->dev, !go);
    if (go) {
        note_segs(c, dtype, segs, nseg);
        return;
    }
    if (nseg) ftar_run(c, dtype, op, segs, nseg, tag);
}

/* A _host entry point's copy (H2D / D2H, or the wait for one) failed on this rank: the job
 * ends (MPI_Abort), as the device path ends it on a launch error.  Returning FTAR_ERR_DEVICE
 * alone would leave the peers spinning in the collective's next barrier for a rank that is
 * alive but gone (the reference's MPI_ERRORS_ARE_FATAL outside the tolerant
 * loops, raben/rabenseifner.c:358-360, rd/recursive_doubling.c:73-75). */
void ftar_host_copy_failed(ftar_comm *c, const char *what)
{
    fprintf(stderr, "ftar: rank %d: %s failed: %s\n", c->wrank, what, fdev_last_error());
    ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
}

int ftar_drain(ftar_comm *c)
{
    double t0 = now_s();
    int rc = fdev_sync(c->dev, ftar_ctrl_poll, &c->job);
    if (!rc) atomic_store_explicit(&c->job.shm->slot[c->wrank].inflight, 0, memory_order_release);
    c->stats.drain_s += now_s() - t0;
    if (rc) {
        fprintf(stderr, "ftar: rank %d: device error: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    return rc;
}

void *ftar_flag(ftar_comm *c, int w)
{
    return c->pwflag_dev ? (char *)c->pwflag_dev + (size_t)w * sizeof(c->job.shm->pwflag[0]) : NULL;
}

int ftar_watch_peers(void *arg)
{
    ftar_comm *c = (ftar_comm *)arg;
    ftar_ctrl_poll(&c->job); /* an abort ends this process here */
    double t = now_s();
    if (t - c->watch_t < 50e-6) return 0;
    c->watch_t = t;
    for (int i = 0; i < c->size; i++) {
        int w = c->order[i];
        if (w != c->wrank && ftar_is_dead(c, w)) {
            fdev_peer_wait_abort(c->dev); /* the wait returns; the next agree reports the failure */
            break;
        }
    }
    return 0;
}

int ftar_drain_watch(ftar_comm *c)
{
    double t0 = now_s();
    int rc = fdev_sync(c->dev, ftar_watch_peers, c);
    if (!rc) atomic_store_explicit(&c->job.shm->slot[c->wrank].inflight, 0, memory_order_release);
    c->stats.drain_s += now_s() - t0;
    if (rc) {
        fprintf(stderr, "ftar: rank %d: device error: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    return rc;
}

int ftar_drain_bg(ftar_comm *c)
{
    double t0 = now_s();
    int rc = fdev_sync_bg(c->dev, ftar_ctrl_poll, &c->job);
    c->stats.drain_s += now_s() - t0;
    if (rc) {
        fprintf(stderr, "ftar: rank %d: device error: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    return rc;
}

int ftar_run_bg(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    note_segs(c, dtype, segs, nseg);
    int rc = fdev_run_bg(c->dev, dtype, op, segs, nseg, tag);
    if (rc) {
        fprintf(stderr, "ftar: rank %d: launch failed: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    return rc;
}

int ftar_run(ftar_comm *c, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    note_segs(c, dtype, segs, nseg);
    int rc = fdev_run(c->dev, dtype, op, segs, nseg, tag);
    if (rc) {
        fprintf(stderr, "ftar: rank %d: launch failed: %s\n", c->wrank, fdev_last_error());
        ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
    }
    return rc;
}

void ftar_regroup(ftar_comm *c, int dead, int repl)
{
    int neworder[FTAR_MAX_RANKS];
    int k = 0;
    for (int i = 0; i < c->size; i++)
        if (i != repl) neworder[k++] = c->order[i];
    if (repl != dead) neworder[(dead < repl) ? dead : dead - 1] = c->order[repl];
    memcpy(c->order, neworder, sizeof(int) * (size_t)k);
    c->size = k;
    recompute_members(c);
}

void ftar_shrink(ftar_comm *c, uint64_t failed)
{
    int k = 0;
    for (int i = 0; i < c->size; i++)
        if (!(failed & (1ull << c->order[i]))) c->order[k++] = c->order[i];
    c->size = k;
    recompute_members(c);
}

/* A comm of one rank -- p = 1, or every peer lost -- has no exchange: the result is the
 * input (raben/util.c:35-42 copy_buffer; rd: N = 1 returns src, DESIGN.md deviation 4).
 * Nothing is exported or staged and the workspace is not touched: one copy launch (none in
 * place), one drain and the closing barrier; the kill points of the schedule's pre- and
 * post-phases are passed in their usual order. */
int ftar_single_rank(ftar_comm *c, const void *sbuf, void *rbuf, size_t bytes)
{
    fdev_order_after(c->dev, c->user_stream);
    ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_BEFORE);
    ftar_enter(c);
    if (sbuf != rbuf) {
        fdev_seg s = {FDEV_COPY, 0, rbuf, sbuf, NULL, bytes / 4, NULL};
        ftar_run(c, FTAR_INT32, FTAR_SUM, &s, 1, FDEV_TAG_LOCAL);
    }
    ftar_launched(c, FTAR_PH_PRE, 0);
    ftar_drain(c);
    ftar_exchange_done(c);
    ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_AFTER);
    ftar_maybe_die(c, FTAR_PH_PRE, 0, FTAR_PT_BARRIER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BEFORE);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_DURING);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_AFTER);
    ftar_maybe_die(c, FTAR_PH_POST, 0, FTAR_PT_BARRIER);
    ftar_sync_fatal(c);
    ftar_stats_end(c);
    return FTAR_SUCCESS;
}

/* ---- workspace ------------------------------------------------------------ */

void *ftar_buf(ftar_comm *c, int w, int b)
{
    if (b == WS_IN) { /* this call's input may be the rank's own send buffer */
        if (w == c->wrank) return c->in_alias ? (void *)c->in_alias : c->ws[WS_IN];
        if (c->peer_in[w]) return c->peer_in[w];
    }
    return (w == c->wrank) ? c->ws[b] : c->peer[w][b];
}

void *ftar_local(ftar_comm *c, int b)
{
    if (b == WS_UIN) return (void *)c->uin;
    if (b == WS_UOUT) return c->uout;
    return ftar_buf(c, c->wrank, b);
}

/* Grow the exported workspace.  The new blocks are allocated, exported and imported
 * while the old ones -- ours and our imports of the peers' -- are still mapped, and only
 * then are the old mappings closed and the old blocks freed.  The other order (close,
 * free, allocate, export) let a fresh hipMalloc land on the address range an import had
 * occupied a moment before, and the runtime then refused to export it
 * (hipIpcGetMemHandle: invalid argument; seen once in 8-rank regrowth sweeps, round 1 and
 * round 2).  Costs the old workspace's memory for the length of the call. */
int ftar_ensure_workspace(ftar_comm *c, size_t bytes)
{
    if (bytes <= c->ws_bytes && c->ws[0]) return FTAR_SUCCESS;
    if (c->ws[0] && bytes < 2 * c->ws_bytes) bytes = 2 * c->ws_bytes; /* grow geometrically: few re-exports */
    size_t nb = (bytes + WS_ALIGN - 1) / WS_ALIGN * WS_ALIGN;
    if (nb == 0) nb = WS_ALIGN;
    void *old_ws[FTAR_NBUF];
    void *old_peer[FTAR_MAX_RANKS][FTAR_NBUF];
    memcpy(old_ws, c->ws, sizeof(old_ws));
    memcpy(old_peer, c->peer, sizeof(old_peer));
    memset(c->peer, 0, sizeof(c->peer));
    ftar_sync_fatal(c); /* everybody is here: nobody reads a workspace until this returns */
    ftar_slot *me = &c->job.shm->slot[c->wrank];
    for (int b = 0; b < FTAR_NBUF; b++) {
        int rc = fdev_alloc_shared(c->dev, nb, &c->ws[b], me->handle[b]);
        if (rc) {
            fprintf(stderr, "ftar: rank %d: workspace allocation of %zu B failed: %s\n", c->wrank, nb,
                    fdev_last_error());
            ftar_ctrl_abort(&c->job, FTAR_ERR_NOMEM);
        }
        fdev_trace_region(c->dev, c->ws[b], nb, c->wrank, ws_name[b]);
    }
    me->ws_bytes = nb;
    atomic_fetch_add(&me->ws_gen, 1);
    c->ws_bytes = nb;
    ftar_sync_fatal(c); /* every new handle is published */
    for (int i = 0; i < c->size; i++) {
        int w = c->order[i];
        if (w == c->wrank) continue;
        ftar_slot *s = &c->job.shm->slot[w];
        for (int b = 0; b < FTAR_NBUF; b++) {
            int rc = fdev_import(c->dev, s->handle[b], &c->peer[w][b]);
            if (rc) {
                fprintf(stderr, "ftar: rank %d: cannot map rank %d buffer %d: %s\n", c->wrank, w, b,
                        fdev_last_error());
                ftar_ctrl_abort(&c->job, FTAR_ERR_DEVICE);
            }
            fdev_trace_region(c->dev, c->peer[w][b], s->ws_bytes, w, ws_name[b]);
        }
        c->peer_bytes[w] = s->ws_bytes;
        c->peer_gen[w] = atomic_load(&s->ws_gen);
    }
    for (int w = 0; w < c->wsize; w++) /* the old mappings, dead ranks' included */
        for (int b = 0; b < FTAR_NBUF; b++)
            if (old_peer[w][b]) {
                fdev_trace_unregion(c->dev, old_peer[w][b]);
                fdev_unimport(c->dev, old_peer[w][b]);
            }
    ftar_sync_fatal(c); /* nobody maps the old buffers */
    for (int b = 0; b < FTAR_NBUF; b++) {
        fdev_trace_unregion(c->dev, old_ws[b]);
        fdev_free(c->dev, old_ws[b]);
    }
    return FTAR_SUCCESS;
}

/* Pinned staging of the _host entry points, grown on demand.  Rank-local: whether a call
 * stages at all is decided per rank (a rank whose caller buffers are pinned runs the
 * device entry point on them in place and never gets here), so this does no collective
 * work.  A rank that cannot allocate ends the job (MPI_Abort) rather than returning alone
 * while its peers wait for it in the collective's first barrier. */
int ftar_ensure_staging(ftar_comm *c, size_t bytes)
{
    if (bytes == 0 || (bytes <= c->hbytes && c->hsend && c->hrecv)) return FTAR_SUCCESS;
    fdev_free(c->dev, c->hsend);
    fdev_free(c->dev, c->hrecv);
    c->hsend = c->hrecv = NULL;
    c->hbytes = 0;
    if (fdev_alloc_plain(c->dev, bytes, &c->hsend) || fdev_alloc_plain(c->dev, bytes, &c->hrecv)) {
        fprintf(stderr, "ftar: rank %d: staging allocation of %zu B failed: %s\n", c->wrank, bytes,
                fdev_last_error());
        fdev_free(c->dev, c->hsend);
        c->hsend = NULL;
        ftar_ctrl_abort(&c->job, FTAR_ERR_NOMEM);
    }
    c->hbytes = bytes;
    return FTAR_SUCCESS;
}

/* ---- statistics ----------------------------------------------------------- */

/* One user call = one stats record and one call index (FTAR_KILL ':call'), also when the
 * host pipeline runs it as several chunk Allreduces (c->chunk_cont set for chunks 2..n):
 * their counters accumulate into the record the first chunk opened. */
void ftar_stats_begin(ftar_comm *c)
{
    if (!c->chunk_cont) {
        c->ncalls++;
        memset(&c->stats, 0, sizeof(c->stats));
        c->t0 = now_s();
    }
    fdev_counters_reset(c->dev);
}

void ftar_stats_end(ftar_comm *c)
{
    /* A gated launch still waiting at the end of the call (a recovery ended the loop before
     * the step it was queued for): give it up now, rather than leave it to time out */
    if (fdev_gate_pending(c->dev)) {
        fdev_gate_open(c->dev, 1);
        c->stats.gated_skips++;
    }
    c->gplan.valid = 0;
    c->gnext.valid = 0;
    fdev_counters k;
    fdev_counters_get(c->dev, &k);
    c->stats.wall_s = now_s() - c->t0;
    c->stats.kernel_ms += k.ms[0] + k.ms[1] + k.ms[2] + k.ms[3] + k.ms[4];
    c->stats.bg_kernel_ms += k.ms[FDEV_TAG_BG];
    c->stats.step0_kernel_ms += k.ms[FDEV_TAG_STEP0];
    c->stats.link_bytes += k.link_bytes;
    c->stats.hbm_bytes += k.hbm_bytes;
    c->stats.kernels += k.launches[0] + k.launches[1] + k.launches[2] + k.launches[3] + k.launches[4];
    c->stats.comm_size_after = c->size;
    c->stats.export_retries = fdev_export_retries(c->dev);
    c->stats.user_stream_waits = fdev_user_host_waits(c->dev);
    c->stats.gate_relaunches = fdev_gate_relaunches(c->dev);
    ftar_inputs_done(c);
}

double ftar_link_bytes(ftar_comm *c)
{
    fdev_counters k;
    fdev_counters_get(c->dev, &k);
    return k.link_bytes;
}

int ftar_last_stats(const ftar_comm *c, ftar_stats *out)
{
    if (!c || !out) return FTAR_ERR_ARG;
    *out = c->stats;
    return FTAR_SUCCESS;
}

int ftar_set_profiling(ftar_comm *c, int on)
{
    if (!c) return FTAR_ERR_ARG;
    c->profiling = on;
    fdev_profiling(c->dev, on);
    return FTAR_SUCCESS;
}

/* ---- local reduce --------------------------------------------------------- */

int ftar_reduce_local(const void *in, void *inout, size_t count, ftar_dtype dtype, ftar_op op, void *stream)
{
    int rc = ftar_check_op((int)dtype, (int)op);
    if (rc) return rc;
    if (count && (!in || !inout)) return FTAR_ERR_ARG;
    rc = fdev_reduce_local(in, inout, count, (int)dtype, (int)op, stream);
    if (rc) fprintf(stderr, "ftar_reduce_local: %s\n", fdev_last_error());
    return rc;
}

int ftar_set_reduce_variant(int v) { return fdev_set_reduce_variant(v) ? FTAR_ERR_ARG : FTAR_SUCCESS; }

const char *ftar_version(void) { return "ftar-mi355x 0.1 (gfx950)"; }
