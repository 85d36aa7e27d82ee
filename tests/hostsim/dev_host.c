/*
 * dev_host.c -- TEST-ONLY host implementation of the device layer (csrc/ftar_dev.h).
 *
 * Lets the CPU test suite run the product's real host logic -- control plane, agree,
 * both schedules, both error handlers, the launcher, kill -9 injection -- as N real
 * processes without a GPU.  "Device" allocations are POSIX shared-memory objects,
 * the "IPC handle" is the object name, kernels are plain loops.  It is linked only
 * into tests/hostsim/_build/libftar_hostsim.so, never into lib/libftar.so, and it is
 * not used for any numerical parity claim about the HIP kernels.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <fcntl.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "../../fault-tolerant_amd/csrc/ftar_dev.h"

struct ftar_dev {
    int device;
    int profiling;
    fdev_counters ctr;
    /* a gated launch (fdev_tree_batch_gated / fdev_run_gated): held until its gate opens,
     * run then unless skipped; any other launch meanwhile gives it up first (opened as
     * skip), as the GPU build does */
    int gate_pending;
    struct {
        int batch; /* 1: a tree batch, 0: segments */
        int dtype, op, nsrc, ntree, tag, nseg;
        const void *src[FDEV_MAX_BATCH * FDEV_MAX_BATCH];
        unsigned remote[FDEV_MAX_BATCH];
        void *out[FDEV_MAX_BATCH];
        size_t n[FDEV_MAX_BATCH];
        fdev_seg segs[FDEV_MAX_SEGS];
    } gated;
    uint64_t gates_run, gates_skipped;
    /* fdev_peer_wait: the next launch runs behind it (pw_pending), if the wait succeeded (pw_go) */
    int pw_pending, pw_armed, pw_go, pw_abort;
    int flag_sync, tree_unroll; /* knobs: no flag path here; flag_sync = 0 turns the gates off, as on the GPU */
};

#define MAXMAP 256
static struct {
    void *p;
    size_t n;
    char name[64];
    int own;
    uint64_t id; /* allocation id (exportable allocations) */
} g_map[MAXMAP];
static uint64_t g_next_id;
static int g_seq;
static char g_err[256];

const char *fdev_last_error(void) { return g_err; }

int fdev_device_count(int *n)
{
    *n = 8;
    return 0;
}

int fdev_open(int device, ftar_dev **out)
{
    ftar_dev *d = (ftar_dev *)calloc(1, sizeof(ftar_dev));
    d->device = device;
    d->flag_sync = getenv("FTAR_FLAG_SYNC") ? atoi(getenv("FTAR_FLAG_SYNC")) != 0 : 1;
    d->tree_unroll = 1;
    *out = d;
    return 0;
}

int fdev_set_knob(ftar_dev *d, int knob, int value)
{
    if (knob == FDEV_KNOB_FLAG_SYNC) {
        if (d->gate_pending) fdev_gate_open(d, 1);
        d->flag_sync = value != 0;
        return 0;
    }
    if (knob == FDEV_KNOB_TREE_UNROLL && (value == 1 || value == 2 || value == 4)) {
        d->tree_unroll = value; /* the loops here have no vectors: same result */
        return 0;
    }
    return 13;
}

int fdev_get_knob(const ftar_dev *d, int knob)
{
    return knob == FDEV_KNOB_FLAG_SYNC ? d->flag_sync : knob == FDEV_KNOB_TREE_UNROLL ? d->tree_unroll : -1;
}

int fdev_gate_relaunches(const ftar_dev *d) { return 0; }

void fdev_close(ftar_dev *d) { free(d); }
int fdev_device(const ftar_dev *d) { return d->device; }

/* "hostsim:<ordinal>", or the FTAR_RANK-th entry of FTAR_HOSTSIM_PHYS (comma list): the
 * case of ranks that see different GPUs under one ordinal (per-rank visibility masks) */
int fdev_physical_id(ftar_dev *d, char *out, size_t n)
{
    const char *l = getenv("FTAR_HOSTSIM_PHYS"), *r = getenv("FTAR_RANK");
    if (l && r) {
        int k = atoi(r);
        while (k-- > 0 && l) {
            l = strchr(l, ',');
            if (l) l++;
        }
        if (l) {
            size_t m = strcspn(l, ",");
            snprintf(out, n, "%.*s", (int)m, l);
            return 0;
        }
    }
    snprintf(out, n, "hostsim:%d", d->device);
    return 0;
}

static int put_map(void *p, size_t n, const char *name, int own)
{
    for (int i = 0; i < MAXMAP; i++)
        if (!g_map[i].p) {
            g_map[i].p = p;
            g_map[i].n = n;
            g_map[i].own = own;
            g_map[i].id = own ? ++g_next_id : 0;
            snprintf(g_map[i].name, sizeof(g_map[i].name), "%.63s", name);
            return 0;
        }
    return -1;
}

/* "Device memory" is /dev/shm, which the whole container shares: every segment is backed
 * when it is allocated (posix_fallocate), so exhaustion is an allocation error here -- the
 * library then ends the job with FTAR_ERR_NOMEM -- and not a SIGBUS at the first touch of a
 * page, which the job would see as a rank death.  FTAR_HOSTSIM_SHM_BUDGET=<bytes>
 * (test-only) makes this process's allocations beyond that total fail the same way. */
int fdev_alloc_shared(ftar_dev *d, size_t bytes, void **ptr, void *handle)
{
    static size_t allocated;
    char name[64];
    const char *tag = getenv("FTAR_HOSTSIM_TAG"), *budget = getenv("FTAR_HOSTSIM_SHM_BUDGET");
    if (budget && allocated + bytes > (size_t)strtoull(budget, NULL, 10)) {
        snprintf(g_err, sizeof(g_err), "out of shared memory: %zu B more than FTAR_HOSTSIM_SHM_BUDGET=%s allows",
                 bytes, budget);
        return 102;
    }
    snprintf(name, sizeof(name), "/ftarhs-%s-%d-%d", tag ? tag : "x", (int)getpid(), g_seq++);
    int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) {
        snprintf(g_err, sizeof(g_err), "shm_open %s failed", name);
        if (fd >= 0) {
            close(fd);
            shm_unlink(name);
        }
        return 101;
    }
    int fe = bytes ? posix_fallocate(fd, 0, (off_t)bytes) : 0;
    if (fe != 0) {
        snprintf(g_err, sizeof(g_err), "out of shared memory: %zu B for %s (%s)", bytes, name, strerror(fe));
        close(fd);
        shm_unlink(name);
        return 102;
    }
    void *p = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        shm_unlink(name);
        return 102;
    }
    allocated += bytes;
    memset(handle, 0, FDEV_HANDLE_BYTES);
    snprintf((char *)handle, FDEV_HANDLE_BYTES, "%s", name);
    put_map(p, bytes, name, 1);
    *ptr = p;
    return 0;
}

/* "device" allocations of the library (the _host entry points' staging buffers) are
 * shared-memory objects too, so they can be exported like hipMalloc memory */
int fdev_alloc_plain(ftar_dev *d, size_t bytes, void **ptr)
{
    /* FTAR_HOSTSIM_FAIL_PLAIN=k: the k-th staging allocation (1-based) of rank
     * FTAR_HOSTSIM_FAIL_RANK (default 0) fails, as hipMalloc out of memory would */
    static int nplain;
    const char *k = getenv("FTAR_HOSTSIM_FAIL_PLAIN"), *fr = getenv("FTAR_HOSTSIM_FAIL_RANK");
    const char *me = getenv("FTAR_RANK");
    if (k && ++nplain == atoi(k) && me && atoi(me) == (fr ? atoi(fr) : 0)) {
        snprintf(g_err, sizeof(g_err), "injected staging allocation failure");
        return 102;
    }
    unsigned char h[FDEV_HANDLE_BYTES];
    return fdev_alloc_shared(d, bytes ? bytes : 1, ptr, h);
}

static int drop(void *ptr, int unlink_it)
{
    for (int i = 0; i < MAXMAP; i++)
        if (g_map[i].p == ptr) {
            munmap(ptr, g_map[i].n);
            if (unlink_it && g_map[i].own) shm_unlink(g_map[i].name);
            g_map[i].p = NULL;
            return 0;
        }
    return -1;
}

int fdev_host_map(ftar_dev *d, void *p, size_t bytes, void **devp)
{
    *devp = p; /* host memory is this layer's device memory */
    return 0;
}

void fdev_host_unmap(ftar_dev *d, void *p) {}

/* TEST-ONLY: "device memory" a caller owns (ftar_probe's send buffers under
 * FTAR_PROBE_CYCLE_SEQ): a shared-memory object like the library's own, so the library can
 * export it and its peers map it, as hipMalloc memory */
void *ftar_hostsim_device_alloc(size_t bytes)
{
    void *p = NULL;
    unsigned char h[FDEV_HANDLE_BYTES];
    return fdev_alloc_shared(NULL, bytes ? bytes : 1, &p, h) == 0 ? p : NULL;
}

void ftar_hostsim_device_free(void *p) { (void)drop(p, 1); }

int fdev_free(ftar_dev *d, void *ptr)
{
    if (!ptr) return 0;
    if (drop(ptr, 1) != 0) free(ptr);
    return 0;
}

int fdev_import(ftar_dev *d, const void *handle, void **ptr)
{
    /* FTAR_HOSTSIM_FAIL_IMPORT=k: the k-th and later imports of this process fail (the
     * workspace takes the first 4 (p - 1); later ones are peers' send buffers) */
    static int nimport;
    const char *fi = getenv("FTAR_HOSTSIM_FAIL_IMPORT");
    if (fi && ++nimport >= atoi(fi)) {
        snprintf(g_err, sizeof(g_err), "import refused (FTAR_HOSTSIM_FAIL_IMPORT)");
        return 101;
    }
    char name[FDEV_HANDLE_BYTES + 1];
    memcpy(name, handle, FDEV_HANDLE_BYTES);
    name[FDEV_HANDLE_BYTES] = 0;
    int fd = shm_open(name, O_RDWR, 0600);
    if (fd < 0) {
        snprintf(g_err, sizeof(g_err), "import %s failed", name);
        return 101;
    }
    struct stat st;
    fstat(fd, &st);
    void *p = mmap(NULL, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return 101;
    put_map(p, (size_t)st.st_size, name, 0);
    *ptr = p;
    return 0;
}

int fdev_unimport(ftar_dev *d, void *ptr) { return drop(ptr, 0) == 0 ? 0 : 101; }

/* shareable when [ptr, ptr + bytes) lies in one of this process's shared-memory
 * allocations; caller memory from malloc is not (the library then stages it) */
int fdev_export_range(ftar_dev *d, const void *ptr, size_t bytes, void *handle, uint64_t *id, size_t *offset)
{
    const char *p = (const char *)ptr;
    for (int i = 0; i < MAXMAP; i++) {
        const char *b = (const char *)g_map[i].p;
        if (!b || !g_map[i].own || p < b || p + bytes > b + g_map[i].n) continue;
        if (handle) { /* NULL: identify only */
            memset(handle, 0, FDEV_HANDLE_BYTES);
            snprintf((char *)handle, FDEV_HANDLE_BYTES, "%s", g_map[i].name);
        }
        *id = g_map[i].id;
        *offset = (size_t)(p - b);
        return 0;
    }
    return 1;
}

/* one element op, the kernels' operand roles (ftar_kernels.hip apply): the arithmetic
 * ops for every type, MPI's logical / bitwise ops (op >= 4) for the integer types only */
#define DEF_OP(NAME, T, UT, INTEGER)                                                                        \
    static inline T NAME(int op, T a, T b)                                                                  \
    {                                                                                                       \
        switch (op) {                                                                                       \
        case 0: return (T)((UT)a + (UT)b);                                                                  \
        case 1: return (T)((UT)a * (UT)b);                                                                  \
        case 2: return (a > b) ? a : b;                                                                     \
        case 3: return (a < b) ? a : b;                                                                     \
        default: return INTEGER(op, a, b);                                                                  \
        }                                                                                                   \
    }
#define INT_OPS(op, a, b)                                                                                   \
    ((op) == 4 ? ((a) != 0 && (b) != 0) : (op) == 5 ? ((a) & (b)) : (op) == 6 ? ((a) != 0 || (b) != 0)       \
     : (op) == 7 ? ((a) | (b)) : (op) == 8 ? (((a) != 0) != ((b) != 0)) : ((a) ^ (b)))
#define NO_OPS(op, a, b) (a) /* never reached: the library refuses these ops on float types */
DEF_OP(op_i32, int32_t, uint32_t, INT_OPS)
DEF_OP(op_i64, int64_t, uint64_t, INT_OPS)
DEF_OP(op_f32, float, float, NO_OPS)
DEF_OP(op_f64, double, double, NO_OPS)

#define LOOP(T, FN)                                                                                         \
    do {                                                                                                    \
        T *o = (T *)s->out;                                                                                 \
        const T *x = (const T *)s->x, *y = (const T *)s->y;                                                 \
        for (size_t i = 0; i < s->n; i++) o[i] = FN(op, x[i], y[i]);                                        \
    } while (0)

static size_t esz(int dt) { return (dt == 0 || dt == 1) ? 4 : 8; }

int fdev_run(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    if (d->gate_pending) fdev_gate_open(d, 1);
    if (d->pw_pending) { /* behind a peer wait: runs only if every peer's flag arrived */
        d->pw_pending = 0;
        d->pw_armed = 1;
        if (!d->pw_go) return 0;
    }
    for (int k = 0; k < nseg; k++) {
        const fdev_seg *s = &segs[k];
        if (s->kind == FDEV_COPY) {
            memmove(s->out, s->x, s->n * esz(dtype));
        } else {
            switch (dtype) {
            case 0: LOOP(int32_t, op_i32); break;
            case 1: LOOP(float, op_f32); break;
            case 2: LOOP(int64_t, op_i64); break;
            default: LOOP(double, op_f64); break;
            }
        }
        if (s->out2) memmove(s->out2, s->out, s->n * esz(dtype));
        if (s->remote & FDEV_REMOTE_OUT) d->ctr.link_bytes += (double)s->n * (double)esz(dtype);
    }
    d->ctr.launches[tag]++;
    return 0;
}

#define TREE(T, FN)                                                                                         \
    do {                                                                                                    \
        for (size_t i = 0; i < n; i++) {                                                                    \
            T v[16];                                                                                        \
            for (int j = 0; j < nsrc; j++) v[j] = ((const T *)src[j])[i];                                   \
            for (int w = 1; w < nsrc; w <<= 1)                                                              \
                for (int j = 0; j < nsrc; j += 2 * w) v[j] = FN(op, v[j], v[j + w]);                        \
            ((T *)out)[i] = v[0];                                                                           \
        }                                                                                                   \
    } while (0)

int fdev_tree_out(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, unsigned remote_mask, void *out,
                  void *const *more, int nmore, int more_remote, size_t n, int tag);

int fdev_tree(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, unsigned remote_mask, void *out,
              size_t n, int tag)
{
    return fdev_tree_out(d, dtype, op, src, nsrc, remote_mask, out, NULL, 0, 0, n, tag);
}

int fdev_tree_out(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, unsigned remote_mask, void *out,
                  void *const *more, int nmore, int more_remote, size_t n, int tag)
{
    if (!(nsrc == 2 || nsrc == 4 || nsrc == 8 || nsrc == 16)) return 13;
    if (d->gate_pending) fdev_gate_open(d, 1);
    switch (dtype) {
    case 0: TREE(int32_t, op_i32); break;
    case 1: TREE(float, op_f32); break;
    case 2: TREE(int64_t, op_i64); break;
    default: TREE(double, op_f64); break;
    }
    for (int o = 0; o < nmore; o++) memcpy(more[o], out, n * esz(dtype));
    d->ctr.link_bytes += (double)n * (double)esz(dtype) * (__builtin_popcount(remote_mask) + (more_remote ? nmore : 0));
    d->ctr.launches[tag]++;
    return 0;
}

int fdev_check_ptr(ftar_dev *d, const void *ptr, size_t bytes) { return ptr == NULL; }
/* host-sim: "device" memory is host memory, so every buffer could be used in place; the
 * _host entry points stage unless FTAR_HOSTSIM_PINNED=1 makes the caller's buffers count
 * as pinned (the zero-copy route of the GPU build, tested with kills on CPU) */
int fdev_host_pinned(const void *ptr) { return ptr && getenv("FTAR_HOSTSIM_PINNED") && atoi(getenv("FTAR_HOSTSIM_PINNED")); }

int fdev_tree_batch(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, const unsigned *remote_mask,
                    void *const *out, const size_t *n, int ntree, int tag)
{
    if (!(nsrc == 2 || nsrc == 4 || nsrc == 8) || ntree < 1 || ntree > FDEV_MAX_BATCH) return 13;
    for (int t = 0; t < ntree; t++) {
        int rc = fdev_tree(d, dtype, op, src + (size_t)t * nsrc, nsrc, remote_mask[t], out[t], n[t], tag);
        if (rc) return rc;
        d->ctr.launches[tag]--; /* one launch for the batch */
    }
    d->ctr.launches[tag]++;
    return 0;
}

/* host-sim: every launch can be gated (FTAR_HOSTSIM_GATE=0 turns it off, as a GPU whose
 * launch could not be); held, and run when the gate opens */
static int can_gate(const ftar_dev *d)
{
    const char *e = getenv("FTAR_HOSTSIM_GATE");
    return !(e && !atoi(e)) && !d->profiling && !d->gate_pending && d->flag_sync;
}

/* TEST-ONLY (FTAR_HOSTSIM_GATE_CORRUPT=1): a gated launch that runs gets its first output
 * element wrong -- the stand-in for a gated path that is not exact on some hardware, which
 * bench.py's exactness leg must catch and route around (tests/test_bench_logic.py) */
static void corrupt_gated(ftar_dev *d)
{
    const char *e = getenv("FTAR_HOSTSIM_GATE_CORRUPT");
    if (!e || !atoi(e)) return;
    size_t n = d->gated.batch ? d->gated.n[0] : d->gated.segs[0].n;
    void *outs[2] = {d->gated.batch ? d->gated.out[0] : d->gated.segs[0].out, d->gated.batch ? NULL : d->gated.segs[0].out2};
    for (int k = 0; k < 2; k++) {
        void *o = outs[k];
        if (!o || !n) continue;
        if (d->gated.dtype == 0) ((int32_t *)o)[0] += 1;
        else if (d->gated.dtype == 1) ((float *)o)[0] += 1.0f;
        else if (d->gated.dtype == 2) ((int64_t *)o)[0] += 1;
        else ((double *)o)[0] += 1.0;
    }
}

int fdev_tree_batch_gated(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc,
                          const unsigned *remote_mask, void *const *out, const size_t *n, int ntree, int tag,
                          int *gated)
{
    *gated = 0;
    if (!can_gate(d)) return 0;
    if (!(nsrc == 2 || nsrc == 4 || nsrc == 8) || ntree < 1 || ntree > FDEV_MAX_BATCH) return 13;
    d->gated.batch = 1;
    d->gated.dtype = dtype;
    d->gated.op = op;
    d->gated.nsrc = nsrc;
    d->gated.ntree = ntree;
    d->gated.tag = tag;
    memcpy(d->gated.src, src, sizeof(void *) * (size_t)(nsrc * ntree));
    memcpy(d->gated.remote, remote_mask, sizeof(unsigned) * (size_t)ntree);
    memcpy(d->gated.out, out, sizeof(void *) * (size_t)ntree);
    memcpy(d->gated.n, n, sizeof(size_t) * (size_t)ntree);
    d->gate_pending = 1;
    *gated = 1;
    return 0;
}

int fdev_tree_batch_staged_gated(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc,
                                 const unsigned *remote_mask, void *const *out, const size_t *n, int ntree, int tag,
                                 void *stage_dst, const void *stage_src, size_t stage_n, int *gated)
{
    *gated = 0;
    if (!can_gate(d)) return 0;
    if (stage_dst && stage_n) memmove(stage_dst, stage_src, stage_n * esz(dtype)); /* before the gate, always */
    return fdev_tree_batch_gated(d, dtype, op, src, nsrc, remote_mask, out, n, ntree, tag, gated);
}

int fdev_run_gated(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag, void *stage_dst,
                   const void *stage_src, size_t stage_n, int *gated)
{
    *gated = 0;
    if (!can_gate(d)) return 0;
    if (stage_dst && stage_n) memmove(stage_dst, stage_src, stage_n * esz(dtype)); /* before the gate, always */
    if (nseg < 0 || nseg > FDEV_MAX_SEGS) return 13;
    d->gated.batch = 0;
    d->gated.dtype = dtype;
    d->gated.op = op;
    d->gated.tag = tag;
    d->gated.nseg = nseg;
    memcpy(d->gated.segs, segs, sizeof(fdev_seg) * (size_t)nseg);
    d->gate_pending = 1;
    *gated = 1;
    return 0;
}

int fdev_gate_open(ftar_dev *d, int skip)
{
    if (!d->gate_pending) return 0;
    d->gate_pending = 0;
    if (skip) {
        d->gates_skipped++;
        return 0;
    }
    d->gates_run++;
    int rc = d->gated.batch ? fdev_tree_batch(d, d->gated.dtype, d->gated.op, d->gated.src, d->gated.nsrc, d->gated.remote,
                                              d->gated.out, d->gated.n, d->gated.ntree, d->gated.tag)
                            : fdev_run(d, d->gated.dtype, d->gated.op, d->gated.segs, d->gated.nseg, d->gated.tag);
    corrupt_gated(d);
    return rc;
}

int fdev_gate_pending(const ftar_dev *d) { return d->gate_pending; }

/* host-sim: the flag is a word of the shared-memory W, the wait spins here on the host */
int fdev_peer_wait(ftar_dev *d, void *flag, void *const *peer_flags, int npeers, uint64_t token,
                   int (*poll)(void *), void *arg)
{
    if (!flag || npeers < 1 || npeers > FDEV_MAX_PEERS) return 13;
    if (d->gate_pending) fdev_gate_open(d, 1);
    __atomic_store_n((uint64_t *)flag, token, __ATOMIC_RELEASE);
    d->pw_abort = d->pw_go = 0;
    /* the device's give-up, as on the GPU: FTAR_GATE_TIMEOUT_MS (default 60 s) */
    const char *gt = getenv("FTAR_GATE_TIMEOUT_MS");
    const double limit = (gt ? atof(gt) : 60000.0) * 1e-3;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (;;) {
        int all = 1;
        for (int i = 0; i < npeers && all; i++) all = __atomic_load_n((const uint64_t *)peer_flags[i], __ATOMIC_ACQUIRE) >= token;
        if (all) {
            d->pw_go = 1;
            break;
        }
        if (poll) poll(arg);
        if (d->pw_abort) break;
        clock_gettime(CLOCK_MONOTONIC, &t1);
        if ((double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec) > limit) break;
        sched_yield();
    }
    d->pw_pending = 1;
    d->pw_armed = 0;
    return 0;
}

void fdev_peer_wait_abort(ftar_dev *d) { d->pw_abort = 1; }

int fdev_peer_wait_verdict(ftar_dev *d)
{
    d->pw_pending = 0;
    if (!d->pw_armed) return 1;
    d->pw_armed = 0;
    return d->pw_go;
}

int fdev_run_bg(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    return fdev_run(d, dtype, op, segs, nseg, tag);
}

int fdev_sync_bg(ftar_dev *d, int (*poll)(void *), void *arg) { return poll ? poll(arg) : 0; }

int fdev_copy(ftar_dev *d, int bg, void *dst, const void *src, size_t bytes, int remote, int tag)
{
    if (d->gate_pending) fdev_gate_open(d, 1);
    memmove(dst, src, bytes);
    if (remote) d->ctr.link_bytes += (double)bytes;
    d->ctr.launches[tag]++;
    return 0;
}

int fdev_order_after(ftar_dev *d, void *s) { return 0; }
int fdev_user_host_waits(const ftar_dev *d) { return 0; }

int fdev_sync(ftar_dev *d, int (*poll)(void *), void *arg)
{
    if (poll) return poll(arg);
    return 0;
}

int fdev_busy(ftar_dev *d) { return 0; } /* host "kernels" complete at launch */
void fdev_fence_next_drain(ftar_dev *d) {}

/* FTAR_HOSTSIM_FAIL_COPY=<rank>:<h2d|d2h>:<k> (test-only): that rank's k-th copy (0-based,
 * counted over the process) in that direction fails, as a HIP copy error would */
static int copy_fails(const char *dir)
{
    static int nh2d, nd2h;
    int *n = dir[0] == 'h' ? &nh2d : &nd2h;
    int k = (*n)++;
    const char *e = getenv("FTAR_HOSTSIM_FAIL_COPY"), *me = getenv("FTAR_RANK");
    int r, want;
    char which[8];
    if (!e || !me || sscanf(e, "%d:%7[a-z0-9]:%d", &r, which, &want) != 3) return 0;
    if (r != atoi(me) || strcmp(which, dir) != 0 || k != want) return 0;
    snprintf(g_err, sizeof(g_err), "injected %s copy failure (copy %d)", dir, k);
    return 1;
}

int fdev_h2d(ftar_dev *d, void *dst, const void *src, size_t n)
{
    if (copy_fails("h2d")) return 101;
    memcpy(dst, src, n);
    return 0;
}
int fdev_h2d_async(ftar_dev *d, void *dst, const void *src, size_t n, int slot)
{
    if (copy_fails("h2d")) return 101;
    memcpy(dst, src, n);
    return 0;
}
int fdev_wait_h2d(ftar_dev *d, int slot, int (*poll)(void *), void *arg) { return poll ? poll(arg) : 0; }
int fdev_d2h_async(ftar_dev *d, void *dst, const void *src, size_t n)
{
    if (copy_fails("d2h")) return 101;
    memcpy(dst, src, n);
    return 0;
}
int fdev_sync_d2h(ftar_dev *d, int (*poll)(void *), void *arg) { return poll ? poll(arg) : 0; }
int fdev_d2h(ftar_dev *d, void *dst, const void *src, size_t n)
{
    if (copy_fails("d2h")) return 101;
    memcpy(dst, src, n);
    return 0;
}

void fdev_profiling(ftar_dev *d, int on) { d->profiling = on; }
void fdev_counters_reset(ftar_dev *d) { memset(&d->ctr, 0, sizeof(d->ctr)); }
void fdev_counters_get(ftar_dev *d, fdev_counters *out) { *out = d->ctr; }
int fdev_set_reduce_variant(int v) { return 0; }

int fdev_reduce_local(const void *in, void *inout, size_t n, int dtype, int op, void *stream)
{
    fdev_seg s = {FDEV_REDUCE, 0, inout, inout, in, n, NULL};
    ftar_dev d;
    memset(&d, 0, sizeof(d));
    return fdev_run(&d, dtype, op, &s, 1, 0);
}

int fdev_export_retries(const ftar_dev *d) { return 0; }

/* FTAR_TRACE is GPU instrumentation (cache release / acquire): nothing to log here */
int fdev_trace_open(ftar_dev *d, const char *path) { return 0; }
void fdev_trace_region(ftar_dev *d, const void *base, size_t bytes, int owner, const char *name) {}
void fdev_trace_unregion(ftar_dev *d, const void *base) {}
void fdev_trace_external_write(ftar_dev *d, const void *p, size_t bytes) {}
void fdev_trace_note(ftar_dev *d, const char *fmt, ...) {}
