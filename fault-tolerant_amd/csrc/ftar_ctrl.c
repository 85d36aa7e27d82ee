/*
 * ftar_ctrl.c -- shared-memory control plane (see ftar_ctrl.h).
 *
 * Restates the ULFM services used by the reference (MPIX_Comm_agree,
 * MPIX_Comm_failure_ack/get_acked, MPI_Barrier error return, MPI_Abort) for ranks
 * that are processes on one node, without MPI:
 *   - rd/recursive_doubling.c:51-53, raben/rabenseifner.c:258-260,330-332
 *     (agree + barrier after every step) -> ftar_ctrl_agree
 *   - rd/errhandler.c:21-40, raben/errhandler.c:15-31 (ack / get_acked / translate)
 *     -> the sealed failure snapshot returned by ftar_ctrl_agree
 *   - MPI_Abort (rd/util.c:75, raben/errhandler.c:38,211,322,378) -> ftar_ctrl_abort
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include "ftar_ctrl.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static inline void cpu_relax(void)
{
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}

static int map_segment(ftar_job *job, int fd)
{
    void *p = mmap(NULL, sizeof(ftar_shm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (p == MAP_FAILED) return FTAR_ERR_NOMEM;
    job->shm = (ftar_shm *)p;
    return FTAR_SUCCESS;
}

int ftar_ctrl_create(ftar_job *job, const char *name, int size)
{
    if (size < 1 || size > FTAR_MAX_RANKS) return FTAR_ERR_ARG;
    memset(job, 0, sizeof(*job));
    snprintf(job->name, sizeof(job->name), "%s", name);
    int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 && errno == EEXIST) { /* stale segment of a crashed job with the same name */
        shm_unlink(name);
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    }
    if (fd < 0) return FTAR_ERR_STATE;
    if (ftruncate(fd, (off_t)sizeof(ftar_shm)) != 0) {
        close(fd);
        return FTAR_ERR_NOMEM;
    }
    int rc = map_segment(job, fd);
    close(fd);
    if (rc) return rc;
    memset(job->shm, 0, sizeof(ftar_shm));
    job->shm->version = FTAR_SHM_VERSION;
    job->shm->abi_id = FTAR_ABI_ID;
    job->shm->size = size;
    for (int i = 0; i < FTAR_DECISIONS; i++) atomic_store(&job->shm->decision[i], FTAR_UNDECIDED);
    /* the magic last: a rank that reads it (ftar_ctrl_attach's header check) reads the
     * version and build written before it */
    __atomic_store_n(&job->shm->magic, FTAR_SHM_MAGIC, __ATOMIC_RELEASE);
    atomic_store_explicit(&job->shm->ready, 1, memory_order_release);
    job->size = size;
    job->rank = -1;
    job->owner = 1;
    return FTAR_SUCCESS;
}

int ftar_ctrl_attach(ftar_job *job, const char *name, int rank, int size, int create_if_rank0)
{
    if (rank < 0 || rank >= size || size > FTAR_MAX_RANKS) return FTAR_ERR_ARG;
    if (create_if_rank0 && rank == 0) {
        int rc = ftar_ctrl_create(job, name, size);
        if (rc) return rc;
        job->rank = 0;
        return FTAR_SUCCESS;
    }
    memset(job, 0, sizeof(*job));
    snprintf(job->name, sizeof(job->name), "%s", name);
    double t0 = now_s();
    for (;;) {
        int fd = shm_open(name, O_RDWR, 0600);
        if (fd >= 0) {
            struct stat st;
            /* the header (magic, version, build) is read before anything else: a launcher of
             * other headers is refused with one clear line, whatever its block's layout */
            struct {
                uint32_t magic, version;
                uint64_t abi_id;
            } hdr;
            if (pread(fd, &hdr, sizeof(hdr), 0) == (ssize_t)sizeof(hdr) && hdr.magic == FTAR_SHM_MAGIC &&
                (hdr.version != FTAR_SHM_VERSION || hdr.abi_id != FTAR_ABI_ID)) {
                fprintf(stderr, "ftar: rank %d: control block %s was created by build %016llx (layout %u), this "
                                "library is build %016llx (layout %u): launcher and library from different "
                                "builds -- rebuild both (make)\n",
                        rank, name, hdr.version == FTAR_SHM_VERSION ? (unsigned long long)hdr.abi_id : 0ull,
                        hdr.version, (unsigned long long)FTAR_ABI_ID, FTAR_SHM_VERSION);
                close(fd);
                return FTAR_ERR_STATE;
            }
            if (fstat(fd, &st) == 0 && st.st_size > 0 && (size_t)st.st_size != sizeof(ftar_shm)) {
                fprintf(stderr, "ftar: rank %d: control block %s has %lld bytes, this build expects %zu "
                                "(launcher and library from different builds?)\n",
                        rank, name, (long long)st.st_size, sizeof(ftar_shm));
                close(fd);
                return FTAR_ERR_STATE;
            }
            if (fstat(fd, &st) == 0 && (size_t)st.st_size == sizeof(ftar_shm)) {
                int rc = map_segment(job, fd);
                close(fd);
                if (rc) return rc;
                while (!atomic_load_explicit(&job->shm->ready, memory_order_acquire)) {
                    if (now_s() - t0 > 120.0) return FTAR_ERR_STATE;
                    usleep(1000);
                }
                break;
            }
            close(fd);
        }
        if (now_s() - t0 > 120.0) {
            fprintf(stderr, "ftar: rank %d: control block %s never appeared\n", rank, name);
            return FTAR_ERR_STATE;
        }
        usleep(1000);
    }
    if (job->shm->magic != FTAR_SHM_MAGIC || job->shm->size != size) return FTAR_ERR_STATE;
    job->rank = rank;
    job->size = size;
    return FTAR_SUCCESS;
}

int ftar_ctrl_join(ftar_job *job, int device, const char *phys)
{
    ftar_slot *s = &job->shm->slot[job->rank];
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
    pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
    if (pthread_mutex_init(&s->alive, &a) != 0) return FTAR_ERR_STATE;
    pthread_mutexattr_destroy(&a);
    if (pthread_mutex_lock(&s->alive) != 0) return FTAR_ERR_STATE;
    s->device = device;
    snprintf(s->phys, sizeof(s->phys), "%s", phys ? phys : "");
    atomic_store(&s->pid, (int)getpid());
    atomic_store(&s->arrive, 0);
    atomic_store_explicit(&s->state, FTAR_SLOT_RUNNING, memory_order_release);
    job->seq = 0;
    return FTAR_SUCCESS;
}

void ftar_ctrl_leave(ftar_job *job)
{
    if (!job->shm || job->rank < 0) return;
    ftar_slot *s = &job->shm->slot[job->rank];
    atomic_store_explicit(&s->state, FTAR_SLOT_FINALIZED, memory_order_release);
    pthread_mutex_unlock(&s->alive);
    atomic_fetch_add(&job->shm->nfinalized, 1);
}

void ftar_ctrl_detach(ftar_job *job)
{
    if (job->shm) munmap(job->shm, sizeof(ftar_shm));
    job->shm = NULL;
}

uint64_t ftar_ctrl_failed(ftar_job *job)
{
    return atomic_load_explicit(&job->shm->failed, memory_order_acquire);
}

static void mark_failed(ftar_job *job, int m)
{
    atomic_fetch_or_explicit(&job->shm->failed, 1ull << m, memory_order_acq_rel);
}

int ftar_ctrl_is_dead(ftar_job *job, int m)
{
    if (ftar_ctrl_failed(job) & (1ull << m)) return 1;
    ftar_slot *s = &job->shm->slot[m];
    if (atomic_load_explicit(&s->state, memory_order_acquire) != FTAR_SLOT_RUNNING) return 0;
    int r = pthread_mutex_trylock(&s->alive);
    if (r == EBUSY) return 0;
    if (r == EOWNERDEAD || r == ENOTRECOVERABLE) {
        mark_failed(job, m);
        if (r == EOWNERDEAD) pthread_mutex_unlock(&s->alive); /* leaves it not recoverable */
        return 1;
    }
    if (r == 0) {
        /* the owner released it: it finalized cleanly between our two reads */
        pthread_mutex_unlock(&s->alive);
        return 0;
    }
    int pid = atomic_load(&s->pid);
    if (pid > 0 && kill(pid, 0) != 0 && errno == ESRCH) {
        mark_failed(job, m);
        return 1;
    }
    return 0;
}

static void exit_aborted(ftar_job *job)
{
    int code = atomic_load(&job->shm->abort_code);
    fflush(stdout);
    _exit(code ? code : 1);
}

/* A member that called ftar_finalize never arrives again: waiting for it is a protocol
 * error (ranks ran different sequences of collectives), not a failure to recover from. */
static void check_finalized(ftar_job *job, int m, _Atomic uint64_t *field, uint64_t seq)
{
    if (atomic_load_explicit(&job->shm->slot[m].state, memory_order_acquire) != FTAR_SLOT_FINALIZED) return;
    /* it may have reached `seq` (and finalized) since the caller's read: re-read */
    if (atomic_load_explicit(field, memory_order_acquire) >= seq) return;
    fprintf(stderr, "ftar: rank %d: rank %d finalized before round %llu (protocol error)\n", job->rank, m,
            (unsigned long long)seq);
    ftar_ctrl_abort(job, FTAR_ERR_STATE);
}

int ftar_ctrl_poll(void *arg)
{
    ftar_job *job = (ftar_job *)arg;
    if (atomic_load_explicit(&job->shm->abort_flag, memory_order_acquire)) exit_aborted(job);
    return 0;
}

/* Every member other than self has arrived at `seq` or is dead? */
static int round_complete(ftar_job *job, uint64_t members, uint64_t seq, double t0)
{
    for (int m = 0; m < job->size; m++) {
        if (!(members & (1ull << m)) || m == job->rank) continue;
        ftar_slot *s = &job->shm->slot[m];
        if (atomic_load_explicit(&s->arrive, memory_order_acquire) >= seq) continue;
        if (ftar_ctrl_is_dead(job, m)) continue;
        check_finalized(job, m, &s->arrive, seq);
        if (atomic_load_explicit(&s->state, memory_order_acquire) == FTAR_SLOT_EMPTY && now_s() - t0 > 120.0) {
            fprintf(stderr, "ftar: rank %d never joined the job\n", m);
            ftar_ctrl_abort(job, FTAR_ERR_STATE);
        }
        return 0;
    }
    return 1;
}

uint64_t ftar_ctrl_agree(ftar_job *job, uint64_t members)
{
    ftar_shm *S = job->shm;
    uint64_t seq = ++job->seq;
    atomic_store_explicit(&S->slot[job->rank].arrive, seq, memory_order_release);
    unsigned idx = (unsigned)(seq % FTAR_DECISIONS);
    double t0 = now_s();
    for (unsigned long it = 0;; it++) {
        if (atomic_load_explicit(&S->abort_flag, memory_order_acquire)) exit_aborted(job);
        uint64_t w = atomic_load_explicit(&S->decision[idx], memory_order_acquire);
        if (w != FTAR_UNDECIDED) return w;
        if (round_complete(job, members, seq, t0)) {
            uint64_t snap = ftar_ctrl_failed(job) & members;
            uint64_t expect = FTAR_UNDECIDED;
            if (atomic_compare_exchange_strong_explicit(&S->decision[idx], &expect, snap,
                                                        memory_order_acq_rel, memory_order_acquire)) {
                /* every live member has read round seq-1 before arriving here: recycle it */
                atomic_store_explicit(&S->decision[(seq - 1) % FTAR_DECISIONS], FTAR_UNDECIDED, memory_order_release);
            }
            continue;
        }
        if (job->wait_hook && (it & 255) == 255 && now_s() - t0 > job->wait_after_s) {
            void (*h)(void *) = job->wait_hook;
            job->wait_hook = NULL; /* once per round */
            h(job->wait_arg);
        }
        cpu_relax();
    }
}

void ftar_ctrl_enter(ftar_job *job)
{
    job->xtok = job->seq + 1;
    atomic_store_explicit(&job->shm->slot[job->rank].entered, job->xtok, memory_order_release);
}

/* Wait until field `f` of rank m's slot reaches the current exchange token (1) or m is
 * dead without it (0).  The field is written before the writer can die past it: re-read
 * after the death test. */
static int wait_token(ftar_job *job, int m, size_t f)
{
    const uint64_t tok = job->xtok;
    _Atomic uint64_t *v = (_Atomic uint64_t *)((char *)&job->shm->slot[m] + f);
    for (;;) {
        if (atomic_load_explicit(v, memory_order_acquire) >= tok) return 1;
        if (ftar_ctrl_is_dead(job, m)) return atomic_load_explicit(v, memory_order_acquire) >= tok;
        check_finalized(job, m, v, tok);
        if (atomic_load_explicit(&job->shm->abort_flag, memory_order_acquire)) exit_aborted(job);
        cpu_relax();
    }
}

int ftar_ctrl_peer_entered(ftar_job *job, int m)
{
    job->xtok = job->seq + 1; /* the caller has entered this exchange itself */
    return wait_token(job, m, offsetof(ftar_slot, entered));
}

void ftar_ctrl_launched(ftar_job *job)
{
    atomic_store_explicit(&job->shm->slot[job->rank].launched, job->xtok, memory_order_release);
}

void ftar_ctrl_done(ftar_job *job)
{
    atomic_store_explicit(&job->shm->slot[job->rank].done, job->xtok, memory_order_release);
}

int ftar_ctrl_peer_done(ftar_job *job, int m) { return wait_token(job, m, offsetof(ftar_slot, done)); }

int ftar_ctrl_wait_peers_launched(ftar_job *job, uint64_t members)
{
    ftar_shm *S = job->shm;
    const uint64_t tok = job->xtok;
    atomic_store_explicit(&S->slot[job->rank].dying, tok, memory_order_release);
    for (;;) {
        int done = 1, launched = 0;
        for (int m = 0; m < job->size && done; m++) {
            if (m == job->rank || !(members & (1ull << m))) continue;
            ftar_slot *s = &S->slot[m];
            if (atomic_load_explicit(&s->launched, memory_order_acquire) >= tok) {
                launched++;
                continue;
            }
            if (atomic_load_explicit(&s->arrive, memory_order_acquire) >= tok) continue;
            if (ftar_ctrl_is_dead(job, m)) continue;
            done = 0;
        }
        if (done) return launched;
        if (atomic_load_explicit(&S->abort_flag, memory_order_acquire)) exit_aborted(job);
        cpu_relax();
    }
}

void ftar_ctrl_wait_peers_before_dying(ftar_job *job, uint64_t members, uint64_t seq)
{
    ftar_shm *S = job->shm;
    atomic_store_explicit(&S->slot[job->rank].dying, seq, memory_order_release);
    for (;;) {
        int done = 1;
        for (int m = 0; m < job->size && done; m++) {
            if (m == job->rank || !(members & (1ull << m))) continue;
            ftar_slot *s = &S->slot[m];
            if (atomic_load_explicit(&s->arrive, memory_order_acquire) >= seq) continue;
            if (atomic_load_explicit(&s->dying, memory_order_acquire) >= seq) continue;
            if (ftar_ctrl_is_dead(job, m)) continue;
            done = 0;
        }
        if (done) return;
        if (atomic_load_explicit(&S->abort_flag, memory_order_acquire)) exit_aborted(job);
        cpu_relax();
    }
}

void ftar_ctrl_wait_peers_arrived(ftar_job *job, uint64_t members, uint64_t seq)
{
    double t0 = now_s();
    while (!round_complete(job, members, seq, t0)) {
        if (atomic_load_explicit(&job->shm->abort_flag, memory_order_acquire)) exit_aborted(job);
        cpu_relax();
    }
}

void ftar_ctrl_abort(ftar_job *job, int code)
{
    ftar_shm *S = job->shm;
    int expect = 0;
    fflush(stdout);
    if (atomic_compare_exchange_strong(&S->abort_flag, &expect, 1)) {
        atomic_store(&S->abort_code, code);
        atomic_store(&S->abort_rank, job->rank);
        fprintf(stderr,
                "--------------------------------------------------------------------------\n"
                "MPI_ABORT was invoked on rank %d in communicator MPI_COMM_WORLD\n"
                "with errorcode %d.\n"
                "--------------------------------------------------------------------------\n",
                job->rank, code);
        fflush(stderr);
        /* like Open MPI's MPI_Abort: take every process of the job down */
        for (int m = 0; m < job->size; m++) {
            if (m == job->rank) continue;
            ftar_slot *s = &S->slot[m];
            int pid = atomic_load(&s->pid);
            if (pid > 0 && atomic_load(&s->state) == FTAR_SLOT_RUNNING) kill(pid, SIGKILL);
        }
    }
    _exit(code ? code : 1);
}
