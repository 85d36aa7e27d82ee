/*
 * ftar_ctrl.h -- per-job shared-memory control plane (host C, no MPI, no HIP).
 *
 * Replaces the ULFM runtime services the reference relies on:
 *   failure detection   -> one process-shared robust mutex per rank, held for the
 *                          rank's lifetime; the kernel releases it with OWNER_DIED the
 *                          instant the process dies (kill -9 included), so a probe
 *                          (trylock) is an authoritative, immediate death test;
 *   MPIX_Comm_agree     -> ftar_ctrl_agree(): a round completes when every member has
 *   + MPI_Barrier          arrived or is dead; the first rank that sees completion seals
 *                          the round's failure snapshot with one CAS, so every survivor
 *                          returns the same set (uniform, unlike a bare ULFM barrier);
 *   MPI_Abort           -> abort flag + SIGKILL of every rank (and the launcher's reaper);
 *   exchange of IPC memory handles and per-step publications (RD's accumulator id).
 */
#ifndef FTAR_CTRL_H
#define FTAR_CTRL_H

#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <sys/types.h>

#include "../../include/ftar.h"
#include "ftar_dev.h"

#define FTAR_SHM_MAGIC 0x46544152u /* "FTAR" */
#define FTAR_SHM_VERSION 8
/* digest of the headers this binary was built from (fault-tolerant_amd/tools/build_id.sh abi,
 * passed by the Makefiles): the launcher writes it into the control block, every rank compares */
#ifndef FTAR_ABI_ID
#define FTAR_ABI_ID 0ull
#endif
#define FTAR_NBUF 4       /* exported workspace buffers per rank (IN, W, T, R) */
#define FTAR_DECISIONS 64 /* ring of agree decisions */

#define FTAR_INFLIGHT_LOCAL 1
#define FTAR_INFLIGHT_PULL 2

#define FTAR_SLOT_EMPTY 0
#define FTAR_SLOT_RUNNING 2
#define FTAR_SLOT_FINALIZED 3

/* an undecided ring entry: never a valid snapshot, which always omits the decider */
#define FTAR_UNDECIDED (~0ull)

typedef struct {
    pthread_mutex_t alive;          /* robust + pshared, locked by the owner while alive */
    _Atomic int state;              /* FTAR_SLOT_* */
    _Atomic int pid;
    int device;                     /* HIP ordinal in the rank's process (its visibility mask applies) */
    char phys[32];                  /* physical device identity (PCI bus id): ordinals of ranks with
                                       different HIP_VISIBLE_DEVICES masks can agree on different GPUs */
    _Atomic uint64_t arrive;        /* last agree sequence number this rank arrived at */
    _Atomic uint64_t ws_gen;        /* generation of the exported workspace */
    uint64_t ws_bytes;
    unsigned char handle[FTAR_NBUF][FDEV_HANDLE_BYTES];
    /* per-round publication (RD: which buffer holds the accumulator), double-buffered by
     * round parity: written before arriving at round s into pubv[s % 2] tagged s */
    _Atomic uint64_t pubv[2];
    /* the current call's send buffer, when the rank exports it instead of staging it in
     * IN (written before the call's first barrier) */
    unsigned char uhandle[FDEV_HANDLE_BYTES]; /* IPC handle of sbuf's allocation */
    uint64_t uid;                             /* its allocation id; 0 = peers read IN */
    uint64_t uoff;                            /* sbuf's byte offset in the allocation */
    uint64_t useq;                            /* the call (1, 2, ...) these fields belong to */
    uint64_t ufail;                           /* call in which this rank failed to map a peer's */
    uint64_t unew;                            /* 1: uid entered the peers' mapping caches with this
                                                 publication (they map it now), 0: they hold it */
    /* exchange entry: set to seq + 1 when the rank passes an exchange step's BEFORE
     * point (the agree sequence number is uniform at every step), so a partner decides
     * "the exchange failed" only for a rank that died before entering it */
    _Atomic uint64_t entered;
    /* the same token once the rank has launched its pulls of the step (or has none), and
     * once its exchange has completed (its pulls drained: the reference's Sendrecv returned) */
    _Atomic uint64_t launched;
    _Atomic uint64_t done;
    /* BARRIER kill point (tests): reached round `dying`'s barrier and will die there */
    _Atomic uint64_t dying;
    /* what this rank's stream runs right now: 0 nothing, FTAR_INFLIGHT_LOCAL a kernel on
     * its own memory, FTAR_INFLIGHT_PULL a kernel reading peers' HBM (an exchange).  Set at
     * launch, cleared when the stream drained; read post mortem by the launcher (ftrun)
     * to say whether a killed rank died mid-exchange. */
    _Atomic int inflight;
    char pad[64];
} ftar_slot;

typedef struct {
    uint32_t magic;
    uint32_t version;
    uint64_t abi_id;                /* FTAR_ABI_ID of the binary that created the block */
    int size;
    _Atomic int ready;
    _Atomic uint64_t failed;        /* one bit per original rank, monotone */
    _Atomic int abort_flag;
    _Atomic int abort_code;
    _Atomic int abort_rank;
    _Atomic int nfinalized;
    _Atomic int launcher_pid;       /* ftrun pid when launched by it, else 0 */
    _Atomic uint64_t decision[FTAR_DECISIONS];
    ftar_slot slot[FTAR_MAX_RANKS];
    /* the mesh's device-wait flags (fdev_peer_wait), one 64-byte line per original rank, in a
     * page of their own: every rank's GPU maps the page (hipHostRegister), its wait kernel
     * stores its token into its own line and polls its peers' over PCIe.  Host memory is
     * the one place every GPU of the node reads coherently while the writer's kernel runs;
     * a flag in the writer's HBM could be served stale from the reader's L2. */
    _Alignas(4096) _Atomic uint64_t pwflag[FTAR_MAX_RANKS][8];
} ftar_shm;

typedef struct {
    ftar_shm *shm;
    char name[128];
    int rank;     /* original rank = slot index */
    int size;
    uint64_t seq; /* agree sequence number */
    uint64_t xtok; /* exchange token of the step this rank last entered (seq + 1 at entry) */
    int owner;    /* created the segment */
    /* optional: called once by ftar_ctrl_agree when a round has waited longer than
     * wait_after_s (the library gives up a launch queued behind a gate there) */
    void (*wait_hook)(void *);
    void *wait_arg;
    double wait_after_s;
} ftar_job;

/* Create (launcher / rank 0) or attach (others) the segment named `name`. */
int ftar_ctrl_create(ftar_job *job, const char *name, int size);
int ftar_ctrl_attach(ftar_job *job, const char *name, int rank, int size, int create_if_rank0);
/* Claim this rank's slot: robust mutex locked, pid, device (ordinal + physical id), state RUNNING. */
int ftar_ctrl_join(ftar_job *job, int device, const char *phys);
void ftar_ctrl_leave(ftar_job *job);
void ftar_ctrl_detach(ftar_job *job);

/* Is original rank m dead?  (failed bit, else robust-mutex probe; marks the bit) */
int ftar_ctrl_is_dead(ftar_job *job, int m);
uint64_t ftar_ctrl_failed(ftar_job *job);

/* Agree round over `members` (bit mask of original ranks, must contain self).
 * Returns the sealed failure snapshot (subset of members).  Never returns on abort. */
uint64_t ftar_ctrl_agree(ftar_job *job, uint64_t members);
/* This rank enters the exchange that precedes round seq + 1. */
void ftar_ctrl_enter(ftar_job *job);
/* Wait until original rank m entered the exchange this rank is in (1) or died before
 * entering it (0).  Never returns on abort. */
int ftar_ctrl_peer_entered(ftar_job *job, int m);
/* This rank has launched its pulls of the exchange it entered (or has none to launch). */
void ftar_ctrl_launched(ftar_job *job);
/* This rank's exchange has completed (its pulls drained). */
void ftar_ctrl_done(ftar_job *job);
/* Wait until original rank m completed the exchange this rank is in (1) or died before
 * completing it (0): the reference's Sendrecv with m failed iff 0. */
int ftar_ctrl_peer_done(ftar_job *job, int m);
/* DURING kill point: block until every other member has launched its pulls of the
 * current exchange, arrived at a later round, or is dead.  Returns how many members had
 * launched (peers that may be reading this rank's HBM). */
int ftar_ctrl_wait_peers_launched(ftar_job *job, uint64_t members);
/* BARRIER kill point: mark this rank as dying at round seq, then block until every
 * other member arrived at round seq, is dead, or is dying at the same round (two victims
 * of one step must not wait for each other). */
void ftar_ctrl_wait_peers_before_dying(ftar_job *job, uint64_t members, uint64_t seq);
/* Block until every member other than self arrived at round `seq` or is dead. */
void ftar_ctrl_wait_peers_arrived(ftar_job *job, uint64_t members, uint64_t seq);

/* MPI_Abort: flag the job, print the OpenMPI-style line on stderr, kill all ranks. */
void ftar_ctrl_abort(ftar_job *job, int code) __attribute__((noreturn));
/* Nonzero if the job is aborting (the caller then exits). */
int ftar_ctrl_poll(void *job);

#endif
