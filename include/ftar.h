/*
 * ftar.h -- C ABI of the MI355X-native fault-tolerant Allreduce (libftar.so).
 *
 * This is the drop-in boundary for the hot path of LucaMica02/Fault-Tolerant:
 * the two fault-tolerant Allreduce schedules (recursive doubling, Rabenseifner)
 * and the local reduction they call after every exchange.  Every entry point is
 * plain C: pointers, sizes and enums, no HIP or torch types in the signatures.
 * Device buffers are passed as `void *` (hipMalloc'd or torch tensor storage).
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   ftar_recursive_doubling      <- recursive_doubling()        src/rd/header.h:29
 *   ftar_allreduce_rabenseifner  <- allreduce_rabenseifner()    src/raben/header.h:14-15
 *   ftar_reduce_local            <- MPI_Reduce_local(in, inout) call sites
 *                                   src/rd/util.c:32, src/rd/recursive_doubling.c:44,48,
 *                                   src/raben/rabenseifner.c:86,117,234-236
 *   ftar_init / ftar_finalize    <- MPI_Init + MPI_Comm_dup(MPI_COMM_WORLD)
 *                                   src/raben/rabenseifner.c:441-454, src/rd/recursive_doubling.c:100
 *   ftar_abort                   <- MPI_Abort   (src/rd/util.c:75, src/raben/errhandler.c:38,211)
 *   ftar_barrier                 <- MPI_Barrier (src/rd/recursive_doubling.c:134)
 *   ULFM MPIX_Comm_agree / failure_ack / failure_get_acked / shrink and the
 *   group re-ordering in the error handlers are internal to the library
 *   (src/rd/errhandler.c, src/raben/errhandler.c); they surface only as the
 *   comm being re-targeted (rank/size queries change) after a recovery.
 */
#ifndef FTAR_H
#define FTAR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes: the MPI error classes the reference relies on ---------- */
#define FTAR_SUCCESS         0   /* MPI_SUCCESS */
#define FTAR_ERR_OP          9   /* MPI_ERR_OP: a bitwise / logical op on a floating-point type */
#define FTAR_ERR_ARG         13  /* MPI_ERR_ARG      (raben/rabenseifner.c:18-20) */
#define FTAR_ERR_UNKNOWN     14  /* MPI_ERR_UNKNOWN  (raben/util.c:40-43) */
#define FTAR_ERR_OTHER       16  /* MPI_ERR_OTHER    (rd/util.c:75) */
#define FTAR_ERR_PROC_FAILED 75  /* MPIX_ERR_PROC_FAILED, hard-coded 75 in rd/recursive_doubling.c:56 */
#define FTAR_ERR_DEVICE      101 /* a HIP call failed */
#define FTAR_ERR_NOMEM       102 /* allocation failed */
#define FTAR_ERR_STATE       103 /* library not initialised / job aborted */

/* ---- element types and reduction ops ------------------------------------- */
typedef enum {
    FTAR_INT32 = 0,   /* MPI_INT (the only type the reference drivers use) */
    FTAR_FLOAT32 = 1, /* north-star type */
    FTAR_INT64 = 2,
    FTAR_FLOAT64 = 3
} ftar_dtype;

/* MPI's predefined reduction ops (MAXLOC / MINLOC need pair types and are not offered).
 * The reference passes its MPI_Op straight to MPI_Reduce_local (raben/rabenseifner.c:
 * 86-87,117,234-236; rd/util.c:32; rd/recursive_doubling.c:44,48), so every op MPI
 * defines for these types is valid there.  As in MPI, the logical and bitwise ops are
 * defined for the integer types only (FTAR_ERR_OP for a float type); the logical ones
 * yield 0 or 1. */
typedef enum {
    FTAR_SUM = 0,  /* MPI_SUM (the only op the reference drivers use) */
    FTAR_PROD = 1,
    FTAR_MAX = 2,
    FTAR_MIN = 3,
    FTAR_LAND = 4, /* MPI_LAND: (a != 0) && (b != 0) */
    FTAR_BAND = 5, /* MPI_BAND: a & b */
    FTAR_LOR = 6,  /* MPI_LOR */
    FTAR_BOR = 7,  /* MPI_BOR */
    FTAR_LXOR = 8, /* MPI_LXOR: (a != 0) != (b != 0) */
    FTAR_BXOR = 9  /* MPI_BXOR */
} ftar_op;
#define FTAR_NOPS 10

/* ---- deterministic fault injection --------------------------------------
 * A kill names the victim (original world rank) and the place in the schedule
 * where it dies.  Phases follow the reference's control flow:
 *   FTAR_PH_PRE   RD reduce_pow2 (rd/util.c:3-34) / Raben pre-step (raben/rabenseifner.c:65-139)
 *   FTAR_PH_LOOP  RD distance loop (rd/recursive_doubling.c:21-71) / Raben reduce-scatter
 *                 loop (raben/rabenseifner.c:170-284); `step` = loop iteration (reference `step`)
 *   FTAR_PH_AG    Raben allgather loop (raben/rabenseifner.c:299-355); `step` = the reference's
 *                 `step` variable, i.e. steps-1 for the first allgather exchange
 *   FTAR_PH_POST  after the fault-tolerant region (ERRORS_ARE_FATAL barrier, fan-out / post-step)
 * Points inside a step:
 *   FTAR_PT_BEFORE   dies before its exchange of that step (partner's receive fails)
 *   FTAR_PT_AFTER    exchange done, dies before its local reduce / before arriving at the barrier
 *   FTAR_PT_BARRIER  completes the step, waits until every peer arrived, then dies (no peer ever
 *                    touches its memory while it dies)
 *   FTAR_PT_DURING   mid-exchange: has entered the step and launched its own pull kernel, waits
 *                    until every peer has launched its pulls of the step (some read this rank's
 *                    HBM), then dies with its kernel in flight.  Like a Sendrecv that fails
 *                    mid-transfer in the reference (raben/rabenseifner.c:209-211, 238-241), the
 *                    partner's exchange of that step counts as failed (`corr`): the window it
 *                    pulled is discarded and rebuilt by the error handler.
 */
#define FTAR_PH_PRE  0
#define FTAR_PH_LOOP 1
#define FTAR_PH_AG   2
#define FTAR_PH_POST 3

#define FTAR_PT_BEFORE  0
#define FTAR_PT_AFTER   1
#define FTAR_PT_BARRIER 2
#define FTAR_PT_DURING  3

typedef struct {
    int rank;  /* original world rank of the victim */
    int phase; /* FTAR_PH_* */
    int step;  /* step inside the phase */
    int point; /* FTAR_PT_* */
} ftar_kill;

#define FTAR_MAX_RANKS 64 /* failure sets are one 64-bit word, one bit per original rank */
#define FTAR_MAX_KILLS 16

/* ---- communicator -------------------------------------------------------- */
typedef struct ftar_comm ftar_comm;

/* Bootstrap from the environment: FTAR_JOB/FTAR_RANK/FTAR_SIZE/FTAR_DEVICE (set by
 * the `ftrun` launcher) or torchrun's RANK/WORLD_SIZE/LOCAL_RANK/MASTER_PORT.  Also
 * reads FTAR_KILL="rank:phase:step:point[,...]" for deterministic fault injection. */
int ftar_init(ftar_comm **comm);
/* Explicit bootstrap: `job` names the shared control block (all ranks pass the same),
 * `device` is the HIP device ordinal this rank drives. */
int ftar_init_rank(ftar_comm **comm, const char *job, int rank, int size, int device);
int ftar_finalize(ftar_comm *comm);

int ftar_comm_rank(const ftar_comm *comm, int *rank);       /* rank in the current (maybe shrunk) comm */
int ftar_comm_size(const ftar_comm *comm, int *size);       /* size of the current comm */
int ftar_world_rank(const ftar_comm *comm, int *rank);      /* original rank (Data.original_rank) */
int ftar_world_size(const ftar_comm *comm, int *size);      /* original size (Data.original_size) */
int ftar_comm_device(const ftar_comm *comm, int *device);   /* HIP device ordinal */

int ftar_barrier(ftar_comm *comm);                 /* ERRORS_ARE_FATAL barrier over the survivors */
void ftar_abort(ftar_comm *comm, int errorcode);   /* MPI_Abort: kills the whole job, never returns */

/* Deterministic fault injection (in addition to FTAR_KILL). */
int ftar_set_kills(ftar_comm *comm, const ftar_kill *kills, int nkills);

/* ---- the hot path ---------------------------------------------------------
 * Device-resident, blocking (return when the result is in the output buffer).
 * `stream` ordering: the call first waits for all work queued on the stream set
 * with ftar_comm_set_stream (default: the null stream) to finish.
 * Buffers must be device-accessible for count elements: memory of the comm's GPU,
 * managed memory, or pinned host memory mapped at its own address (hipHostMalloc, a
 * pinned torch tensor), which this rank's kernels read and write in place over PCIe.
 * Pageable host memory, another GPU's memory, or a range running past the end of its
 * allocation returns FTAR_ERR_ARG before anything is launched (the _host entry points
 * take any host buffer).
 */

/* Fault-tolerant Rabenseifner Allreduce (raben/rabenseifner.c:3-395).
 * sbuf is never written (the reference writes through its const sbuf; the build stages
 * what peers read in its own exported buffer); sbuf == rbuf (in place) is allowed.
 * On recovery the comm is re-targeted in place:
 * ftar_comm_rank/size change exactly as the reference's *comm replacement does. */
int ftar_allreduce_rabenseifner(const void *sbuf, void *rbuf, size_t count,
                                ftar_dtype dtype, ftar_op op, ftar_comm *comm);

/* Fault-tolerant recursive doubling (rd/recursive_doubling.c:6-90).  The reference
 * clobbers src as its accumulator; the build leaves src untouched.  The Data struct of
 * the reference (rd/header.h:16-26) lives inside the comm. */
int ftar_recursive_doubling(const void *src, void *dst, size_t count,
                            ftar_dtype dtype, ftar_op op, ftar_comm *comm);

/* Same schedules on host buffers: pinned H2D, device-resident allreduce, D2H. */
int ftar_allreduce_rabenseifner_host(const void *sbuf, void *rbuf, size_t count,
                                     ftar_dtype dtype, ftar_op op, ftar_comm *comm);
int ftar_recursive_doubling_host(const void *src, void *dst, size_t count,
                                 ftar_dtype dtype, ftar_op op, ftar_comm *comm);

/* MPI_Reduce_local(in, inout, count, dtype, op) on the device:
 * inout[i] = in[i] (op) inout[i] with the reference's operand roles.
 * `stream` is a hipStream_t (NULL = null stream); the call is asynchronous.
 * Each operand is memory of the current device or pinned host memory (hipHostMalloc /
 * hipHostRegister): the reference reduces host buffers, and on pinned ones the kernel
 * reads and writes them in place over PCIe (zero copy, both link directions at once).
 * Pageable or unknown memory, or a range past its allocation: FTAR_ERR_ARG, nothing
 * launched. */
int ftar_reduce_local(const void *in, void *inout, size_t count,
                      ftar_dtype dtype, ftar_op op, void *stream);

/* Which implementation of the local-reduce kernel ftar_reduce_local launches:
 * 0 = register-streaming float4 kernel, 1 = LDS-DMA staged kernel (default). */
int ftar_set_reduce_variant(int variant);

/* Stream the comm orders its work after (hipStream_t, NULL = null stream). */
int ftar_comm_set_stream(ftar_comm *comm, void *stream);

/* Transport options (defaults come from the FTAR_* environment at init).  Collective:
 * every live rank of the comm must set the same value before its next call. */
typedef enum {
    FTAR_OPT_OVERLAP = 0,      /* Raben step-0 redundancy copy on a background stream (0/1) */
    FTAR_OPT_RELAY = 1,        /* stripe exchanges over 2-hop relay paths (0/1) */
    FTAR_OPT_RELAY_MIN = 2,    /* smallest window, in bytes, that is relayed */
    FTAR_OPT_LOOP_SECONDS = 3, /* stretch of the step loop for fault-injection runs */
    FTAR_OPT_COPY_ENGINE = 4,  /* direct pulls as hipMemcpyAsync copies + local reduce (0/1) */
    FTAR_OPT_REDUNDANCY = 5,   /* Raben step-0 recovery copy (the reference's tmp, raben/rabenseifner.c:
                                  206-211): 2 = auto (default): moved when a spare exists and the comm
                                  spans more than one GPU, else a replay reads the dead rank's input
                                  in place; 1 = always moved (the reference's shape, also at
                                  power-of-two p); 0 = never moved (opt-in: the replay reads the dead
                                  rank's input through its peer mapping on any layout) */
    FTAR_OPT_MESH = 6,         /* Raben at power-of-two p without a spare: one-hop reduce-scatter and
                                  allgather over the full mesh, same reduction tree (0/1) */
    FTAR_OPT_ONESHOT_MAX = 7,  /* mesh Raben up to this many bytes per vector (any size at p = 2): one
                                  launch computes every block in its owner's tree into rbuf (0 = off) */
    FTAR_OPT_PUSH = 8,         /* mesh Raben by remote stores: 1 = reduce-scatter (every rank writes its part
                                  of each block into the owner's HBM, the owner reduces locally), 2 = both
                                  phases (the owner's tree also stores its block into every peer; p <= 8),
                                  0 = remote loads (default) */
    FTAR_OPT_GATE = 9,         /* queue small exchange launches (Raben one-shot, RD steps) ahead of the
                                  barrier that readies their operands, the staging copy folded into the
                                  first, their workgroups waiting on a gate the barrier opens (0/1,
                                  default 1): the launch latency overlaps the wait for the peers.  A
                                  barrier that waits longer than FTAR_GATE_HOLD_US (default 2000 us)
                                  gives the gated launch up and the step launches after it; a gate the
                                  device gave up on (FTAR_GATE_TIMEOUT_MS, default 60000) is relaunched
                                  ungated at the next drain */
    FTAR_OPT_FLAG_SYNC = 10,   /* short launches (<= 64 workgroups) signal their own completion through
                                  a pinned host word instead of a fenced marker drain (0/1, default 1;
                                  0 also turns the gates off) */
    FTAR_OPT_TREE_UNROLL = 11, /* 16-byte vectors per lane and source in the mesh's tree kernel at
                                  p = 4, 8 (1, 2 or 4; default 1): more loads in flight per lane for
                                  remote (xGMI) sources; same bits */
    FTAR_OPT_GATE_MAX = 12,    /* largest vector, in bytes, whose predictable launches are queued ahead
                                  behind gates (default 1 MiB).  Above 1 MiB (mid-size: RD steps 1..,
                                  the mesh's allgather) the gate is relayed through device memory and
                                  the launch waits on up to half the CUs -- slower on a GPU shared by
                                  several ranks, so bench.py times it on the node */
    FTAR_OPT_MESH_WAIT = 13    /* the mesh's allgather queued right behind its reduce-scatter, ordered on
                                  the device: each rank publishes a flag in its HBM once its tree is
                                  released, and the allgather waits for the peers' flags instead of a
                                  host agree round and a drain (0/1, default 1) */
} ftar_option;

int ftar_comm_set_option(ftar_comm *comm, ftar_option opt, double value);
int ftar_comm_get_option(const ftar_comm *comm, ftar_option opt, double *value);

/* ---- statistics of the last allreduce call on this rank ----------------- */
typedef struct {
    int    steps;            /* exchange steps executed (pre/loop/allgather/post) */
    int    recoveries;       /* error-handler invocations that recovered */
    int    comm_size_after;  /* comm size after the call */
    double wall_s;           /* host wall time of the call */
    double kernel_ms;        /* sum of device time of all kernels of the call (profiling on) */
    double step0_kernel_ms;  /* device time of the dominant kernel (RD step / Raben step 0) */
    double link_bytes;       /* bytes this rank pulled over the fabric (algorithmic) */
    double hbm_bytes;        /* algorithmic HBM bytes of this rank's kernels */
    int    kernels;          /* kernels launched */
    double step0_link_bytes; /* fabric bytes the dominant kernel pulls per call */
    double bg_kernel_ms;     /* device time of background-stream kernels (Raben redundancy copy) */
    double sync_wait_s;      /* host time spent in agree/barrier rounds */
    double drain_s;          /* host time spent waiting for the device stream */
    int    syncs;            /* agree/barrier rounds */
    int    relayed_steps;    /* exchange steps striped over 2-hop relays */
    int    mesh_steps;       /* one-hop mesh exchanges (Raben reduce-scatter / allgather) */
    int    export_retries;   /* workspace blocks the runtime refused to export (IPC) and that were
                                re-allocated, cumulative since ftar_init (expected: 0) */
    int    gated_launches;   /* launches queued ahead of their barrier (FTAR_OPT_GATE) */
    int    gated_skips;      /* ... of them replaced after the barrier (a peer's input moved) */
    int    user_stream_waits; /* calls that found the caller's stream busy and waited for it on the host,
                                 cumulative since ftar_init */
    int    step0_copy;       /* Raben: this call moved the step-0 recovery copy (FTAR_OPT_REDUNDANCY) */
    int    gate_holds;       /* gated launches given up because their barrier waited past FTAR_GATE_HOLD_US */
    int    gate_relaunches;  /* gated launches the device gave up on (gate timeout), relaunched ungated;
                                cumulative since ftar_init */
    int    peer_waits;       /* mesh allgathers ordered behind the peers' trees on the device (FTAR_OPT_MESH_WAIT) */
    int    peer_wait_skips;  /* ... of them given up (a peer died, or the wait timed out) and settled by an agree */
} ftar_stats;

int ftar_last_stats(const ftar_comm *comm, ftar_stats *out);
/* Record hipEvents around every kernel of the schedules (for bench.py's roofline). */
int ftar_set_profiling(ftar_comm *comm, int on);

/* Version string of the library build. */
const char *ftar_version(void);
/* Identity of this build: "ftar-build abi=<16 hex> src=<16 hex>" -- the digest of the
 * headers every binary of a job shares (a launcher of other headers is refused when a rank
 * attaches) and of every product source the library was linked from. */
const char *ftar_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* FTAR_H */
