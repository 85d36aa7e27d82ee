/*
 * ftar_oracle.h -- CPU restatement of the reference's fault-tolerant Allreduce.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product path (libftar.so) never links or calls it.
 *
 * It restates, as a deterministic global simulation of p ranks in one process:
 *   - MPI_Reduce_local (OpenMPI op semantics: inout = inout <op> in)
 *   - recursive_doubling + reduce_pow2 + errhandler    (src/rd/{recursive_doubling,util,errhandler}.c)
 *   - allreduce_rabenseifner + errhandler_reduce_scatter + errhandler_allgather
 *                                                      (src/raben/{rabenseifner,util,errhandler}.c)
 * with deterministic fault injection (ftar_kill, see include/ftar.h).
 *
 * Parity pinning: int32 SUM is pinned by the reference's own recorded checksums
 * (data/data_compare/{rd,raben,original_rd,original_raben}.csv, every row satisfies RESULT = ((NP(NP-1)/2)%17)*SIZE) and
 * by the recovery outcomes recorded in data/data_fault/log_single_{RD,Raben}.csv (see tests/golden/).
 * float32 SUM: parity unpinned against the reference (it never runs float); the oracle
 * fixes the reduction tree of the schedule, so the build must be bit-exact to it.
 * The reference could not be compiled or run here (permission denied in the survey,
 * SURVEY.md section 8c), so there is no oracle/_ref.
 */
#ifndef FTAR_ORACLE_H
#define FTAR_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/ftar.h"

#ifdef __cplusplus
extern "C" {
#endif

/* per-rank outcome */
#define FTAR_ORACLE_OK      0  /* survived, result valid */
#define FTAR_ORACLE_DEAD    1  /* killed by the injection */
#define FTAR_ORACLE_ABORTED 2  /* the job aborted (MPI_Abort) */

/* deviations from the reference that the oracle implements as "evident intent" */
#define FTAR_DEV_RD_MASTER_LOOP   0x1  /* rd/errhandler.c:100-111 never increments j (infinite loop) */
#define FTAR_DEV_RD_SHORT_SHRINK  0x2  /* rd/errhandler.c:186-216 picks fewer than p ranks (UB) -> abort */
#define FTAR_DEV_RD_FANOUT        0x4  /* more inactive than active ranks: reference hangs -> abort */
#define FTAR_DEV_RABEN_NO_RECOV   0x8  /* impersonator lacks its step-0 copy: reference computes garbage -> abort */
#define FTAR_DEV_RD_SINGLE        0x10 /* N=1: reference leaves dst uninitialised -> dst = src */

typedef struct {
    int status[FTAR_MAX_RANKS];     /* FTAR_ORACLE_* per original rank */
    int aborted;                    /* 1 if the job aborted */
    int abort_code;                 /* MPI_Abort error code */
    int recoveries;                 /* error-handler invocations that completed */
    int deviations;                 /* FTAR_DEV_* bits that were exercised */
    int ret;                        /* return value of the allreduce (FTAR_SUCCESS/ERR_*) */
    int size_after;                 /* comm size after the call */
    int order_after[FTAR_MAX_RANKS];/* comm rank -> original rank after the call */
} ftar_oracle_result;

size_t ftar_oracle_esize(int dtype);

/* MPI_Reduce_local(in, inout, n, dtype, op): inout[i] = inout[i] <op> in[i]. */
int ftar_oracle_reduce_local(int dtype, int op, const void *in, void *inout, size_t n);

/* The reference drivers' checksum: int res = sum_i (result[i] % 17), 32-bit wrap
 * (rd/recursive_doubling.c:139-144, raben/rabenseifner.c:420-424). */
int32_t ftar_oracle_checksum17(const int32_t *buf, size_t n);
/* Same on a float32 result whose values are integers (the float variant of the driver). */
int32_t ftar_oracle_checksum17_f32(const float *buf, size_t n);

/* Global simulations.  inputs[r] (count elements) is rank r's send buffer and is not
 * modified; outputs[r] receives rank r's result (left untouched for dead/aborted ranks
 * and when the call returns an error). */
int ftar_oracle_rabenseifner(int p, size_t count, int dtype, int op,
                             const void *const *inputs, void *const *outputs,
                             const ftar_kill *kills, int nkills, ftar_oracle_result *res);

int ftar_oracle_recursive_doubling(int p, size_t count, int dtype, int op,
                                   const void *const *inputs, void *const *outputs,
                                   const ftar_kill *kills, int nkills, ftar_oracle_result *res);

#ifdef __cplusplus
}
#endif
#endif
