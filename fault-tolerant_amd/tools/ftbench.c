/*
 * ftbench -- one rank of a timed, device-resident Allreduce job under ftrun: the C5 leg
 * of bench.py (BASELINE configs[4]: Rabenseifner, 256 MiB float32 SUM, 9 ranks = 8 GPUs +
 * one idle spare, a single kill mid-exchange, ULFM-style shrink + recovery).
 *
 *   ftrun -np N --devmap d0,d1,... ftbench <raben|rd> <count> <calls>
 *
 * Every rank hipMallocs float32 send / receive vectors of `count` elements on its device,
 * fills the send vector with its original rank (the reference drivers' input,
 * rd/recursive_doubling.c:112-115 / raben/rabenseifner.c:408-411, as float32: every
 * partial sum is an exact integer, so the result is independent of the reduction tree)
 * and runs `calls` Allreduces through the C ABI.  FTAR_KILL (with a call index, e.g.
 * "6:1:1:3:1") injects the fault.  Per call it records the library's wall time
 * (ftar_last_stats), the recoveries, the comm size after the call, and the result read
 * back after the timed region: its first element and whether every element equals it.
 * One JSON line per surviving rank on stdout.  The reference's own numbers for this case
 * are data/data_fault/log_single_Raben.csv (N = 9, clock() seconds per run).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "ftar.h"

#define MAX_CALLS 16

#define CHECK_HIP(x)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "ftbench: %s: %s\n", #x, hipGetErrorString(e_));                       \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: ftbench <raben|rd> <count> <calls>\n");
        return 2;
    }
    int rd = !strcmp(argv[1], "rd");
    size_t count = strtoull(argv[2], NULL, 10);
    int calls = atoi(argv[3]);
    if (count == 0 || calls < 1 || calls > MAX_CALLS) return 2;

    ftar_comm *comm;
    if (ftar_init(&comm) != FTAR_SUCCESS) return 3;
    int wrank, wsize, dev;
    ftar_world_rank(comm, &wrank);
    ftar_world_size(comm, &wsize);
    ftar_comm_device(comm, &dev);
    CHECK_HIP(hipSetDevice(dev));

    /* FTBENCH_PATTERN=1: x_r[i] = (7 i + 13 r) mod 4096 instead of r, so every element
     * has its own exact sum (all partial sums are integers < 2^24) and a misplaced
     * window or a 32-bit index wrap shows as a wrong element (the size tests beyond
     * 2^31 elements); "uniform" then means "every element equals its exact sum". */
    const char *pe = getenv("FTBENCH_PATTERN");
    const int pattern = pe && atoi(pe) != 0;
    float *h = malloc(count * sizeof(float));
    if (!h) return 4;
    for (size_t i = 0; i < count; i++) h[i] = pattern ? (float)((7 * i + 13 * (size_t)wrank) % 4096) : (float)wrank;
    float *s = NULL, *r = NULL;
    CHECK_HIP(hipMalloc((void **)&s, count * sizeof(float)));
    CHECK_HIP(hipMalloc((void **)&r, count * sizeof(float)));
    CHECK_HIP(hipMemcpy(s, h, count * sizeof(float), hipMemcpyHostToDevice));
    CHECK_HIP(hipDeviceSynchronize());

    double ms[MAX_CALLS], value[MAX_CALLS], hbm[MAX_CALLS];
    int rc[MAX_CALLS], rec[MAX_CALLS], size_after[MAX_CALLS], uniform[MAX_CALLS], step0_copy = 0;
    for (int c = 0; c < calls; c++) {
        rc[c] = rd ? ftar_recursive_doubling(s, r, count, FTAR_FLOAT32, FTAR_SUM, comm)
                   : ftar_allreduce_rabenseifner(s, r, count, FTAR_FLOAT32, FTAR_SUM, comm);
        ftar_stats st;
        ftar_last_stats(comm, &st);
        ms[c] = st.wall_s * 1e3;
        hbm[c] = st.hbm_bytes; /* algorithmic local HBM bytes of this rank's kernels */
        rec[c] = st.recoveries;
        size_after[c] = st.comm_size_after;
        step0_copy |= st.step0_copy;
        /* outside the call's timed region: read the result back and check it is uniform */
        CHECK_HIP(hipMemcpy(h, r, count * sizeof(float), hipMemcpyDeviceToHost));
        value[c] = h[0];
        uniform[c] = 1;
        const int members = size_after[c]; /* the original ranks 0 .. members-1 (no fault) */
        for (size_t i = 0; i < count; i++) {
            float want = h[0];
            if (pattern) {
                size_t sum = 0;
                for (int q = 0; q < members; q++) sum += (7 * i + 13 * (size_t)q) % 4096;
                want = (float)sum;
            }
            if (h[i] != want) {
                uniform[c] = 0;
                break;
            }
        }
    }
    printf("{\"rank\": %d, \"size\": %d, \"device\": %d, \"step0_copy\": %d, \"calls\": [", wrank, wsize, dev,
           step0_copy);
    for (int c = 0; c < calls; c++)
        printf("%s{\"rc\": %d, \"ms\": %.4f, \"recoveries\": %d, \"comm_size\": %d, \"value\": %.1f, \"uniform\": %s, "
               "\"hbm_bytes\": %.0f}",
               c ? ", " : "", rc[c], ms[c], rec[c], size_after[c], value[c], uniform[c] ? "true" : "false", hbm[c]);
    printf("]}\n");
    fflush(stdout);
    ftar_finalize(comm);
    (void)hipFree(s);
    (void)hipFree(r);
    free(h);
    return 0;
}
