/*
 * src/raben/main -- drop-in for the reference's src/raben/main (raben/rabenseifner.c:397-460).
 *
 *   ftrun -np N ./main <count>
 *
 * Same CLI and the same four stdout lines per surviving rank, which
 * analysis/check_fault.py and check_compare.py parse:
 *   P: <N> / Size: <count> / Time: <seconds> /
 *   Hello from <rank> of <N> and the result is: <sum_i result[i] % 17>
 * Inputs are buffer[i] = rank, MPI_INT + MPI_SUM as in the reference; FTAR_DTYPE=float32
 * runs the same test on float32 (checksum unchanged).  The buffers start and end in
 * host memory like the reference's; the Allreduce itself is device-resident on the
 * rank's MI355X (H2D, ftar_allreduce_rabenseifner, D2H).  Time: is wall-clock seconds of
 * that end-to-end call plus the closing barrier (the reference prints clock() CPU time).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ftar.h"

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int test(int buf_size, int rank, int size, ftar_comm *comm, ftar_dtype dt)
{
    size_t es = (dt == FTAR_FLOAT32) ? sizeof(float) : sizeof(int);
    void *buffer = malloc((size_t)buf_size * es + 1);
    void *result = malloc((size_t)buf_size * es + 1);
    /* FTAR_FILL_OFFSET=k (default 0, the reference's input): buffer[i] = rank + k, so a one-rank
     * run has a nonzero checksum, ((N(N-1)/2 + N k) % 17) * count */
    const int fill = getenv("FTAR_FILL_OFFSET") ? atoi(getenv("FTAR_FILL_OFFSET")) : 0;
    for (int i = 0; i < buf_size; i++) {
        if (dt == FTAR_FLOAT32) ((float *)buffer)[i] = (float)(rank + fill);
        else ((int *)buffer)[i] = rank + fill;
    }
    double t0 = now_s();
    ftar_allreduce_rabenseifner_host(buffer, result, (size_t)buf_size, dt, FTAR_SUM, comm);
    ftar_barrier(comm);
    double t1 = now_s();
    uint32_t res = 0; /* int res with wrap-around, as the reference's */
    for (int i = 0; i < buf_size; i++) {
        int v = (dt == FTAR_FLOAT32) ? (int)((float *)result)[i] : ((int *)result)[i];
        res += (uint32_t)(v % 17);
    }
    printf("P: %d\n", size);
    printf("Size: %d\n", buf_size);
    printf("Time: %lf\n", t1 - t0);
    printf("Hello from %d of %d and the result is: %d\n", rank, size, (int)res);
    fflush(stdout);
    free(buffer);
    free(result);
    return 0;
}

int main(int argc, char *argv[])
{
    ftar_comm *comm;
    if (ftar_init(&comm) != FTAR_SUCCESS) {
        fprintf(stderr, "ftar_init failed\n");
        return EXIT_FAILURE;
    }
    int rank, size;
    ftar_world_rank(comm, &rank);
    ftar_world_size(comm, &size);
    if (argc < 2) {
        printf("Error: buffer size expected\n");
        return EXIT_FAILURE;
    }
    int buf_size = atoi(argv[1]);
    const char *dts = getenv("FTAR_DTYPE");
    ftar_dtype dt = (dts && !strcmp(dts, "float32")) ? FTAR_FLOAT32 : FTAR_INT32;
    test(buf_size, rank, size, comm, dt);
    ftar_finalize(comm);
    return 0;
}
