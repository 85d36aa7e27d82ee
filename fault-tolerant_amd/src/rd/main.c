/*
 * src/rd/main -- drop-in for the reference's src/rd/main (rd/recursive_doubling.c:95-163).
 *
 *   ftrun -np N ./main <count>
 *
 * Same CLI and stdout lines as the reference (P:, Size:, Time:, Hello ... result is:),
 * buffer[i] = rank, MPI_INT + MPI_SUM; FTAR_DTYPE=float32 for float32.  The
 * Allreduce runs device-resident on the rank's MI355X between an H2D and a D2H copy;
 * Time: is the wall-clock seconds of that call plus the closing barrier.
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
    ftar_recursive_doubling_host(buffer, result, (size_t)buf_size, dt, FTAR_SUM, comm);
    ftar_barrier(comm);
    double t1 = now_s();
    uint32_t res = 0;
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
    ftar_finalize(comm);
    return 0;
}
