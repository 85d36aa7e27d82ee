/*
 * ftar_probe.c -- TEST driver: one rank of a parity run.
 *
 * Launched by ftrun; reads its input vector from $FTAR_PROBE_DIR/in_<rank>.bin, runs
 * the selected schedule through the C ABI (host-buffer entry points, so the
 * device-resident path runs inside), and writes $FTAR_PROBE_DIR/out_<rank>_<iter>.bin
 * plus a status line.  Built twice: against libftar.so (GPU parity tests) and against
 * the host-sim library (CPU tests of the host logic).
 *
 * env: FTAR_PROBE_DIR, FTAR_PROBE_ALGO=rd|raben, FTAR_PROBE_DTYPE=0..3,
 *      FTAR_PROBE_OP=0..3, FTAR_PROBE_COUNT, FTAR_PROBE_ITERS (default 1),
 *      FTAR_PROBE_DEVICE=1 (device-pointer entry points instead of the host ones)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ftar.h"

static size_t esize(int dt) { return (dt == 0 || dt == 1) ? 4 : 8; }

int main(void)
{
    const char *dir = getenv("FTAR_PROBE_DIR");
    const char *algo = getenv("FTAR_PROBE_ALGO");
    if (!dir || !algo) return 2;
    int dt = getenv("FTAR_PROBE_DTYPE") ? atoi(getenv("FTAR_PROBE_DTYPE")) : 0;
    int op = getenv("FTAR_PROBE_OP") ? atoi(getenv("FTAR_PROBE_OP")) : 0;
    size_t count = getenv("FTAR_PROBE_COUNT") ? strtoull(getenv("FTAR_PROBE_COUNT"), NULL, 10) : 0;
    int iters = getenv("FTAR_PROBE_ITERS") ? atoi(getenv("FTAR_PROBE_ITERS")) : 1;

    ftar_comm *comm;
    if (ftar_init(&comm) != FTAR_SUCCESS) return 3;
    int rank;
    ftar_world_rank(comm, &rank);
    size_t bytes = count * esize(dt);
    void *in = malloc(bytes + 16), *out = malloc(bytes + 16);
    char path[512];
    snprintf(path, sizeof(path), "%s/in_%d.bin", dir, rank);
    FILE *f = fopen(path, "rb");
    if (!f || fread(in, 1, bytes, f) != bytes) return 4;
    fclose(f);
    for (int it = 0; it < iters; it++) {
        memset(out, 0xEE, bytes);
        int rc = !strcmp(algo, "rd") ? ftar_recursive_doubling_host(in, out, count, (ftar_dtype)dt, (ftar_op)op, comm)
                                     : ftar_allreduce_rabenseifner_host(in, out, count, (ftar_dtype)dt,
                                                                        (ftar_op)op, comm);
        int crank = -1, csize = -1;
        ftar_comm_rank(comm, &crank);
        ftar_comm_size(comm, &csize);
        ftar_stats st;
        ftar_last_stats(comm, &st);
        snprintf(path, sizeof(path), "%s/out_%d_%d.bin", dir, rank, it);
        f = fopen(path, "wb");
        fwrite(out, 1, bytes, f);
        fclose(f);
        snprintf(path, sizeof(path), "%s/status_%d_%d.txt", dir, rank, it);
        f = fopen(path, "w");
        fprintf(f, "%d %d %d %d %lld %lld %lld %d %d\n", rc, crank, csize, st.recoveries, (long long)(st.wall_s * 1e6),
                (long long)(st.sync_wait_s * 1e6), (long long)(st.drain_s * 1e6), st.syncs, st.relayed_steps);
        fclose(f);
    }
    ftar_finalize(comm);
    return 0;
}
