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
 *      FTAR_PROBE_DEVICE=1 (device-pointer entry points on this process's own malloc buffers:
 *      host-sim: "device" memory is host memory; GPU build: must be refused),
 *      FTAR_PROBE_INPLACE=1 (send buffer = receive buffer),
 *      FTAR_PROBE_OFFSET=k (buffers start k elements past a 16-byte boundary),
 *      FTAR_PROBE_PINNED=1 (buffers from hipHostMalloc, looked up in the loaded HIP runtime:
 *      the _host entry points then run zero copy; host-sim build: no runtime, plain memory),
 *      FTAR_PROBE_SLEEP_US=t (sleep before every call: a late rank, with FTAR_PROBE_RANK_ENV),
 *      FTAR_PROBE_CYCLE_SEQ=i,j,... (host-sim, with FTAR_PROBE_DEVICE=1: call k sends from
 *      exportable buffer number seq[k], each holding the input -- a caller cycling its send
 *      buffers through the peers' mapping caches)
 */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "ftar.h"

static size_t esize(int dt) { return (dt == 0 || dt == 1) ? 4 : 8; }

static char *probe_alloc(size_t n, int pinned)
{
    if (pinned) {
        int (*host_malloc)(void **, size_t, unsigned) =
            (int (*)(void **, size_t, unsigned))dlsym(RTLD_DEFAULT, "hipHostMalloc");
        if (host_malloc) {
            void *p = NULL;
            return host_malloc(&p, n, 0) == 0 ? p : NULL;
        }
    }
    return aligned_alloc(64, n);
}

static void probe_free(char *p, int pinned)
{
    int (*host_free)(void *) = pinned ? (int (*)(void *))dlsym(RTLD_DEFAULT, "hipHostFree") : NULL;
    if (host_free)
        host_free(p);
    else
        free(p);
}

int main(void)
{
    const char *dir = getenv("FTAR_PROBE_DIR");
    const char *algo = getenv("FTAR_PROBE_ALGO");
    if (!dir || !algo) return 2;
    int dt = getenv("FTAR_PROBE_DTYPE") ? atoi(getenv("FTAR_PROBE_DTYPE")) : 0;
    int op = getenv("FTAR_PROBE_OP") ? atoi(getenv("FTAR_PROBE_OP")) : 0;
    size_t count = getenv("FTAR_PROBE_COUNT") ? strtoull(getenv("FTAR_PROBE_COUNT"), NULL, 10) : 0;
    int iters = getenv("FTAR_PROBE_ITERS") ? atoi(getenv("FTAR_PROBE_ITERS")) : 1;
    int dev = getenv("FTAR_PROBE_DEVICE") ? atoi(getenv("FTAR_PROBE_DEVICE")) : 0;
    int inplace = getenv("FTAR_PROBE_INPLACE") ? atoi(getenv("FTAR_PROBE_INPLACE")) : 0;
    size_t off = getenv("FTAR_PROBE_OFFSET") ? strtoull(getenv("FTAR_PROBE_OFFSET"), NULL, 10) : 0;

    /* FTAR_PROBE_RANK_ENV="r:NAME=VALUE": one rank's own setting (a knob the launcher would
     * otherwise give every rank alike) */
    const char *re = getenv("FTAR_PROBE_RANK_ENV"), *me = getenv("FTAR_RANK");
    if (re && me && atoi(re) == atoi(me) && strchr(re, ':') && strchr(re, '=')) {
        char kv[256];
        snprintf(kv, sizeof(kv), "%s", strchr(re, ':') + 1);
        char *eq = strchr(kv, '=');
        *eq = 0;
        setenv(kv, eq + 1, 1);
    }
    ftar_comm *comm;
    if (ftar_init(&comm) != FTAR_SUCCESS) return 3;
    int rank;
    ftar_world_rank(comm, &rank);
    size_t bytes = count * esize(dt);
    size_t pad = off * esize(dt);
    int pinned = getenv("FTAR_PROBE_PINNED") ? atoi(getenv("FTAR_PROBE_PINNED")) : 0;
    char *in_mem = probe_alloc((bytes + pad + 64) / 64 * 64, pinned);
    char *out_mem = probe_alloc((bytes + pad + 64) / 64 * 64, pinned);
    if (!in_mem || !out_mem) return 5;
    void *in = in_mem + pad, *out = out_mem + pad;
    char path[512];
    snprintf(path, sizeof(path), "%s/in_%d.bin", dir, rank);
    FILE *f = fopen(path, "rb");
    if (!f || fread(in, 1, bytes, f) != bytes) return 4;
    fclose(f);
    void *pristine = malloc(bytes ? bytes : 1);
    memcpy(pristine, in, bytes);
    /* FTAR_PROBE_CYCLE_SEQ: the send buffer of every call, from a set of exportable buffers */
    int seq[256], nseq = 0, nbuf = 0;
    char *cyc[64] = {0};
    void *(*dev_alloc)(size_t) = NULL;
    void (*dev_free)(void *) = NULL;
    if (getenv("FTAR_PROBE_CYCLE_SEQ")) {
        dev_alloc = (void *(*)(size_t))dlsym(RTLD_DEFAULT, "ftar_hostsim_device_alloc");
        dev_free = (void (*)(void *))dlsym(RTLD_DEFAULT, "ftar_hostsim_device_free");
        if (!dev_alloc || !dev_free) return 6;
        for (const char *q = getenv("FTAR_PROBE_CYCLE_SEQ"); *q && nseq < 256; q += strcspn(q, ","), q += *q == ',') {
            seq[nseq] = atoi(q);
            if (seq[nseq] < 0 || seq[nseq] >= 64) return 6;
            if (seq[nseq] + 1 > nbuf) nbuf = seq[nseq] + 1;
            nseq++;
        }
        for (int b = 0; b < nbuf; b++) {
            if (!(cyc[b] = dev_alloc(bytes + pad + 64))) return 5;
            memcpy(cyc[b] + pad, in, bytes);
        }
    }
    for (int it = 0; it < iters; it++) {
        memset(out, 0xEE, bytes);
        const void *src = nseq ? (const void *)(cyc[seq[it % nseq]] + pad) : in;
        if (inplace) {
            memcpy(out, in, bytes);
            src = out;
        }
        int rd = !strcmp(algo, "rd"), rc;
        /* FTAR_PROBE_SLEEP_US (with FTAR_PROBE_RANK_ENV: one rank): arrive late at every call */
        if (getenv("FTAR_PROBE_SLEEP_US")) usleep((useconds_t)atoll(getenv("FTAR_PROBE_SLEEP_US")));
        if (dev)
            rc = rd ? ftar_recursive_doubling(src, out, count, (ftar_dtype)dt, (ftar_op)op, comm)
                    : ftar_allreduce_rabenseifner(src, out, count, (ftar_dtype)dt, (ftar_op)op, comm);
        else
            rc = rd ? ftar_recursive_doubling_host(src, out, count, (ftar_dtype)dt, (ftar_op)op, comm)
                    : ftar_allreduce_rabenseifner_host(src, out, count, (ftar_dtype)dt, (ftar_op)op, comm);
        if (!inplace && memcmp(src, pristine, bytes) != 0) rc = 99; /* the send buffer was written */
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
        fprintf(f, "%d %d %d %d %lld %lld %lld %d %d %d %d %d %d %d %d %d %d\n", rc, crank, csize, st.recoveries,
                (long long)(st.wall_s * 1e6), (long long)(st.sync_wait_s * 1e6), (long long)(st.drain_s * 1e6), st.syncs,
                st.relayed_steps, st.mesh_steps, st.gated_launches, st.gated_skips, st.step0_copy, st.gate_holds,
                st.gate_relaunches, st.peer_waits, st.peer_wait_skips);
        fclose(f);
    }
    ftar_finalize(comm);
    for (int b = 0; b < nbuf; b++) dev_free(cyc[b]);
    free(pristine);
    probe_free(in_mem, pinned);
    probe_free(out_mem, pinned);
    return 0;
}
