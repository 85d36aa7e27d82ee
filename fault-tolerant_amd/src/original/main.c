/*
 * src/original/{rd,raben}.exe -- the vendor baseline of the compare campaign, the
 * counterpart of the reference's src/original/rd.c and raben.c (non-fault-tolerant
 * MPI_Allreduce with Open MPI's recursive-doubling / Rabenseifner algorithm forced).
 *
 *   ftrun -np N ./rd.exe <count>
 *
 * On MI355X the vendor Allreduce is RCCL's ncclAllReduce over xGMI.  RCCL has no
 * recursive-doubling or Rabenseifner selection (it tunes ring/tree itself), so both
 * executables run the same call; they exist so the campaign and check_compare.py keep
 * the reference's four-way layout (rd, original_rd, raben, original_raben).
 *
 * Same CLI, inputs (buffer[i] = rank, int32 SUM; FTAR_DTYPE=float32 for float) and
 * stdout grammar as the fault-tolerant drivers, and the same timed region: host
 * buffers, H2D + Allreduce + D2H + closing barrier, wall clock.  The RCCL unique id is
 * handed from rank 0 to the others through a file named after the ftrun job.
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#define CHECK_HIP(x)                                                                  \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(EXIT_FAILURE);                                                       \
        }                                                                             \
    } while (0)
#define CHECK_NCCL(x)                                                                 \
    do {                                                                              \
        ncclResult_t r_ = (x);                                                        \
        if (r_ != ncclSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_)); \
            exit(EXIT_FAILURE);                                                       \
        }                                                                             \
    } while (0)

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int env_int(const char *name, int dflt)
{
    const char *v = getenv(name);
    return v ? atoi(v) : dflt;
}

/* rank 0 publishes the unique id (write + rename, so readers never see a partial file) */
static void exchange_id(ncclUniqueId *id, int rank, char *path, size_t plen)
{
    const char *job = getenv("FTAR_JOB");
    snprintf(path, plen, "/dev/shm/ftar-rccl-id%s", job ? job : "-default");
    for (char *p = path + strlen("/dev/shm/"); *p; p++)
        if (*p == '/') *p = '-';
    if (rank == 0) {
        CHECK_NCCL(ncclGetUniqueId(id));
        char tmp[520];
        snprintf(tmp, sizeof(tmp), "%s.tmp", path);
        FILE *f = fopen(tmp, "wb");
        if (!f || fwrite(id, sizeof(*id), 1, f) != 1) {
            fprintf(stderr, "cannot write %s: %s\n", tmp, strerror(errno));
            exit(EXIT_FAILURE);
        }
        fclose(f);
        if (rename(tmp, path) != 0) {
            fprintf(stderr, "cannot publish %s: %s\n", path, strerror(errno));
            exit(EXIT_FAILURE);
        }
        return;
    }
    double t0 = now_s();
    for (;;) {
        FILE *f = fopen(path, "rb");
        if (f) {
            size_t got = fread(id, sizeof(*id), 1, f);
            fclose(f);
            if (got == 1) return;
        }
        if (now_s() - t0 > 120.0) {
            fprintf(stderr, "rank %d: no RCCL id at %s\n", rank, path);
            exit(EXIT_FAILURE);
        }
        usleep(1000);
    }
}

int main(int argc, char *argv[])
{
    if (argc < 2) {
        printf("Error: buffer size expected\n");
        return EXIT_FAILURE;
    }
    int rank = env_int("FTAR_RANK", env_int("RANK", 0));
    int size = env_int("FTAR_SIZE", env_int("WORLD_SIZE", 1));
    int ngpu = 0;
    CHECK_HIP(hipGetDeviceCount(&ngpu));
    if (ngpu <= 0) {
        fprintf(stderr, "no GPU\n");
        return EXIT_FAILURE;
    }
    int dev = env_int("FTAR_DEVICE", rank % ngpu);
    CHECK_HIP(hipSetDevice(dev));
    int buf_size = atoi(argv[1]);
    const char *dts = getenv("FTAR_DTYPE");
    int is_float = dts && !strcmp(dts, "float32");
    size_t bytes = (size_t)buf_size * 4;

    char idpath[512];
    ncclUniqueId id;
    exchange_id(&id, rank, idpath, sizeof(idpath));
    ncclComm_t comm;
    CHECK_NCCL(ncclCommInitRank(&comm, size, id, rank));
    hipStream_t s;
    CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

    void *buffer = malloc(bytes + 4), *result = malloc(bytes + 4);
    /* FTAR_FILL_OFFSET=k (default 0, the reference's input): buffer[i] = rank + k, so a one-rank
     * run has a nonzero checksum, ((N(N-1)/2 + N k) % 17) * count */
    const int fill = getenv("FTAR_FILL_OFFSET") ? atoi(getenv("FTAR_FILL_OFFSET")) : 0;
    for (int i = 0; i < buf_size; i++) {
        if (is_float) ((float *)buffer)[i] = (float)(rank + fill);
        else ((int *)buffer)[i] = rank + fill;
    }
    void *d_buf = NULL, *d_res = NULL, *d_bar = NULL;
    CHECK_HIP(hipMalloc(&d_buf, bytes + 4));
    CHECK_HIP(hipMalloc(&d_res, bytes + 4));
    CHECK_HIP(hipMalloc(&d_bar, 4));
    CHECK_HIP(hipMemset(d_bar, 0, 4));
    /* the communicator is up on every rank: the id file is no longer needed */
    CHECK_NCCL(ncclAllReduce(d_bar, d_bar, 1, ncclInt32, ncclSum, comm, s));
    CHECK_HIP(hipStreamSynchronize(s));
    if (rank == 0) unlink(idpath);

    double t0 = now_s();
    CHECK_HIP(hipMemcpyAsync(d_buf, buffer, bytes, hipMemcpyHostToDevice, s));
    CHECK_NCCL(ncclAllReduce(d_buf, d_res, (size_t)buf_size, is_float ? ncclFloat32 : ncclInt32, ncclSum, comm, s));
    CHECK_HIP(hipMemcpyAsync(result, d_res, bytes, hipMemcpyDeviceToHost, s));
    CHECK_NCCL(ncclAllReduce(d_bar, d_bar, 1, ncclInt32, ncclSum, comm, s)); /* MPI_Barrier */
    CHECK_HIP(hipStreamSynchronize(s));
    double t1 = now_s();

    uint32_t res = 0; /* int res with wrap-around, as the reference's */
    for (int i = 0; i < buf_size; i++) {
        int v = is_float ? (int)((float *)result)[i] : ((int *)result)[i];
        res += (uint32_t)(v % 17);
    }
    if (rank == 0) {
        printf("P: %d\n", size);
        printf("Size: %d\n", buf_size);
        printf("Time: %lf\n", t1 - t0);
    }
    printf("Hello from %d of %d and the result is: %d\n", rank, size, (int)res);
    fflush(stdout);

    CHECK_NCCL(ncclCommDestroy(comm));
    CHECK_HIP(hipFree(d_buf));
    CHECK_HIP(hipFree(d_res));
    CHECK_HIP(hipFree(d_bar));
    CHECK_HIP(hipStreamDestroy(s));
    free(buffer);
    free(result);
    return 0;
}
