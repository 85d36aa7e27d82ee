// ipc_probe.hip -- why did hipIpcGetMemHandle refuse a fresh workspace block (round 1,
// "invalid argument" when the workspace grew mid-job)?
//
// Two processes on GPU 0 (forked before any HIP call, a shared-memory barrier between
// them).  Each phase prints one JSON line.
//   importer_reuse: B imports A's block, closes the mapping, then hipMallocs blocks of
//       the same and of larger sizes and exports each: does an export fail, and does the
//       failing block overlap the VA range B's closed import occupied?
//   growth: the library's workspace pattern -- both processes allocate 4 blocks, export,
//       import the peer's 4, close them, free their own, grow x2, for 2 MiB .. 1 GiB --
//       counting exports refused on the first try, with the overlap test.
//   capacity: the per-process IPC resources of the reference's largest NP (4
//       exported buffers x 31 peers = 124 imports per rank at N = 32, 252 at N = 64, which one
//       GPU cannot host as 32 / 64 processes): each process exports K blocks (a distinct
//       pattern in each), imports the peer's K, checks every import reads its owner's pattern,
//       stores a word into every imported block, and each owner checks the words landed;
//       import / close times reported at 124 and at K.
//   reexport: one allocation exported again and again (a fresh handle per round) and
//       imported by the peer under three disciplines -- each handle opened and closed before
//       the next export; the first handle re-opened after its close; each new handle opened
//       while the previous import is still open -- the error of every open.
// Usage: ipc_probe [K blocks per process, default 252] [MiB per block, default 4]
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/ipc_probe.hip -o tools/_build/ipc_probe
#include <hip/hip_runtime.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#define NB 4
#define MAXR 16
#define MAXK 256

struct Shm {
    _Atomic int bar[2];
    hipIpcMemHandle_t h[2][NB];
    hipIpcMemHandle_t hk[2][MAXK];
    int fail;
};

static Shm *S;
static int me;
static int gen;

static void barrier()
{
    gen++;
    atomic_store(&S->bar[me], gen);
    while (atomic_load(&S->bar[1 - me]) < gen) usleep(50);
}

struct Range {
    uintptr_t b, e;
};

static bool overlaps(void *p, size_t n, const Range *r, int nr)
{
    uintptr_t b = (uintptr_t)p, e = b + n;
    for (int i = 0; i < nr; i++)
        if (b < r[i].e && r[i].b < e) return true;
    return false;
}

static void importer_reuse()
{
    const size_t s = 64ull << 20;
    void *x = nullptr;
    if (me == 0) {
        (void)hipMalloc(&x, s);
        (void)hipIpcGetMemHandle(&S->h[0][0], x);
    }
    barrier();
    if (me == 1) {
        void *imp = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&imp, S->h[0][0], hipIpcMemLazyEnablePeerAccess);
        Range r = {(uintptr_t)imp, (uintptr_t)imp + s};
        (void)hipIpcCloseMemHandle(imp);
        printf("{\"phase\": \"importer_reuse\", \"open\": %d, \"import_va\": \"%p\", \"allocs\": [", (int)e, imp);
        const size_t sizes[] = {64ull << 20, 32ull << 20, 128ull << 20, 2ull << 20, 256ull << 20};
        for (int i = 0; i < 5; i++) {
            void *y = nullptr;
            (void)hipMalloc(&y, sizes[i]);
            hipIpcMemHandle_t h;
            hipError_t ee = hipIpcGetMemHandle(&h, y);
            if (ee != hipSuccess) (void)hipGetLastError();
            printf("%s{\"MiB\": %zu, \"va\": \"%p\", \"overlaps_closed_import\": %s, \"export\": \"%s\"}", i ? ", " : "",
                   sizes[i] >> 20, y, overlaps(y, sizes[i], &r, 1) ? "true" : "false", hipGetErrorString(ee));
            (void)hipFree(y);
        }
        printf("]}\n");
        fflush(stdout);
    }
    barrier();
    if (me == 0) (void)hipFree(x);
    barrier();
}

static void growth()
{
    Range closed[MAXR * NB];
    int nclosed = 0, refused = 0, refused_overlap = 0, rounds = 0;
    void *own[NB] = {};
    size_t s = 2ull << 20;
    char log[8192];
    log[0] = 0;
    int off = 0;
    for (int r = 0; r < 10; r++, s *= 2, rounds++) {
        for (int b = 0; b < NB; b++) {
            (void)hipMalloc(&own[b], s);
            hipError_t e = hipIpcGetMemHandle(&S->h[me][b], own[b]);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                refused++;
                bool ov = overlaps(own[b], s, closed, nclosed);
                refused_overlap += ov;
                off += snprintf(log + off, sizeof(log) - off, "%s{\"round\": %d, \"MiB\": %zu, \"va\": \"%p\", "
                                "\"overlaps_closed_import\": %s, \"err\": \"%s\"}", off ? ", " : "", r, s >> 20,
                                own[b], ov ? "true" : "false", hipGetErrorString(e));
                // keep it (like the library's retry) and try once more
                void *again = nullptr;
                (void)hipMalloc(&again, s);
                e = hipIpcGetMemHandle(&S->h[me][b], again);
                (void)hipFree(own[b]);
                own[b] = again;
                if (e != hipSuccess) {
                    (void)hipGetLastError();
                    S->fail = 1;
                }
            }
        }
        barrier();
        void *imp[NB];
        for (int b = 0; b < NB; b++) {
            imp[b] = nullptr;
            if (hipIpcOpenMemHandle(&imp[b], S->h[1 - me][b], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                (void)hipGetLastError();
                S->fail = 1;
            }
        }
        barrier();
        for (int b = 0; b < NB; b++) {
            if (imp[b] && nclosed < MAXR * NB) closed[nclosed++] = Range{(uintptr_t)imp[b], (uintptr_t)imp[b] + s};
            if (imp[b]) (void)hipIpcCloseMemHandle(imp[b]);
        }
        barrier();
        for (int b = 0; b < NB; b++) (void)hipFree(own[b]);
    }
    printf("{\"phase\": \"growth\", \"rank\": %d, \"rounds\": %d, \"refused_first_try\": %d, "
           "\"refused_overlapping_closed_import\": %d, \"refusals\": [%s]}\n",
           me, rounds, refused, refused_overlap, log);
    fflush(stdout);
}

static double now_ms()
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

static unsigned pattern(int owner, int b) { return 0x51000000u + (unsigned)owner * 0x10000u + (unsigned)b; }

static void capacity(int K, size_t s)
{
    static void *own[MAXK], *imp[MAXK];
    int alloc_ok = 0, export_ok = 0, import_ok = 0, read_ok = 0, write_ok = 0, landed_ok = 0;
    for (int b = 0; b < K; b++) {
        own[b] = nullptr;
        if (hipMalloc(&own[b], s) != hipSuccess) {
            (void)hipGetLastError();
            own[b] = nullptr;
            continue;
        }
        alloc_ok++;
        (void)hipMemsetD32((hipDeviceptr_t)own[b], pattern(me, b), s / 4);
        if (hipIpcGetMemHandle(&S->hk[me][b], own[b]) == hipSuccess) export_ok++;
        else (void)hipGetLastError();
    }
    (void)hipDeviceSynchronize();
    barrier();
    double t0 = now_ms(), t124 = 0;
    for (int b = 0; b < K; b++) {
        imp[b] = nullptr;
        if (hipIpcOpenMemHandle(&imp[b], S->hk[1 - me][b], hipIpcMemLazyEnablePeerAccess) == hipSuccess) import_ok++;
        else {
            (void)hipGetLastError();
            imp[b] = nullptr;
        }
        if (b + 1 == 124) t124 = now_ms() - t0;
    }
    const double t_import = now_ms() - t0;
    for (int b = 0; b < K; b++) {
        if (!imp[b]) continue;
        unsigned head[4] = {}, tail[4] = {};
        if (hipMemcpy(head, imp[b], 16, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(tail, (char *)imp[b] + s - 16, 16, hipMemcpyDeviceToHost) != hipSuccess) {
            (void)hipGetLastError();
            continue;
        }
        bool ok = true;
        for (int i = 0; i < 4; i++) ok = ok && head[i] == pattern(1 - me, b) && tail[i] == pattern(1 - me, b);
        read_ok += ok;
        const unsigned mark = 0xABC00000u + (unsigned)me * 0x1000u + (unsigned)b;
        if (hipMemcpy((char *)imp[b] + 64, &mark, 4, hipMemcpyHostToDevice) == hipSuccess) write_ok++;
        else (void)hipGetLastError();
    }
    (void)hipDeviceSynchronize();
    barrier();
    for (int b = 0; b < K; b++) {
        unsigned w = 0;
        if (own[b] && hipMemcpy(&w, (char *)own[b] + 64, 4, hipMemcpyDeviceToHost) == hipSuccess)
            landed_ok += w == 0xABC00000u + (unsigned)(1 - me) * 0x1000u + (unsigned)b;
    }
    barrier();
    t0 = now_ms();
    for (int b = 0; b < K; b++)
        if (imp[b]) (void)hipIpcCloseMemHandle(imp[b]);
    const double t_close = now_ms() - t0;
    barrier();
    for (int b = 0; b < K; b++)
        if (own[b]) (void)hipFree(own[b]);
    const bool all = alloc_ok == K && export_ok == K && import_ok == K && read_ok == K && write_ok == K && landed_ok == K;
    if (!all) S->fail = 1;
    printf("{\"phase\": \"capacity\", \"rank\": %d, \"blocks\": %d, \"MiB_per_block\": %zu, \"mapped_GiB\": %.2f, "
           "\"alloc_ok\": %d, \"export_ok\": %d, \"import_ok\": %d, \"read_ok\": %d, \"write_ok\": %d, "
           "\"landed_ok\": %d, \"all_ok\": %s, \"import_ms_first_124\": %.2f, \"import_ms_all\": %.2f, "
           "\"close_ms_all\": %.2f}\n",
           me, K, s >> 20, (double)K * (double)s / (1u << 30), alloc_ok, export_ok, import_ok, read_ok, write_ok,
           landed_ok, all ? "true" : "false", t124, t_import, t_close);
    fflush(stdout);
}

static void reexport()
{
    const size_t s = 16ull << 20;
    void *a = nullptr;
    if (me == 0) {
        (void)hipMalloc(&a, s);
        (void)hipMemsetD32((hipDeviceptr_t)a, pattern(0, 7), s / 4);
        (void)hipDeviceSynchronize();
    }
    const char *names[3] = {"open_close_each", "reopen_first_after_close", "open_while_previous_open"};
    for (int mode = 0; mode < 3; mode++) {
        char log[1024];
        int off = 0, bad = 0;
        void *prev = nullptr;
        for (int r = 0; r < 5; r++) {
            if (me == 0 && (mode != 1 || r == 0)) {
                if (hipIpcGetMemHandle(&S->hk[0][r], a) != hipSuccess) {
                    (void)hipGetLastError();
                    S->fail = 1;
                }
            }
            barrier();
            if (me == 1) {
                void *imp = nullptr;
                hipError_t e = hipIpcOpenMemHandle(&imp, S->hk[0][mode == 1 ? 0 : r], hipIpcMemLazyEnablePeerAccess);
                unsigned w = 0;
                if (e == hipSuccess) {
                    if (hipMemcpy(&w, imp, 4, hipMemcpyDeviceToHost) != hipSuccess) (void)hipGetLastError();
                } else {
                    (void)hipGetLastError();
                }
                const bool ok = e == hipSuccess && w == pattern(0, 7);
                bad += !ok;
                off += snprintf(log + off, sizeof(log) - off, "%s\"%s\"", r ? ", " : "", ok ? "ok" : hipGetErrorString(e));
                if (mode == 2) {
                    if (prev) (void)hipIpcCloseMemHandle(prev);
                    prev = imp;
                } else if (imp) {
                    (void)hipIpcCloseMemHandle(imp);
                }
            }
            barrier();
        }
        if (me == 1) {
            if (prev) (void)hipIpcCloseMemHandle(prev);
            printf("{\"phase\": \"reexport\", \"mode\": \"%s\", \"bad\": %d, \"opens\": [%s]}\n", names[mode], bad, log);
            fflush(stdout);
        }
        barrier();
    }
    if (me == 0) (void)hipFree(a);
    barrier();
}

int main(int argc, char **argv)
{
    int K = argc > 1 ? atoi(argv[1]) : 252;
    size_t mib = argc > 2 ? (size_t)atoll(argv[2]) : 4;
    if (K < 1 || K > MAXK || mib < 1 || mib > 1024) {
        fprintf(stderr, "usage: ipc_probe [K 1..%d] [MiB 1..1024]\n", MAXK);
        return 2;
    }
    S = (Shm *)mmap(nullptr, sizeof(Shm), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    memset(S, 0, sizeof(Shm));
    pid_t kids[2];
    for (int k = 0; k < 2; k++) {
        kids[k] = fork();
        if (kids[k] == 0) {
            me = k;
            if (hipSetDevice(0) != hipSuccess) _exit(3);
            importer_reuse();
            growth();
            capacity(K, mib << 20);
            reexport();
            _exit(0);
        }
    }
    int rc = 0;
    for (int k = 0; k < 2; k++) {
        int st = 0;
        waitpid(kids[k], &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
    }
    printf("{\"phase\": \"done\", \"ok\": %s, \"fail\": %d}\n", rc ? "false" : "true", S->fail);
    return rc;
}
