// xgmi_probe.hip -- the node's xGMI fabric in the access patterns the exchanges use,
// measured from ONE process that drives every GPU of the job (peer access enabled
// between all pairs; no IPC).  SURVEY.md 8d asks for B_link "calibrated ... with both
// directions loaded"; bench.py's N > 1 line carries this probe's JSON as `xgmi_probe`.
//
//   pull1 / push1          GPU 0 reads from / writes to GPU 1 with a copy kernel
//                          (one link, one direction)
//   pull1_bidir / push1_bidir   GPUs 0 and 1 at once, each from / to the other
//                          (one link, both directions loaded: the B_link of SURVEY 8d)
//   sdma1_bidir            the same with hipMemcpyPeerAsync (the copy engines)
//   pull_all / push_all    every GPU reads from / writes to all n - 1 peers at once, S/n
//                          per peer -- the one-hop mesh's reduce-scatter / allgather
//                          pattern -- (n - 1) S / n per GPU per direction
//
// Kernels: 16-byte non-temporal loads and stores, 4 per lane in flight (the product's
// tile), workgroups dealt round-robin over the peers so every link streams at once.
// Each pattern: 2 untimed runs, then `iters` timed runs between hipEvents on every
// device; the time is the max over the GPUs involved.  Every pattern's destination is
// checked (a sample of elements against the value its source holds).
//
//   xgmi_probe [ngpus] [MiB] [iters]      (defaults: every visible GPU, 256, 10)
// With one GPU it runs the kernels in loopback (device 0 to itself) and reports no link
// figures; XGMI_PROBE_VIRTUAL=n runs every pattern with n "GPUs" on device 0 (a self-test
// of the patterns and their checks; the figures are HBM figures).  One JSON line on stdout.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#define CHK(x)                                                                                    \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));                      \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

constexpr int kMaxSeg = 8;
constexpr int kBlock = 256, kUnroll = 4;
constexpr size_t kTile = (size_t)kBlock * kUnroll; // 16-byte vectors per workgroup pass

struct Seg {
    const uint4 *src;
    uint4 *dst;
    size_t nv; // 16-byte vectors
};
struct SegList {
    Seg s[kMaxSeg];
    int n;
};

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// workgroup b copies tiles b / n, b / n + G / n, ... of segment b % n
__global__ __launch_bounds__(kBlock) void multi_copy(SegList L)
{
    const int n = L.n;
    const int sg = (int)(blockIdx.x % (unsigned)n);
    const size_t per = gridDim.x / (unsigned)n;
    const Seg S = L.s[sg];
    const v4u *src = (const v4u *)S.src;
    v4u *dst = (v4u *)S.dst;
    for (size_t base = (size_t)(blockIdx.x / (unsigned)n) * kTile; base < S.nv; base += per * kTile) {
        const size_t i = base + threadIdx.x;
        if (base + kTile <= S.nv) {
            v4u v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; u++) v[u] = __builtin_nontemporal_load(src + i + u * kBlock);
#pragma unroll
            for (int u = 0; u < kUnroll; u++) __builtin_nontemporal_store(v[u], dst + i + u * kBlock);
        } else {
            for (size_t j = i; j < S.nv; j += kBlock) __builtin_nontemporal_store(__builtin_nontemporal_load(src + j), dst + j);
        }
    }
}

__global__ void fill(float *p, size_t n, float base)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = base + (float)(i % 4093);
}

struct Dev {
    hipStream_t st;
    hipEvent_t e0, e1;
    float *src, *dst; // S bytes each
};

static int g_n;
static size_t g_bytes;
static std::vector<Dev> D;
static int g_visible = 1, g_virtual = 0;
// the physical device of (virtual) GPU d: itself, or GPU 0 for every d in the
// self-test mode (XGMI_PROBE_VIRTUAL=n: n "GPUs" on one device, the n > 1 patterns and
// their checks run, the figures are HBM figures)
static int phys(int d) { return g_virtual ? 0 : d; }

// one launch of `L` on device d (grid: 2048 workgroups per segment at most)
static void launch(int d, const SegList &L)
{
    size_t tiles = 0;
    for (int k = 0; k < L.n; k++) tiles = L.s[k].nv / kTile > tiles ? L.s[k].nv / kTile : tiles;
    size_t per = tiles < 2048 ? (tiles ? tiles : 1) : 2048;
    CHK(hipSetDevice(phys(d)));
    hipLaunchKernelGGL(multi_copy, dim3((unsigned)(per * (size_t)L.n)), dim3(kBlock), 0, D[d].st, L);
    CHK(hipGetLastError());
}

static void sync_all(const std::vector<int> &devs)
{
    for (int d : devs) {
        CHK(hipSetDevice(phys(d)));
        CHK(hipStreamSynchronize(D[d].st));
    }
}

// times `body(d)` issued on every device of `devs` at once; returns ms per run (max over
// the devices of the event time)
template <class F> static double timed(const std::vector<int> &devs, int iters, F body)
{
    for (int w = 0; w < 2; w++)
        for (int d : devs) body(d);
    sync_all(devs);
    for (int d : devs) {
        CHK(hipSetDevice(phys(d)));
        CHK(hipEventRecord(D[d].e0, D[d].st));
    }
    for (int it = 0; it < iters; it++)
        for (int d : devs) body(d);
    for (int d : devs) {
        CHK(hipSetDevice(phys(d)));
        CHK(hipEventRecord(D[d].e1, D[d].st));
    }
    sync_all(devs);
    double worst = 0;
    for (int d : devs) {
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, D[d].e0, D[d].e1));
        if (ms > worst) worst = ms;
    }
    return worst / iters;
}

// element i of the destination at `dst_off` bytes equals element i of device `from`'s
// source at `src_off` bytes (sampled)
static bool check(int d, size_t dst_off, int from, size_t src_off, size_t bytes)
{
    const size_t n = bytes / 4;
    const size_t idx[4] = {0, n / 3, n / 2 + 1, n - 1};
    for (size_t k : idx) {
        float got, want;
        CHK(hipMemcpy(&got, (char *)D[d].dst + dst_off + 4 * k, 4, hipMemcpyDefault));
        CHK(hipMemcpy(&want, (char *)D[from].src + src_off + 4 * k, 4, hipMemcpyDefault));
        if (got != want) return false;
    }
    return true;
}

static void clear_dst(const std::vector<int> &devs)
{
    for (int d : devs) {
        CHK(hipSetDevice(phys(d)));
        CHK(hipMemsetAsync(D[d].dst, 0, g_bytes, D[d].st));
    }
    sync_all(devs);
}

int main(int argc, char **argv)
{
    int visible = 0;
    CHK(hipGetDeviceCount(&visible));
    g_visible = visible;
    const char *ve = getenv("XGMI_PROBE_VIRTUAL");
    g_virtual = ve ? atoi(ve) : 0;
    g_n = argc > 1 && atoi(argv[1]) > 0 ? atoi(argv[1]) : visible;
    if (g_virtual > 0) g_n = g_virtual;
    else if (g_n > visible) g_n = visible;
    if (g_n > kMaxSeg) g_n = kMaxSeg;
    const size_t mib = argc > 2 ? strtoull(argv[2], nullptr, 10) : 256;
    const int iters = argc > 3 ? atoi(argv[3]) : 10;
    const size_t unit = 4096 * (size_t)g_n; // S / n stays a whole number of 4 KiB pages
    g_bytes = (mib << 20) / unit * unit;
    const size_t S = g_bytes;
    D.resize(g_n);
    int peer_ok = 1;
    for (int d = 0; d < g_n; d++) {
        CHK(hipSetDevice(phys(d)));
        CHK(hipStreamCreateWithFlags(&D[d].st, hipStreamNonBlocking));
        CHK(hipEventCreate(&D[d].e0));
        CHK(hipEventCreate(&D[d].e1));
        CHK(hipMalloc(&D[d].src, S));
        CHK(hipMalloc(&D[d].dst, S));
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, D[d].st, D[d].src, S / 4, 10000.0f * (float)(d + 1));
        CHK(hipGetLastError());
        for (int q = 0; q < g_n; q++) {
            if (q == d || g_virtual) continue;
            int can = 0;
            CHK(hipDeviceCanAccessPeer(&can, d, q));
            if (!can) {
                peer_ok = 0;
                continue;
            }
            hipError_t e = hipDeviceEnablePeerAccess(q, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) peer_ok = 0;
            (void)hipGetLastError();
        }
    }
    std::vector<int> all;
    for (int d = 0; d < g_n; d++) all.push_back(d);
    sync_all(all);

    std::string out = "{\"tool\": \"xgmi_probe\", \"gpus\": " + std::to_string(g_n) +
                      (g_virtual ? ", \"virtual_on_one_device\": true" : "") +
                      ", \"bytes\": " + std::to_string(S) + ", \"iters\": " + std::to_string(iters) +
                      ", \"peer_access\": " + (peer_ok ? "true" : "false") + ", \"patterns\": {";
    bool first = true, all_ok = true;
    char buf[512];
    auto emit = [&](const char *name, double ms, double bytes_per_gpu, int links, bool ok) {
        const double gbs = bytes_per_gpu / (ms * 1e-3) / 1e9;
        char per_link[32] = "null";
        if (links) snprintf(per_link, sizeof(per_link), "%.1f", gbs / links);
        snprintf(buf, sizeof(buf), "%s\"%s\": {\"ms\": %.4f, \"GBps_per_gpu\": %.1f, \"GBps_per_link\": %s, \"ok\": %s}",
                 first ? "" : ", ", name, ms, gbs, per_link, ok ? "true" : "false");
        out += buf;
        first = false;
        all_ok = all_ok && ok;
    };
    const size_t nv = S / 16;
    if (g_n < 2 || !peer_ok) {
        // loopback: the kernel on device 0's own memory (no link in the path)
        clear_dst(all);
        SegList L{};
        L.n = 1;
        L.s[0] = {(const uint4 *)D[0].src, (uint4 *)D[0].dst, nv};
        double ms = timed({0}, iters, [&](int) { launch(0, L); });
        emit("loopback_copy", ms, (double)S, 0, check(0, 0, 0, 0, S));
    } else {
        // one link, one direction
        clear_dst(all);
        {
            SegList L{};
            L.n = 1;
            L.s[0] = {(const uint4 *)D[1].src, (uint4 *)D[0].dst, nv};
            double ms = timed({0}, iters, [&](int) { launch(0, L); });
            emit("pull1", ms, (double)S, 1, check(0, 0, 1, 0, S));
        }
        clear_dst(all);
        {
            SegList L{};
            L.n = 1;
            L.s[0] = {(const uint4 *)D[0].src, (uint4 *)D[1].dst, nv};
            double ms = timed({0}, iters, [&](int) { launch(0, L); });
            emit("push1", ms, (double)S, 1, check(1, 0, 0, 0, S));
        }
        // one link, both directions
        clear_dst(all);
        {
            SegList L[2]{};
            for (int d = 0; d < 2; d++) {
                L[d].n = 1;
                L[d].s[0] = {(const uint4 *)D[1 - d].src, (uint4 *)D[d].dst, nv};
            }
            double ms = timed({0, 1}, iters, [&](int d) { launch(d, L[d]); });
            emit("pull1_bidir", ms, (double)S, 1, check(0, 0, 1, 0, S) && check(1, 0, 0, 0, S));
        }
        clear_dst(all);
        {
            SegList L[2]{};
            for (int d = 0; d < 2; d++) {
                L[d].n = 1;
                L[d].s[0] = {(const uint4 *)D[d].src, (uint4 *)D[1 - d].dst, nv};
            }
            double ms = timed({0, 1}, iters, [&](int d) { launch(d, L[d]); });
            emit("push1_bidir", ms, (double)S, 1, check(0, 0, 1, 0, S) && check(1, 0, 0, 0, S));
        }
        clear_dst(all);
        {
            double ms = timed({0, 1}, iters, [&](int d) {
                CHK(hipSetDevice(phys(d)));
                CHK(hipMemcpyPeerAsync(D[d].dst, phys(d), D[1 - d].src, phys(1 - d), S, D[d].st));
            });
            emit("sdma1_bidir", ms, (double)S, 1, check(0, 0, 1, 0, S) && check(1, 0, 0, 0, S));
        }
        // every GPU with all n - 1 peers at once: block q of S/n bytes per peer
        const size_t blk = S / (size_t)g_n, bv = blk / 16;
        clear_dst(all);
        {
            std::vector<SegList> L(g_n);
            for (int d = 0; d < g_n; d++) {
                L[d].n = 0;
                for (int q = 0; q < g_n; q++)
                    if (q != d)
                        L[d].s[L[d].n++] = {(const uint4 *)((char *)D[q].src + (size_t)d * blk),
                                            (uint4 *)((char *)D[d].dst + (size_t)q * blk), bv};
            }
            double ms = timed(all, iters, [&](int d) { launch(d, L[d]); });
            bool ok = true;
            for (int d = 0; d < g_n; d++)
                for (int q = 0; q < g_n; q++)
                    if (q != d) ok = ok && check(d, (size_t)q * blk, q, (size_t)d * blk, blk);
            emit("pull_all", ms, (double)blk * (g_n - 1), g_n - 1, ok);
        }
        clear_dst(all);
        {
            std::vector<SegList> L(g_n);
            for (int d = 0; d < g_n; d++) {
                L[d].n = 0;
                for (int q = 0; q < g_n; q++)
                    if (q != d)
                        L[d].s[L[d].n++] = {(const uint4 *)((char *)D[d].src + (size_t)q * blk),
                                            (uint4 *)((char *)D[q].dst + (size_t)d * blk), bv};
            }
            double ms = timed(all, iters, [&](int d) { launch(d, L[d]); });
            bool ok = true;
            for (int d = 0; d < g_n; d++)
                for (int q = 0; q < g_n; q++)
                    if (q != d) ok = ok && check(q, (size_t)d * blk, d, (size_t)q * blk, blk);
            emit("push_all", ms, (double)blk * (g_n - 1), g_n - 1, ok);
        }
    }
    out += std::string("}, \"ok\": ") + (all_ok ? "true" : "false") + "}";
    printf("%s\n", out.c_str());
    for (int d = 0; d < g_n; d++) {
        CHK(hipSetDevice(phys(d)));
        CHK(hipFree(D[d].src));
        CHK(hipFree(D[d].dst));
        CHK(hipStreamDestroy(D[d].st));
    }
    return all_ok ? 0 : 1;
}
