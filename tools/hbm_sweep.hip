// hbm_sweep.hip -- C2 local-reduce (inout += in, fp32, 2 x 256 MiB) variants timed on
// ROTATING buffers: every launch works on one of R pairs (R x 512 MiB, default 4 = 2 GiB),
// so the 256 MiB Infinity Cache never holds the operands of the next launch -- an HBM
// number, unlike a loop over one pair (round 1 measured 7.0 TB/s that way, 6.0 rotating).
// Also the calibration streams: read-only, write-only, copy, hipMemcpy D2D.
//   name  kernel_us  GB/s(algorithmic)  ok
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/hbm_sweep.hip -o tools/_build/hbm_sweep
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x)                                                                                              \
    do {                                                                                                    \
        hipError_t e = (x);                                                                                 \
        if (e != hipSuccess) {                                                                              \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                                          \
            exit(1);                                                                                        \
        }                                                                                                   \
    } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4f ldnt(const v4f *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ v4f ldpl(const v4f *p) { return *p; }
template <int NT> __device__ __forceinline__ v4f ld(const v4f *p)
{
    if constexpr (NT) return ldnt(p);
    else return ldpl(p);
}
template <int NT> __device__ __forceinline__ void st(v4f *p, v4f v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// remap the block index so each XCD (blocks are dispatched round-robin over the 8 XCDs)
// streams one contiguous 1/8 of the grid's tiles
template <int XCD> __device__ __forceinline__ unsigned blk()
{
    unsigned b = blockIdx.x;
    if constexpr (XCD) {
        const unsigned per = gridDim.x / 8;
        b = (b % 8) * per + b / 8;
    }
    return b;
}

// one tile of U * BS vectors per block (the product's segment-kernel mapping)
template <int U, int BS, int XCD, int NTL, int NTS>
__global__ __launch_bounds__(BS) void k_tile(v4f *__restrict__ io, const v4f *__restrict__ in, size_t nv)
{
    const size_t base = (size_t)blk<XCD>() * U * BS + threadIdx.x;
    v4f a[U], c[U];
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = ld<NTL>(io + base + u * BS);
#pragma unroll
    for (int u = 0; u < U; u++) c[u] = ld<NTL>(in + base + u * BS);
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(io + base + u * BS, a[u] + c[u]);
}

// the product's LDS-DMA variant: `in` HBM -> LDS (global_load_lds_dwordx4), io to VGPRs
template <int U, int XCD, int AUX, int NTS = 0>
__global__ __launch_bounds__(256) void k_lds(v4f *__restrict__ io, const v4f *__restrict__ in, size_t nv)
{
    __shared__ v4f stage[U * 256];
    const int wave = threadIdx.x >> 6;
    const size_t base = (size_t)blk<XCD>() * U * 256;
#pragma unroll
    for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(in + base + u * 256 + threadIdx.x),
                                         (__attribute__((address_space(3))) void *)&stage[u * 256 + wave * 64], 16, 0, AUX);
    v4f a[U];
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = ld<1>(io + base + u * 256 + threadIdx.x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(io + base + u * 256 + threadIdx.x, a[u] + stage[u * 256 + threadIdx.x]);
}

// both operands staged HBM -> LDS by the DMA path (no VGPR loads at all); stores as k_lds
template <int U, int AUX, int NTS>
__global__ __launch_bounds__(256) void k_lds2(v4f *__restrict__ io, const v4f *__restrict__ in, size_t nv)
{
    __shared__ v4f sa[U * 256], sb[U * 256];
    const int wave = threadIdx.x >> 6;
    const size_t base = (size_t)blockIdx.x * U * 256;
#pragma unroll
    for (int u = 0; u < U; u++) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(io + base + u * 256 + threadIdx.x),
                                         (__attribute__((address_space(3))) void *)&sa[u * 256 + wave * 64], 16, 0, AUX);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(in + base + u * 256 + threadIdx.x),
                                         (__attribute__((address_space(3))) void *)&sb[u * 256 + wave * 64], 16, 0, AUX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(io + base + u * 256 + threadIdx.x, sa[u * 256 + threadIdx.x] + sb[u * 256 + threadIdx.x]);
}

// the product's LDS-DMA kernel with the 16-byte stores' cache policy set explicitly
// (POL: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1, 4 sc0 sc1 nt, 5 sc1 nt)
template <int POL> __device__ __forceinline__ void stp(v4f *p, v4f v)
{
    if constexpr (POL == 0) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
}
template <int U, int POL>
__global__ __launch_bounds__(256) void k_ldsp(v4f *__restrict__ io, const v4f *__restrict__ in, size_t nv)
{
    __shared__ v4f stage[U * 256];
    const int wave = threadIdx.x >> 6;
    const size_t base = (size_t)blockIdx.x * U * 256;
#pragma unroll
    for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(in + base + u * 256 + threadIdx.x),
                                         (__attribute__((address_space(3))) void *)&stage[u * 256 + wave * 64], 16, 0, 2);
    v4f a[U];
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = ld<1>(io + base + u * 256 + threadIdx.x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++) stp<POL>(io + base + u * 256 + threadIdx.x, a[u] + stage[u * 256 + threadIdx.x]);
}

// persistent grid-stride with a software pipeline: the next tile's loads are issued
// before the current tile's stores
template <int U, int NTL, int NTS = 0>
__global__ __launch_bounds__(256) void k_pipe(v4f *__restrict__ io, const v4f *__restrict__ in, size_t nv)
{
    const size_t tile = (size_t)U * 256;
    const size_t ntiles = nv / tile;
    size_t t = blockIdx.x;
    if (t >= ntiles) return;
    v4f a[U], c[U];
    size_t base = t * tile + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = ld<NTL>(io + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) c[u] = ld<NTL>(in + base + u * 256);
    for (;;) {
        size_t tn = t + gridDim.x;
        v4f r[U];
#pragma unroll
        for (int u = 0; u < U; u++) r[u] = a[u] + c[u];
        const size_t cur = base;
        if (tn < ntiles) {
            base = tn * tile + threadIdx.x;
#pragma unroll
            for (int u = 0; u < U; u++) a[u] = ld<NTL>(io + base + u * 256);
#pragma unroll
            for (int u = 0; u < U; u++) c[u] = ld<NTL>(in + base + u * 256);
        }
#pragma unroll
        for (int u = 0; u < U; u++) st<NTS>(io + cur + u * 256, r[u]);
        if (tn >= ntiles) break;
        t = tn;
    }
}

// calibration streams
template <int U>
__global__ __launch_bounds__(256) void k_read(const v4f *__restrict__ in, v4f *__restrict__ sink, size_t nv)
{
    const size_t base = (size_t)blockIdx.x * U * 256 + threadIdx.x;
    v4f s = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; u++) s += ldnt(in + base + u * 256);
    if (s.x == 12345.f) sink[threadIdx.x] = s; // never true on the fill data
}
template <int U, int NTS = 0>
__global__ __launch_bounds__(256) void k_write(v4f *__restrict__ out, size_t nv)
{
    const size_t base = (size_t)blockIdx.x * U * 256 + threadIdx.x;
    const v4f v = {1.f, 2.f, 3.f, (float)threadIdx.x};
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(out + base + u * 256, v);
}
template <int U, int NTS = 0>
__global__ __launch_bounds__(256) void k_copy(v4f *__restrict__ out, const v4f *__restrict__ in, size_t nv)
{
    const size_t base = (size_t)blockIdx.x * U * 256 + threadIdx.x;
    v4f a[U];
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = ldnt(in + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(out + base + u * 256, a[u]);
}

__global__ void k_fill(v4f *p, size_t nv, float s)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x)
        p[i] = v4f{s * (float)(i & 7), s, -s, s * 0.5f};
}

int main(int argc, char **argv)
{
    const size_t n = 1ull << 26, nv = n / 4;
    const int R = argc > 2 ? atoi(argv[2]) : 4;
    const int iters = argc > 1 ? atoi(argv[1]) : 40;
    std::vector<v4f *> io(R), in(R);
    for (int r = 0; r < R; r++) {
        CHK(hipMalloc(&io[r], n * 4));
        CHK(hipMalloc(&in[r], n * 4));
    }
    v4f *sink;
    CHK(hipMalloc(&sink, 1 << 20));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    double best_us = 1e30;
    char best[96] = "";
    // launch(r): one launch on pair r; bytes = algorithmic bytes per launch
    auto run = [&](const char *name, double bytes, bool check, auto launch) {
        for (int r = 0; r < R; r++) {
            k_fill<<<2048, 256>>>(io[r], nv, 1.0f);
            k_fill<<<2048, 256>>>(in[r], nv, 2.0f);
        }
        CHK(hipDeviceSynchronize());
        launch(0); // the check: one launch on fresh data
        CHK(hipDeviceSynchronize());
        bool ok = true;
        if (check) {
            v4f h[2];
            CHK(hipMemcpy(h, io[0] + 12345, sizeof(h), hipMemcpyDeviceToHost));
            ok = fabsf(h[0].y - 3.0f) < 1e-6f && fabsf(h[0].z + 3.0f) < 1e-6f;
        }
        for (int it = 0; it < R; it++) launch(it % R); // warm
        CHK(hipEventRecord(e0));
        for (int it = 0; it < iters; it++) launch(it % R);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        double us = ms * 1000.0 / iters;
        printf("%-44s %8.1f us %8.1f GB/s %s\n", name, us, bytes / (us * 1e-6) / 1e9, ok ? "ok" : "BAD");
        fflush(stdout);
        if (check && ok && us < best_us) {
            best_us = us;
            snprintf(best, sizeof(best), "%s", name);
        }
    };
    const double B3 = 3.0 * n * 4, B2 = 2.0 * n * 4, B1 = 1.0 * n * 4;
    char nm[96];
#define TILE(U, BS, X, NL, NS)                                                                              \
    snprintf(nm, sizeof(nm), "tile U%d bs%d xcd%d ntl%d nts%d", U, BS, X, NL, NS);                         \
    run(nm, B3, true, [&](int r) { k_tile<U, BS, X, NL, NS><<<(unsigned)(nv / (U * BS)), BS>>>(io[r], in[r], nv); });
#define LDS(U, X, AUX)                                                                                      \
    snprintf(nm, sizeof(nm), "lds U%d xcd%d aux%d", U, X, AUX);                                            \
    run(nm, B3, true, [&](int r) { k_lds<U, X, AUX><<<(unsigned)(nv / (U * 256)), 256>>>(io[r], in[r], nv); });
#define PIPE(U, NL, G)                                                                                      \
    snprintf(nm, sizeof(nm), "pipe U%d ntl%d grid%d", U, NL, G);                                           \
    run(nm, B3, true, [&](int r) { k_pipe<U, NL><<<G, 256>>>(io[r], in[r], nv); });

#define LDSS(U, X, AUX, NS)                                                                                 \
    snprintf(nm, sizeof(nm), "lds U%d xcd%d aux%d nts%d", U, X, AUX, NS);                                  \
    run(nm, B3, true, [&](int r) { k_lds<U, X, AUX, NS><<<(unsigned)(nv / (U * 256)), 256>>>(io[r], in[r], nv); });
    if (argc > 3 && argv[3][0] == 'g') { // nt-store calibration and persistent / pipelined grids
        for (int rep = 0; rep < 2; rep++) {
            run("read-only U4 (1 stream)", B1, false, [&](int r) { k_read<4><<<(unsigned)(nv / 1024), 256>>>(in[r], sink, nv); });
            run("write-only U4 (1 stream)", B1, false, [&](int r) { k_write<4><<<(unsigned)(nv / 1024), 256>>>(io[r], nv); });
            run("write-only U4 nt (1 stream)", B1, false, [&](int r) { k_write<4, 1><<<(unsigned)(nv / 1024), 256>>>(io[r], nv); });
            run("copy U4 nt-store (2 streams)", B2, false, [&](int r) { k_copy<4, 1><<<(unsigned)(nv / 1024), 256>>>(io[r], in[r], nv); });
            TILE(4, 256, 0, 1, 1)
            LDSS(4, 0, 2, 1)
            for (int G : {1024, 2048, 4096, 8192, 16384}) {
                snprintf(nm, sizeof(nm), "pipe U4 ntl1 nts1 grid%d", G);
                run(nm, B3, true, [&](int r) { k_pipe<4, 1, 1><<<G, 256>>>(io[r], in[r], nv); });
                snprintf(nm, sizeof(nm), "pipe U2 ntl1 nts1 grid%d", G);
                run(nm, B3, true, [&](int r) { k_pipe<2, 1, 1><<<G, 256>>>(io[r], in[r], nv); });
            }
        }
        printf("BEST %s %.1f us %.1f GB/s\n", best, best_us, B3 / (best_us * 1e-6) / 1e9);
        return 0;
    }
    if (argc > 3 && argv[3][0] == 'x') { // both operands by LDS DMA; explicit store policies
        for (int rep = 0; rep < 3; rep++) {
            LDSS(4, 0, 2, 1) // the product's kernel
#define LDS2(U, AUX, NS)                                                                                    \
    snprintf(nm, sizeof(nm), "lds2 U%d aux%d nts%d", U, AUX, NS);                                          \
    run(nm, B3, true, [&](int r) { k_lds2<U, AUX, NS><<<(unsigned)(nv / (U * 256)), 256>>>(io[r], in[r], nv); });
#define LDSP(U, POL)                                                                                        \
    snprintf(nm, sizeof(nm), "lds U%d store-policy %d", U, POL);                                           \
    run(nm, B3, true, [&](int r) { k_ldsp<U, POL><<<(unsigned)(nv / (U * 256)), 256>>>(io[r], in[r], nv); });
            LDS2(2, 2, 1)
            LDS2(4, 2, 1)
            LDS2(4, 0, 1)
            LDS2(8, 2, 1)
            LDSP(4, 0)
            LDSP(4, 1)
            LDSP(4, 2)
            LDSP(4, 3)
            LDSP(4, 4)
            LDSP(4, 5)
        }
        printf("BEST %s %.1f us %.1f GB/s\n", best, best_us, B3 / (best_us * 1e-6) / 1e9);
        return 0;
    }
    if (argc > 3 && argv[3][0] == 'f') { // focused: nt stores, three repetitions each
        for (int rep = 0; rep < 3; rep++) {
            TILE(2, 256, 0, 1, 1)
            TILE(4, 256, 0, 1, 1)
            TILE(1, 256, 0, 1, 1)
            TILE(2, 256, 1, 1, 1)
            TILE(2, 512, 0, 1, 1)
            TILE(8, 256, 0, 1, 1)
            TILE(2, 256, 0, 1, 0)
            LDSS(2, 0, 0, 1)
            LDSS(2, 0, 2, 1)
            LDSS(4, 0, 0, 1)
            LDSS(4, 0, 2, 1)
            LDSS(2, 0, 0, 0)
            run("copy U2 nt-store (2 streams)", B2, false, [&](int r) { k_copy<2, 1><<<(unsigned)(nv / 512), 256>>>(io[r], in[r], nv); });
        }
        printf("BEST %s %.1f us %.1f GB/s\n", best, best_us, B3 / (best_us * 1e-6) / 1e9);
        return 0;
    }
    // calibration
    run("read-only U4 (1 stream)", B1, false, [&](int r) { k_read<4><<<(unsigned)(nv / 1024), 256>>>(in[r], sink, nv); });
    run("write-only U4 (1 stream)", B1, false, [&](int r) { k_write<4><<<(unsigned)(nv / 1024), 256>>>(io[r], nv); });
    run("copy U2 (2 streams)", B2, false, [&](int r) { k_copy<2><<<(unsigned)(nv / 512), 256>>>(io[r], in[r], nv); });
    run("copy U4 (2 streams)", B2, false, [&](int r) { k_copy<4><<<(unsigned)(nv / 1024), 256>>>(io[r], in[r], nv); });
    run("hipMemcpyD2D (2 streams)", B2, false,
        [&](int r) { CHK(hipMemcpyAsync(io[r], in[r], n * 4, hipMemcpyDeviceToDevice, 0)); });
    // reduce variants
    TILE(2, 256, 0, 1, 0)  // the product's segment kernel
    TILE(2, 256, 1, 1, 0)
    TILE(2, 256, 0, 0, 0)
    TILE(2, 256, 0, 1, 1)
    TILE(2, 256, 0, 0, 1)
    TILE(1, 256, 0, 1, 0)
    TILE(4, 256, 0, 1, 0)
    TILE(4, 256, 1, 1, 0)
    TILE(8, 256, 0, 1, 0)
    TILE(4, 128, 0, 1, 0)
    TILE(2, 512, 0, 1, 0)
    TILE(4, 512, 0, 1, 0)
    TILE(1, 1024, 0, 1, 0)
    LDS(2, 0, 2)  // the product's LDS-DMA kernel (nt)
    LDS(2, 0, 0)
    LDS(2, 1, 2)
    LDS(4, 0, 2)
    LDS(4, 1, 2)
    LDS(8, 0, 2)
    for (int G : {1024, 2048, 4096, 8192}) {
        PIPE(2, 1, G)
        PIPE(4, 1, G)
    }
    printf("BEST %s %.1f us %.1f GB/s\n", best, best_us, B3 / (best_us * 1e-6) / 1e9);
    return 0;
}
