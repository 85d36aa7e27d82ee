// reduce_sweep.hip -- tuning sweep for the streaming local-reduce (out = x + y, fp32,
// 2 x 256 MiB) on one MI355X: work mapping, unroll, block size, grid size,
// non-temporal loads/stores, LDS-DMA staging.  Prints one line per config:
//   name  kernel_us  GB/s(3 streams)  ok
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/reduce_sweep.hip -o build/reduce_sweep
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

__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

typedef float v4f __attribute__((ext_vector_type(4)));
template <bool NT> __device__ __forceinline__ float4 ld(const float4 *p)
{
    if constexpr (NT) {
        v4f v = __builtin_nontemporal_load((const v4f *)p);
        return make_float4(v.x, v.y, v.z, v.w);
    } else return *p;
}
template <bool NT> __device__ __forceinline__ void st(float4 *p, float4 v)
{
    if constexpr (NT) {
        v4f w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, (v4f *)p);
    } else *p = v;
}

// grid-stride, U independent vectors per thread per iteration
template <int U, bool NTL, bool NTS>
__global__ void k_gs(float4 *__restrict__ io, const float4 *__restrict__ in, size_t nv)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < nv; i += U * stride) {
        float4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; u++) a[u] = ld<NTL>(io + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; u++) b[u] = ld<NTL>(in + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; u++) st<NTS>(io + i + u * stride, add4(a[u], b[u]));
    }
    for (; i < nv; i += stride) st<NTS>(io + i, add4(ld<NTL>(io + i), ld<NTL>(in + i)));
}

// block-contiguous: block b owns [b*chunk, (b+1)*chunk); inner step = blockDim*U
template <int U, bool NTL, bool NTS>
__global__ void k_bc(float4 *__restrict__ io, const float4 *__restrict__ in, size_t nv, size_t chunk)
{
    size_t beg = (size_t)blockIdx.x * chunk;
    size_t end = beg + chunk < nv ? beg + chunk : nv;
    const size_t bs = blockDim.x;
    size_t i = beg + threadIdx.x;
    for (; i + (U - 1) * bs < end; i += U * bs) {
        float4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; u++) a[u] = ld<NTL>(io + i + u * bs);
#pragma unroll
        for (int u = 0; u < U; u++) b[u] = ld<NTL>(in + i + u * bs);
#pragma unroll
        for (int u = 0; u < U; u++) st<NTS>(io + i + u * bs, add4(a[u], b[u]));
    }
    for (; i < end; i += bs) st<NTS>(io + i, add4(ld<NTL>(io + i), ld<NTL>(in + i)));
}

// LDS-DMA: `in` staged HBM->LDS by global_load_lds_dwordx4, io in registers
template <int U>
__global__ void k_lds(float4 *__restrict__ io, const float4 *__restrict__ in, size_t nv)
{
    __shared__ float4 stage[U * 256];
    const int wave = threadIdx.x >> 6;
    const size_t tile = (size_t)U * 256;
    for (size_t base = (size_t)blockIdx.x * tile; base < nv; base += (size_t)gridDim.x * tile) {
        if (base + tile <= nv) {
            float4 a[U];
#pragma unroll
            for (int u = 0; u < U; u++)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(in + base + u * 256 + threadIdx.x),
                                                 (__attribute__((address_space(3))) void *)&stage[u * 256 + wave * 64], 16, 0, 0);
#pragma unroll
            for (int u = 0; u < U; u++) a[u] = io[base + u * 256 + threadIdx.x];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int u = 0; u < U; u++) io[base + u * 256 + threadIdx.x] = add4(a[u], stage[u * 256 + threadIdx.x]);
        } else {
            for (size_t i = base + threadIdx.x; i < nv; i += 256) io[i] = add4(io[i], in[i]);
        }
    }
}

// one tile of U*BS vectors per block (the product's mapping); XCD = 1 remaps blocks so
// each XCD (blocks round-robin over 8 XCDs) streams one contiguous eighth of the data
template <int U, int BS, int XCD>
__global__ __launch_bounds__(BS) void k_tile(float4 *__restrict__ io, const float4 *__restrict__ in, size_t nv)
{
    unsigned b = blockIdx.x;
    if constexpr (XCD) {
        const unsigned per = gridDim.x / 8;
        b = (b % 8) * per + b / 8;
    }
    const size_t base = (size_t)b * U * BS + threadIdx.x;
    float4 a[U], c[U];
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = ld<true>(io + base + u * BS);
#pragma unroll
    for (int u = 0; u < U; u++) c[u] = ld<true>(in + base + u * BS);
#pragma unroll
    for (int u = 0; u < U; u++) io[base + u * BS] = add4(a[u], c[u]);
}

__global__ void k_fill(float4 *p, size_t nv, float s)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(s * (i & 7), s, -s, s * 0.5f);
}

struct Res {
    char name[96];
    float us;
};

int main(int argc, char **argv)
{
    const size_t n = 1ull << 26, nv = n / 4;
    const double bytes = 3.0 * n * 4;
    float4 *io, *in;
    CHK(hipMalloc(&io, n * 4));
    CHK(hipMalloc(&in, n * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    std::vector<Res> out;
    int iters = argc > 1 ? atoi(argv[1]) : 30;
    auto run = [&](const char *name, auto launch) {
        k_fill<<<2048, 256>>>(io, nv, 1.0f);
        k_fill<<<2048, 256>>>(in, nv, 2.0f);
        launch(); // warm
        CHK(hipDeviceSynchronize());
        // correctness of one launch on fresh data
        k_fill<<<2048, 256>>>(io, nv, 1.0f);
        launch();
        float4 h[4];
        CHK(hipMemcpy(h, io + 12345, sizeof(h), hipMemcpyDeviceToHost));
        bool ok = fabsf(h[0].y - 3.0f) < 1e-6f && fabsf(h[0].z + 3.0f) < 1e-6f;
        CHK(hipEventRecord(e0));
        for (int it = 0; it < iters; it++) launch();
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        float us = ms * 1000.f / iters;
        printf("%-48s %8.1f us %8.1f GB/s %s\n", name, us, bytes / (us * 1e-6) / 1e9, ok ? "ok" : "BAD");
        fflush(stdout);
        Res r;
        snprintf(r.name, sizeof(r.name), "%s", name);
        r.us = us;
        out.push_back(r);
    };
    char nm[96];
#define GS(U, NTL, NTS, BS, G)                                                                              \
    snprintf(nm, sizeof(nm), "gs U%d ntl%d nts%d bs%d grid%d", U, NTL, NTS, BS, G);                        \
    run(nm, [&] { k_gs<U, NTL, NTS><<<G, BS>>>(io, in, nv); });
#define BC(U, NTL, NTS, BS, G)                                                                              \
    snprintf(nm, sizeof(nm), "bc U%d ntl%d nts%d bs%d grid%d", U, NTL, NTS, BS, G);                        \
    run(nm, [&] { size_t ch = (nv + G - 1) / G; k_bc<U, NTL, NTS><<<G, BS>>>(io, in, nv, ch); });

    if (argc > 2 && argv[2][0] == 't') { // tile mapping variants (nv divisible by every tile)
#define TL(U, BS, X)                                                                                        \
    snprintf(nm, sizeof(nm), "tile U%d bs%d xcd%d", U, BS, X);                                             \
    run(nm, [&] { k_tile<U, BS, X><<<(unsigned)(nv / (U * BS)), BS>>>(io, in, nv); });
        TL(2, 256, 0)
        TL(2, 256, 1)
        TL(1, 256, 0)
        TL(4, 256, 0)
        TL(4, 256, 1)
        TL(2, 128, 0)
        TL(4, 128, 0)
        TL(2, 512, 0)
        TL(1, 512, 0)
        TL(8, 256, 0)
        TL(2, 256, 0)
        goto done;
    }
    if (argc > 2) { // focused sweep around the optimum
        for (int G : {4096, 8192, 16384, 32768}) {
            GS(4, 1, 0, 256, G)
            GS(2, 1, 0, 256, G)
            GS(8, 1, 0, 256, G)
            GS(4, 1, 0, 512, G / 2)
            BC(4, 1, 0, 256, G)
        }
        int G1 = (int)(nv / 256);
        GS(1, 1, 0, 256, G1)
        GS(1, 1, 0, 512, G1 / 2)
        GS(2, 1, 0, 256, G1 / 2)
        goto done;
    }
    for (int G : {1024, 2048, 4096, 8192}) {
        GS(1, 0, 0, 256, G)
        GS(2, 0, 0, 256, G)
        GS(4, 0, 0, 256, G)
        GS(8, 0, 0, 256, G)
        GS(4, 1, 0, 256, G)
        GS(4, 0, 1, 256, G)
        GS(4, 1, 1, 256, G)
        GS(2, 1, 1, 256, G)
        GS(4, 0, 0, 512, G / 2)
        GS(4, 0, 0, 1024, G / 4)
    }
    {
        int G = (int)(nv / 256);
        GS(1, 0, 0, 256, G)
        GS(1, 1, 1, 256, G)
        G = (int)(nv / 1024);
        GS(4, 0, 0, 256, G)
        GS(4, 1, 1, 256, G)
    }
    for (int G : {1024, 2048, 4096, 8192, 16384}) {
        BC(4, 0, 0, 256, G)
        BC(8, 0, 0, 256, G)
        BC(4, 1, 1, 256, G)
        BC(2, 1, 1, 256, G)
    }
    for (int G : {1024, 2048, 4096, 8192}) {
        snprintf(nm, sizeof(nm), "lds U4 grid%d", G);
        run(nm, [&] { k_lds<4><<<G, 256>>>(io, in, nv); });
        snprintf(nm, sizeof(nm), "lds U8 grid%d", G);
        run(nm, [&] { k_lds<8><<<G, 256>>>(io, in, nv); });
        snprintf(nm, sizeof(nm), "lds U2 grid%d", G);
        run(nm, [&] { k_lds<2><<<G, 256>>>(io, in, nv); });
    }
    // copy roofline reference: hipMemcpy D2D of 256 MiB (2 streams)
    {
        CHK(hipEventRecord(e0));
        for (int it = 0; it < iters; it++) CHK(hipMemcpyAsync(io, in, n * 4, hipMemcpyDeviceToDevice, 0));
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        float us = ms * 1000.f / iters;
        printf("%-48s %8.1f us %8.1f GB/s (2 streams)\n", "hipMemcpyD2D 256MiB", us, 2.0 * n * 4 / (us * 1e-6) / 1e9);
    }
done:
    Res best = out[0];
    for (auto &r : out)
        if (r.us < best.us) best = r;
    printf("BEST %s %.1f us %.1f GB/s\n", best.name, best.us, bytes / (best.us * 1e-6) / 1e9);
    return 0;
}
