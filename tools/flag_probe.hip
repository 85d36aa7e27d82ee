// flag_probe.hip -- how fast can the host learn that a short step kernel finished?
// ("Per-call fixed cost").  One process, one GPU:
//   event      : kernel, fenced marker event (system-scope release + invalidate), spin on
//                hipEventQuery -- what ftar_drain does today
//   flag       : the kernel itself signals: every workgroup, after its stores, runs a
//                system-scope release (write-back of its XCD's L2) and adds to a counter;
//                the last one stores a flag word into pinned host memory, the host spins
//                on that word (no marker packet, no runtime call in the wait)
//   writevalue : kernel, then hipStreamWriteValue32 of the flag into pinned host memory
// for kernels of 1, 4 and 64 workgroups copying 16 KiB each, plus the host-side price of
// the runtime calls a small Allreduce makes.
//   hipcc --offload-arch=gfx950 -O3 -o flag_probe tools/flag_probe.hip && ./flag_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CHK(x)                                                                                              \
    do {                                                                                                    \
        hipError_t err_ = (x);                                                                              \
        if (err_ != hipSuccess) {                                                                           \
            printf("%s: %s\n", #x, hipGetErrorString(err_));                                                \
            return 1;                                                                                       \
        }                                                                                                   \
    } while (0)

// 256 threads x 16 B x 4 = 16 KiB per workgroup
__global__ void copy_plain(uint4 *__restrict__ o, const uint4 *__restrict__ i)
{
    size_t b = (size_t)blockIdx.x * 1024;
    for (int k = 0; k < 4; k++) o[b + k * 256 + threadIdx.x] = i[b + k * 256 + threadIdx.x];
}

__global__ void copy_flag(uint4 *__restrict__ o, const uint4 *__restrict__ i, unsigned *cnt, unsigned *flag,
                          unsigned tag)
{
    size_t b = (size_t)blockIdx.x * 1024;
    for (int k = 0; k < 4; k++) o[b + k * 256 + threadIdx.x] = i[b + k * 256 + threadIdx.x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); // system scope: this XCD's dirty lines to HBM
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(flag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t fenced, plain;
    CHK(hipEventCreateWithFlags(&fenced, hipEventDisableTiming));
    CHK(hipEventCreateWithFlags(&plain, hipEventDisableSystemFence));
    const size_t bytes = 64u * 16384;
    uint4 *a, *b;
    unsigned *cnt, *hflag, *dflag;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&b, bytes));
    CHK(hipMalloc(&cnt, 64));
    CHK(hipMemset(a, 1, bytes));
    CHK(hipMemset(cnt, 0, 64));
    CHK(hipHostMalloc(&hflag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CHK(hipHostGetDevicePointer((void **)&dflag, hflag, 0));
    *(volatile unsigned *)hflag = 0;
    CHK(hipDeviceSynchronize());
    const int iters = 400;
    unsigned tag = 0;
    printf("{\"probe\": \"flag_probe\", \"dflag_eq_hflag\": %d, \"rows\": [\n", dflag == hflag);
    const unsigned grids[3] = {1, 4, 64};
    bool first = true;
    for (unsigned g : grids)
        for (int m = 0; m < 3; m++) {
            double tot = 0, tlaunch = 0;
            for (int it = -20; it < iters; it++) {
                double t0 = now_us(), t1;
                if (m == 1) {
                    ++tag;
                    hipLaunchKernelGGL(copy_flag, dim3(g), dim3(256), 0, s, b, a, cnt, dflag, tag);
                    t1 = now_us();
                    while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != tag) {
                    }
                } else {
                    hipLaunchKernelGGL(copy_plain, dim3(g), dim3(256), 0, s, b, a);
                    t1 = now_us();
                    if (m == 0) {
                        CHK(hipEventRecord(fenced, s));
                        while (hipEventQuery(fenced) == hipErrorNotReady) {
                        }
                    } else {
                        ++tag;
                        CHK(hipStreamWriteValue32(s, dflag, tag, 0));
                        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != tag) {
                        }
                    }
                }
                double t2 = now_us();
                if (it >= 0) {
                    tot += t2 - t0;
                    tlaunch += t1 - t0;
                }
            }
            static const char *mn[3] = {"event", "flag", "writevalue"};
            printf("%s{\"workgroups\": %u, \"mode\": \"%s\", \"us_round_trip\": %.2f, \"us_launch_call\": %.2f}\n",
                   first ? "" : ",", g, mn[m], tot / iters, tlaunch / iters);
            first = false;
        }
    CHK(hipStreamSynchronize(s));
    // host-side price of the runtime calls one small Allreduce makes
    {
        hipPointerAttribute_t at;
        hipDeviceptr_t base;
        size_t sz;
        unsigned long long bid;
        double t0 = now_us();
        for (int k = 0; k < 2000; k++) (void)hipPointerGetAttributes(&at, a);
        double t1 = now_us();
        for (int k = 0; k < 2000; k++) (void)hipMemGetAddressRange(&base, &sz, (hipDeviceptr_t)a);
        double t2 = now_us();
        for (int k = 0; k < 2000; k++) (void)hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)a);
        double t3 = now_us();
        for (int k = 0; k < 2000; k++) {
            (void)hipEventRecord(plain, s);
            (void)hipStreamWaitEvent(s, plain, 0);
        }
        double t4 = now_us();
        for (int k = 0; k < 2000; k++) (void)hipStreamQuery(s);
        double t5 = now_us();
        for (int k = 0; k < 2000; k++) (void)hipSetDevice(0);
        double t6 = now_us();
        CHK(hipStreamSynchronize(s));
        printf(",{\"host_us\": {\"hipPointerGetAttributes\": %.3f, \"hipMemGetAddressRange\": %.3f, "
               "\"hipPointerGetAttribute_buffer_id\": %.3f, \"hipEventRecord+hipStreamWaitEvent\": %.3f, "
               "\"hipStreamQuery_idle\": %.3f, \"hipSetDevice\": %.3f}}\n",
               (t1 - t0) / 2000, (t2 - t1) / 2000, (t3 - t2) / 2000, (t4 - t3) / 2000, (t5 - t4) / 2000,
               (t6 - t5) / 2000);
    }
    printf("]}\n");
    return 0;
}
