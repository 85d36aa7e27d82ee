// sync_probe.hip -- cost of one schedule step's device round trip on MI355X:
// launch a segment-sized kernel, record a marker event, spin on hipEventQuery (what
// ftar_drain does), for three marker kinds:
//   fenced   : default event (system-scope release + invalidate), the library's choice
//   nofence  : hipEventDisableSystemFence
//   nomarker : spin on hipStreamQuery
// and two kernels: a 1-workgroup no-op and a 64 MiB copy (dirty L2 at the marker).
//   hipcc --offload-arch=gfx950 -O3 -o sync_probe tools/sync_probe.hip && ./sync_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CHK(x)                                                                                              \
    do {                                                                                                    \
        hipError_t err_ = (x);                                                                                 \
        if (err_ != hipSuccess) {                                                                            \
            printf("%s: %s\n", #x, hipGetErrorString(err_));                                                   \
            return 1;                                                                                       \
        }                                                                                                   \
    } while (0)

__global__ void noop(int *p)
{
    if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

__global__ void copy(uint4 *__restrict__ o, const uint4 *__restrict__ i, size_t n)
{
    size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) o[k] = i[k];
}

int main()
{
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t fenced, nofence;
    CHK(hipEventCreateWithFlags(&fenced, hipEventDisableTiming));
    CHK(hipEventCreateWithFlags(&nofence, hipEventDisableTiming | hipEventDisableSystemFence));
    size_t bytes = 64u << 20, nv = bytes / 16;
    uint4 *a, *b;
    int *flag;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&b, bytes));
    CHK(hipMalloc(&flag, 64));
    CHK(hipMemset(a, 1, bytes));
    CHK(hipMemset(flag, 0, 64));
    CHK(hipDeviceSynchronize());
    const char *kname[2] = {"noop", "copy64MiB"};
    const char *mname[3] = {"fenced", "nofence", "nomarker"};
    for (int k = 0; k < 2; k++)
        for (int m = 0; m < 3; m++) {
            const int iters = 400;
            double tot = 0;
            for (int it = -20; it < iters; it++) {
                auto t0 = std::chrono::steady_clock::now();
                if (k == 0) hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s, flag);
                else hipLaunchKernelGGL(copy, dim3((unsigned)(nv / 256)), dim3(256), 0, s, b, a, nv);
                if (m < 2) {
                    hipEvent_t e = m == 0 ? fenced : nofence;
                    CHK(hipEventRecord(e, s));
                    while (hipEventQuery(e) == hipErrorNotReady) {
                    }
                } else {
                    while (hipStreamQuery(s) == hipErrorNotReady) {
                    }
                }
                auto t1 = std::chrono::steady_clock::now();
                if (it >= 0) tot += std::chrono::duration<double, std::micro>(t1 - t0).count();
            }
            printf("{\"kernel\": \"%s\", \"marker\": \"%s\", \"us_per_round_trip\": %.2f}\n", kname[k], mname[m],
                   tot / iters);
        }
    return 0;
}
