// nullq_probe.hip -- how the runtime reports a caller's stream (here the null stream) idle,
// which decides how ftar orders its work after the caller's (fdev_order_after):
// the query's price on a never-used null stream, and how many queries still say "not
// ready" after a kernel on it has completed (the lag that made a queued cross-stream wait
// re-queue itself on every call).
//   hipcc --offload-arch=gfx950 -O2 -o tools/_build/nullq_probe tools/nullq_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
__global__ void k(float *p) { p[threadIdx.x] = threadIdx.x; }
static void probe(const char *what, hipStream_t mine)
{
    int notready = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) {
        hipError_t e = hipStreamQuery(nullptr);
        if (e == hipErrorNotReady) notready++;
        else if (e != hipSuccess) { printf("err %d\n", (int)e); (void)hipGetLastError(); }
    }
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 1000;
    printf("%-48s notready %4d / 1000, %.2f us per query\n", what, notready, us);
}
__global__ void spin(unsigned long long t) { auto t0 = wall_clock64(); while (wall_clock64() - t0 < t) __builtin_amdgcn_s_sleep(8); }
int main()
{
    float *p;
    if (hipMalloc(&p, 4096) != hipSuccess) return 1;
    hipStream_t mine;
    if (hipStreamCreateWithFlags(&mine, hipStreamNonBlocking) != hipSuccess) return 1;
    probe("fresh process", mine);
    k<<<1, 64>>>(p); // like torch.rand on the null stream, no sync
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    probe("after a null-stream kernel (done, unsynced)", mine);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, mine, 100000000ull); // 1 s busy on OUR non-blocking stream
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    probe("... while our non-blocking stream is busy", mine);
    (void)hipStreamSynchronize(mine);
    (void)hipDeviceSynchronize();
    probe("after hipDeviceSynchronize", mine);
    k<<<1, 64>>>(p);
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    probe("after another null-stream kernel (unsynced)", mine);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, mine, 100000000ull);
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    probe("... while our non-blocking stream is busy (2)", mine);
    (void)hipDeviceSynchronize();
    return 0;
}
