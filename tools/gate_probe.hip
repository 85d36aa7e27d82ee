// gate_probe.hip -- the product's gated launch (ftar_kernels.h KSignal gate, DESIGN.md 6
// "Launches queued ahead of their barrier") on its own, one process, one GPU, built against
// the product's segment kernel (fault-tolerant_amd/csrc/ftar_kernels.hip):
//   latency   : a short signalled copy launched after a simulated 30 us barrier (launch ->
//               completion flag) vs the same copy queued before it behind a gate (gate opened
//               -> completion flag): the part of a small call's step the gate hides
//   go / skip : a gate opened as go copies, one opened as skip leaves the output untouched;
//               both raise the completion flag
//   timeout   : a gate never opened: after gate_ticks the workgroups give up (no copy), the
//               timeout word holds the gate's value and the flag is raised -- no hang
//   overtaken : a gate whose word already holds a later sequence when its workgroups look
//               (they started late): skip + the timeout word, never a blind run
//   staged    : the staging phase ahead of the gate -- the staged data is there and signalled
//               before the gate opens, the gated work only after
// Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I fault-tolerant_amd/csrc tools/gate_probe.hip \
//         fault-tolerant_amd/csrc/ftar_kernels.hip -o tools/_build/gate_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "ftar_kernels.h"

#define CHK(x)                                                                                              \
    do {                                                                                                    \
        hipError_t err_ = (x);                                                                              \
        if (err_ != hipSuccess) {                                                                           \
            printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(err_));                               \
            return 1;                                                                                       \
        }                                                                                                   \
    } while (0)

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

// keeps the stream busy for ~`ns` nanoseconds of device wall clock (delays a later launch)
__global__ void busy_kernel(unsigned long long ticks)
{
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

struct Probe {
    unsigned *cnt = nullptr, *sig = nullptr;
    unsigned tag = 0;
    hipStream_t st = nullptr;
    unsigned *gate(unsigned seq) { return sig + 16 + seq % ftar::kGateSlots; }
    unsigned *err() { return sig + 32; }
    void wait_flag(unsigned t)
    {
        while ((int)(__atomic_load_n(sig, __ATOMIC_ACQUIRE) - t) < 0) {
        }
    }
};

// one signalled copy launch of n floats (the product's planner and kernel); gate = nullptr:
// not gated
static hipError_t launch_copy(Probe &P, float *dst, const float *src, size_t n, unsigned seq, bool gated,
                              unsigned long long ticks)
{
    ftar::SegIn in{ftar::kCopy, dst, src, nullptr, n, nullptr};
    ftar::KSegList L;
    unsigned grid = ftar::plan_segments(&in, 1, 4, 1 << 20, &L);
    L.nt_store = 1;
    L.sig = ftar::KSignal{P.cnt, P.sig, ++P.tag, 1u, gated ? P.gate(seq) : nullptr, 2u * seq, P.err(), ticks};
    return ftar::launch_segments(ftar::kFloat32, ftar::kSum, L, grid, P.st);
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main()
{
    Probe P;
    int khz = 0;
    CHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const unsigned long long tick_per_us = (unsigned long long)khz / 1000ull;
    const size_t n = 16 * 4096; // 256 KiB: 16 workgroups of the segment kernel
    float *src, *dst;
    CHK(hipMalloc(&src, n * 4));
    CHK(hipMalloc(&dst, n * 4));
    CHK(hipMalloc(&P.cnt, 256));
    CHK(hipMemset(P.cnt, 0, 256));
    CHK(hipHostMalloc((void **)&P.sig, 256, hipHostMallocCoherent | hipHostMallocMapped));
    memset(P.sig, 0, 256);
    CHK(hipStreamCreateWithFlags(&P.st, hipStreamNonBlocking));
    std::vector<float> h(n);
    for (size_t i = 0; i < n; i++) h[i] = (float)i;
    CHK(hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice));
    const unsigned long long gate_ticks = 60ull * 1000000ull * tick_per_us;
    unsigned seq = 0;

    // latency: 200 calls each way
    std::vector<double> plain, gated;
    for (int it = 0; it < 220; it++) {
        auto b0 = clk::now(); // the barrier: 30 us of host time
        while (us_since(b0) < 30.0) {
        }
        auto t0 = clk::now();
        CHK(launch_copy(P, dst, src, n, 0, false, 0));
        P.wait_flag(P.tag);
        if (it >= 20) plain.push_back(us_since(t0));
    }
    for (int it = 0; it < 220; it++) {
        ++seq;
        CHK(launch_copy(P, dst, src, n, seq, true, gate_ticks)); // queued before the barrier
        auto b0 = clk::now();
        while (us_since(b0) < 30.0) {
        }
        auto t0 = clk::now();
        __atomic_store_n(P.gate(seq), 2u * seq, __ATOMIC_RELEASE); // go
        P.wait_flag(P.tag);
        if (it >= 20) gated.push_back(us_since(t0));
    }
    bool lat_ok = __atomic_load_n(P.err(), __ATOMIC_ACQUIRE) == 0;

    // go / skip
    CHK(hipMemset(dst, 0, n * 4));
    CHK(hipDeviceSynchronize());
    ++seq;
    CHK(launch_copy(P, dst, src, n, seq, true, gate_ticks));
    __atomic_store_n(P.gate(seq), 2u * seq + 1u, __ATOMIC_RELEASE); // skip
    P.wait_flag(P.tag);
    CHK(hipStreamSynchronize(P.st));
    std::vector<float> o(n);
    CHK(hipMemcpy(o.data(), dst, n * 4, hipMemcpyDeviceToHost));
    bool skip_ok = std::all_of(o.begin(), o.end(), [](float v) { return v == 0.f; });
    ++seq;
    CHK(launch_copy(P, dst, src, n, seq, true, gate_ticks));
    __atomic_store_n(P.gate(seq), 2u * seq, __ATOMIC_RELEASE); // go
    P.wait_flag(P.tag);
    CHK(hipStreamSynchronize(P.st));
    CHK(hipMemcpy(o.data(), dst, n * 4, hipMemcpyDeviceToHost));
    bool go_ok = o == h;

    // timeout: never opened, 100 ms
    CHK(hipMemset(dst, 0, n * 4));
    CHK(hipDeviceSynchronize());
    ++seq;
    auto t0 = clk::now();
    CHK(launch_copy(P, dst, src, n, seq, true, 100000ull * tick_per_us));
    P.wait_flag(P.tag);
    double timeout_ms = us_since(t0) / 1e3;
    CHK(hipStreamSynchronize(P.st));
    unsigned terr = __atomic_exchange_n(P.err(), 0u, __ATOMIC_ACQ_REL);
    CHK(hipMemcpy(o.data(), dst, n * 4, hipMemcpyDeviceToHost));
    bool timeout_ok = terr == 2u * seq && std::all_of(o.begin(), o.end(), [](float v) { return v == 0.f; });

    // overtaken: the workgroups start 20 ms late and find a later sequence in their slot
    ++seq;
    hipLaunchKernelGGL(busy_kernel, dim3(1), dim3(64), 0, P.st, 20000ull * tick_per_us);
    CHK(launch_copy(P, dst, src, n, seq, true, gate_ticks));
    __atomic_store_n(P.gate(seq), 2u * (seq + ftar::kGateSlots), __ATOMIC_RELEASE);
    P.wait_flag(P.tag);
    CHK(hipStreamSynchronize(P.st));
    unsigned oerr = __atomic_exchange_n(P.err(), 0u, __ATOMIC_ACQ_REL);
    CHK(hipMemcpy(o.data(), dst, n * 4, hipMemcpyDeviceToHost));
    bool overtaken_ok = oerr == 2u * seq && std::all_of(o.begin(), o.end(), [](float v) { return v == 0.f; });

    // staged: the launch first stages n floats (into pinned host memory here, so the host can
    // look without a runtime call) and raises the flag with the staging tag, then waits at
    // its gate; the host sees the staged data before it opens the gate
    float *hstage = nullptr, *hdst = nullptr; // both pinned: the host looks without a runtime call
    CHK(hipHostMalloc((void **)&hstage, n * 4, hipHostMallocCoherent | hipHostMallocMapped));
    CHK(hipHostMalloc((void **)&hdst, n * 4, hipHostMallocCoherent | hipHostMallocMapped));
    memset(hstage, 0, n * 4);
    memset(hdst, 0, n * 4);
    CHK(hipDeviceSynchronize());
    ++seq;
    {
        ftar::SegIn in{ftar::kCopy, hdst, src, nullptr, n, nullptr};
        ftar::KSegList L;
        unsigned grid = ftar::plan_segments(&in, 1, 4, 1 << 20, &L);
        L.nt_store = 1;
        const unsigned stage_tag = ++P.tag;
        L.sig = ftar::KSignal{P.cnt, P.sig, ++P.tag, 1u, P.gate(seq), 2u * seq, P.err(), gate_ticks, nullptr, nullptr,
                              src, hstage, n, 4u, stage_tag, P.cnt + 16};
        CHK(ftar::launch_segments(ftar::kFloat32, ftar::kSum, L, grid, P.st));
        P.wait_flag(stage_tag);
    }
    bool staged_before_gate = memcmp(hstage, h.data(), n * 4) == 0;
    bool gated_not_run = std::all_of(hdst, hdst + n, [](float v) { return v == 0.f; }); // still at its gate
    __atomic_store_n(P.gate(seq), 2u * seq, __ATOMIC_RELEASE);
    P.wait_flag(P.tag);
    CHK(hipStreamSynchronize(P.st));
    bool staged_ok = staged_before_gate && gated_not_run && memcmp(hdst, h.data(), n * 4) == 0;

    printf("{\"tool\": \"gate_probe\", \"bytes\": %zu, \"workgroups\": 16, \"barrier_us\": 30, "
           "\"launch_after_barrier_to_flag_us\": %.2f, \"gate_open_to_flag_us\": %.2f, \"hidden_us\": %.2f, "
           "\"latency_runs_ok\": %s, \"go_ok\": %s, \"skip_ok\": %s, \"timeout_ok\": %s, \"timeout_ms\": %.1f, "
           "\"overtaken_ok\": %s, \"staged_ok\": %s, \"ok\": %s}\n",
           n * 4, median(plain), median(gated), median(plain) - median(gated), lat_ok ? "true" : "false",
           go_ok ? "true" : "false", skip_ok ? "true" : "false", timeout_ok ? "true" : "false", timeout_ms,
           overtaken_ok ? "true" : "false", staged_ok ? "true" : "false",
           (lat_ok && go_ok && skip_ok && timeout_ok && overtaken_ok && staged_ok) ? "true" : "false");
    return (lat_ok && go_ok && skip_ok && timeout_ok && overtaken_ok && staged_ok) ? 0 : 1;
}
