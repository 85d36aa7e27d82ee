// ftar_dev_hip.cpp -- HIP runtime glue of libftar: device/stream setup, IPC (xGMI peer)
// mappings, segment-kernel launches with optional hipEvent timing, busy-wait sync.
//
// One process per rank.  Peer buffers are exported with hipIpcGetMemHandle and mapped
// with hipIpcOpenMemHandle(hipIpcMemLazyEnablePeerAccess); a kernel then reads a peer's
// HBM directly over xGMI ("pull"), so a dead sender can never wedge a receiver's queue.

#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "ftar_dev.h"
#include "ftar_kernels.h"

namespace {

char g_err[512];
int g_reduce_variant = 1; // LDS-DMA staged (equal or faster than 0 in every C2 run)

// A numeric FTAR_* knob of the device layer: the whole string must be a whole number in
// [lo, hi]; anything else is refused with g_err naming it (atoi would read "off" or "2k" as
// 0 or 2 without a word).
bool env_knob(const char *name, long long lo, long long hi, long long dflt, long long *out)
{
    const char *e = getenv(name);
    *out = dflt;
    if (!e) return true;
    char *end = nullptr;
    long long v = strtoll(e, &end, 10);
    if (end == e || *end != 0 || v < lo || v > hi) {
        snprintf(g_err, sizeof(g_err), "%s=%s is not a whole number in [%lld, %lld]: refused", name, e, lo, hi);
        return false;
    }
    *out = v;
    return true;
}

// The process-wide streaming knobs, read once: FTAR_NT_STORE (non-temporal 16-byte stores in
// every streaming kernel, default 1: see ftar_kernels.hip, measured on rotating buffers in
// profiles/r02) and FTAR_BLOCKS_PER_CU (grid cap, below).  -1: a value was refused.
long long g_nt = -1, g_bpc = -1;
int g_knobs = 0; // 0 unread, 1 valid, -1 refused

int process_knobs()
{
    if (g_knobs == 0)
        g_knobs = env_knob("FTAR_NT_STORE", 0, 1, 1, &g_nt) && env_knob("FTAR_BLOCKS_PER_CU", 1, 4096, 1024, &g_bpc)
                      ? 1
                      : -1;
    return g_knobs == 1 ? 0 : 13;
}

unsigned nt_store() { return g_nt == 0 ? 0u : 1u; }

int set_err(hipError_t e, const char *what)
{
    snprintf(g_err, sizeof(g_err), "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    return 101; // FTAR_ERR_DEVICE
}

#define HIPCHK(call)                                                                                        \
    do {                                                                                                    \
        hipError_t _e = (call);                                                                             \
        if (_e != hipSuccess) return set_err(_e, #call);                                                    \
    } while (0)

size_t esize_of(int dtype)
{
    switch (dtype) {
    case ftar::kInt32:
    case ftar::kFloat32: return 4;
    case ftar::kInt64:
    case ftar::kFloat64: return 8;
    default: return 0;
    }
}

// Grid cap for the streaming kernels, in 256-thread workgroups per CU.  The default
// (1024/CU = 262144 workgroups) never binds below 2 GiB per operand: every 8 KiB tile
// gets its own short-lived workgroup, the fastest mapping of the C2 sweep
// (tools/reduce_sweep.hip, profiles/).
unsigned blocks_per_cu() { return g_bpc > 0 ? (unsigned)g_bpc : 1024u; }

struct Pending {
    hipEvent_t start, stop;
    int tag;
};

// Host memory a kernel may read and write through the caller's own pointer: pinned
// (hipHostMalloc, or registered) AND mapped into the device at the same virtual address.
// Registered memory can be mapped elsewhere (its device pointer then differs), and a
// kernel using the host address would fault: such memory is treated as not shareable.
bool host_same_va(const hipPointerAttribute_t &a)
{
    return a.type == hipMemoryTypeHost && a.hostPointer && a.hostPointer == a.devicePointer;
}

// [ptr, ptr + bytes) inside ONE allocation the runtime knows (device memory, or pinned host
// memory: hipHostMalloc / hipHostRegister ranges are tracked like device allocations).  A
// range running past its allocation would be launched on and fault the GPU.
bool range_inside(const void *ptr, size_t bytes)
{
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr) != hipSuccess || !base) {
        (void)hipGetLastError();
        return false;
    }
    size_t off = (size_t)((const char *)ptr - (const char *)base);
    return off <= size && bytes <= size - off;
}

} // namespace

struct ftar_dev {
    int device;
    hipStream_t stream;
    hipStream_t bg;
    hipEvent_t fence_main; // fenced markers that sync_stream waits on
    hipEvent_t fence_bg;
    hipStream_t h2d, d2h;  // host-buffer pipeline streams (created on first use)
    hipEvent_t h2d_done[FDEV_MAX_CHUNKS], fence_d2h;
    int profiling;
    unsigned max_blocks;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
    fdev_counters ctr;
    struct { // recently exported caller allocations (a handle per allocation id)
        unsigned long long id, used;
        unsigned char handle[FDEV_HANDLE_BYTES];
    } exp[4];
    unsigned long long exp_clock;
    int export_retries;
    // Completion signals of short launches (ftar_kernels.h KSignal): a drain
    // whose stream holds only signalled launches since the previous drain waits for the
    // kernel's own flag in pinned host memory instead of a fenced marker packet.
    unsigned *sig_cnt;     // device counter of the signalling workgroups
    unsigned *sig_flag;    // pinned host word, mapped at the same address
    unsigned sig_tag;      // tag of the last signalled launch
    int flag_sync;         // FTAR_FLAG_SYNC (default 1)
    unsigned flag_max;     // FTAR_FLAG_MAX_BLOCKS: largest grid that signals (default 64)
    int unsignalled;       // main-stream launches / copies since the last drain without a signal
    int signalled;         // ... with one
    int need_acquire;      // the last drain was a signal: no marker has invalidated the caches since
    int force_fence;       // the next drain must be a fenced marker (peers read caller memory in place)
    // A launch queued ahead of its barrier (fdev_tree_batch_gated / fdev_run_gated): its
    // workgroups wait on a gate word (sig_flag[16 + seq % 8]) until fdev_gate_open; a gate
    // that timed out (or was found overtaken) is reported in its slot's word sig_flag[32 + seq % 8].
    unsigned gate_seq;     // sequence of the last gate (the word's value = 2 x seq, + 1 = skip)
    int gate_pending;      // queued, gate still closed
    int pre_gate_any;      // signalled launches queued before the gated one since the last drain ...
    unsigned pre_gate_tag; // ... the last of them
    unsigned long long gate_ticks; // wall-clock ticks before a closed gate counts as timed out
    double gate_link, gate_hbm;    // the gated launch's bytes (counted if it runs)
    int user_host_waits;           // calls that found the caller's stream busy and waited for it
    // The plan of each recent gated launch (by gate sequence parity: the one being verified
    // and the one pending), kept so that a launch whose gate timed out on the device -- its
    // workgroups returned without touching memory -- is relaunched ungated at the drain
    // (gated launches never write what they read, so running a part of one twice is harmless).
    struct GatedPlan {
        int valid, batch, dtype, op, nsrc;
        int opened; // opened as go: check its timeout word once it has completed (verify_gate)
        unsigned grid, seq;
        ftar::KSegList L;
        ftar::TreeBatch B;
        std::string tr_rw; // the launch's regions (FTAR_TRACE), for the relaunch's line
    } gp[2];
    int gate_relaunches;
    unsigned tree_unroll;          // FDEV_KNOB_TREE_UNROLL
    // Mid-size gated launches (more workgroups than signal cheaply): queued behind a fenced
    // marker (fence_pre) the drain before the barrier waits on, grid capped at big_blocks so a
    // waiting launch holds a part of the device only, the gate relayed through device words
    // (gate_dw: election words [0..7], verdict words [32..39], one per gate slot).
    hipEvent_t fence_pre;
    unsigned *gate_dw;
    unsigned big_blocks;
    int big_pending;               // the pending gated launch is a relayed (mid-size) one
    unsigned relay_min;            // FTAR_GATE_RELAY_MIN: short gated launches of this many workgroups or
                                   // more relay their gate too (one PCIe poller instead of one per workgroup)
    // FTAR_TRACE (test instrumentation, tests/fence_check.py): every launch with the regions it
    // reads and writes, its release / acquire, every fenced marker, drain, gate verdict and
    // barrier, one line each.  Off (trace == nullptr) in every measured run.
    FILE *trace;
    struct Region {
        uintptr_t base;
        size_t bytes;
        int owner;
        std::string name;
    };
    std::vector<Region> regions;
    int tr_fenced;     // note_launch recorded a fenced marker in front of the launch being traced
    int tr_drop;       // FTAR_TRACE_DROP (test-only): 1 = marker drains without their system fence, 2 = no acquires
    hipEvent_t nofence_main, nofence_bg; // the unfenced markers of tr_drop = 1
    unsigned long long tr_n;
    // fdev_peer_wait: the wait kernel's verdict words (sig_flag[48] pinned, gate_dw[48] device),
    // the host's abort word (sig_flag[49]); pw_pending: the next main-stream launch runs behind
    // the wait; pw_armed: its verdict is read after the drain
    unsigned pw_seq, pw_vval;
    int pw_pending, pw_armed;
    unsigned long long pw_launch_n;
};

extern "C" {

const char *fdev_last_error(void) { return g_err; }

int fdev_device_count(int *n)
{
    HIPCHK(hipGetDeviceCount(n));
    return 0;
}

int fdev_open(int device, ftar_dev **out)
{
    *out = nullptr;
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) {
        snprintf(g_err, sizeof(g_err), "device %d out of range (%d visible)", device, ndev);
        return 101;
    }
    // every knob checked before anything is allocated: a refused value fails the open cleanly
    long long k_sync, k_max, k_unroll, k_ms, k_relay, k_big;
    if (process_knobs() || !env_knob("FTAR_FLAG_SYNC", 0, 1, 1, &k_sync) ||
        !env_knob("FTAR_FLAG_MAX_BLOCKS", 1, 1 << 20, 64, &k_max) || !env_knob("FTAR_TREE_UNROLL", 1, 4, 1, &k_unroll) ||
        !env_knob("FTAR_GATE_TIMEOUT_MS", 1, 1ll << 40, 60000, &k_ms) ||
        !env_knob("FTAR_GATE_RELAY_MIN", 1, 1 << 20, 2, &k_relay) || !env_knob("FTAR_GATE_BIG_BLOCKS", 0, 1 << 20, 0, &k_big))
        return 13;
    if (k_unroll == 3) {
        snprintf(g_err, sizeof(g_err), "FTAR_TREE_UNROLL=3 is not 1, 2 or 4: refused");
        return 13;
    }
    HIPCHK(hipSetDevice(device));
    ftar_dev *d = new ftar_dev();
    d->device = device;
    d->profiling = 0;
    memset(d->exp, 0, sizeof(d->exp));
    d->exp_clock = 0;
    memset(&d->ctr, 0, sizeof(d->ctr));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    d->max_blocks = (unsigned)prop.multiProcessorCount * blocks_per_cu();
    if (d->max_blocks == 0) d->max_blocks = 2048;
    HIPCHK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    d->bg = nullptr; // created on first use (ensure_bg): one hardware queue less per rank
    // default (fenced) events: recording one performs a system-scope sequentially
    // consistent fence -- L2 writeback and invalidation -- see sync_stream
    HIPCHK(hipEventCreateWithFlags(&d->fence_main, hipEventDisableTiming));
    d->fence_bg = nullptr;
    {
        d->flag_sync = (int)k_sync;
        d->flag_max = (unsigned)k_max;
        d->sig_cnt = nullptr;
        d->sig_flag = nullptr;
        d->sig_tag = 0;
        d->unsignalled = d->signalled = d->need_acquire = d->force_fence = 0;
        d->gate_seq = 0;
        d->gate_pending = d->pre_gate_any = 0;
        d->user_host_waits = 0;
        d->pre_gate_tag = 0;
        d->gate_relaunches = 0;
        d->gp[0].valid = d->gp[1].valid = 0;
        d->tree_unroll = (unsigned)k_unroll;
        int khz = 0; // wall clock of the kernels (s_memrealtime), 100 MHz on CDNA
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) {
            (void)hipGetLastError();
            khz = 100000;
        }
        // FTAR_GATE_TIMEOUT_MS (default 60 s): a gate still closed this long is given up by
        // the device (the workgroups return untouched) and the launch is relaunched ungated at
        // the next drain; the host normally gives a gate up far sooner (FTAR_GATE_HOLD_US)
        d->gate_ticks = (unsigned long long)khz * (unsigned long long)k_ms;
        if (d->flag_sync) {
            HIPCHK(hipMalloc((void **)&d->sig_cnt, 256));
            HIPCHK(hipMemset(d->sig_cnt, 0, 256));
            HIPCHK(hipHostMalloc((void **)&d->sig_flag, 256, hipHostMallocCoherent | hipHostMallocMapped));
            void *dp = nullptr;
            HIPCHK(hipHostGetDevicePointer(&dp, d->sig_flag, 0));
            if (dp != (void *)d->sig_flag) { // the kernels store through the host address
                (void)hipHostFree(d->sig_flag);
                (void)hipFree(d->sig_cnt);
                d->sig_flag = nullptr;
                d->sig_cnt = nullptr;
                d->flag_sync = 0;
            } else {
                memset(d->sig_flag, 0, 256); // flag [0], gates [16..23], their timeout words [32..39]
                __atomic_store_n(d->sig_flag, 0u, __ATOMIC_RELEASE);
            }
            HIPCHK(hipDeviceSynchronize());
        }
        d->fence_pre = nullptr;
        d->gate_dw = nullptr;
        d->big_pending = 0;
        // FTAR_GATE_BIG_BLOCKS unset (0): half the CUs
        d->big_blocks = k_big > 0 ? (unsigned)k_big : (unsigned)(prop.multiProcessorCount / 2 > 0 ? prop.multiProcessorCount / 2 : 1);
        d->relay_min = (unsigned)k_relay;
        if (d->flag_sync) {
            HIPCHK(hipEventCreateWithFlags(&d->fence_pre, hipEventDisableTiming)); // fenced, see sync_stream
            HIPCHK(hipMalloc((void **)&d->gate_dw, 256));
            HIPCHK(hipMemset(d->gate_dw, 0, 256));
            HIPCHK(hipDeviceSynchronize());
        }
    }
    d->h2d = d->d2h = nullptr;
    d->fence_d2h = nullptr;
    d->trace = nullptr;
    d->tr_fenced = d->tr_drop = 0;
    d->nofence_main = d->nofence_bg = nullptr;
    d->tr_n = 0;
    d->pw_seq = d->pw_vval = 0;
    d->pw_pending = d->pw_armed = 0;
    d->pw_launch_n = 0;
    memset(d->h2d_done, 0, sizeof(d->h2d_done));
    // Peer access to every other GPU of the node: the exchanges read peers' HBM.
    for (int p = 0; p < ndev; p++) {
        if (p == device) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, device, p) == hipSuccess && can) {
            hipError_t e = hipDeviceEnablePeerAccess(p, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
        }
    }
    *out = d;
    return 0;
}

void fdev_close(ftar_dev *d)
{
    if (!d) return;
    (void)hipSetDevice(d->device);
    (void)fdev_gate_open(d, 1); // a launch still waiting on its gate returns without work
    (void)hipStreamSynchronize(d->stream);
    if (d->bg) (void)hipStreamSynchronize(d->bg);
    if (d->h2d) (void)hipStreamSynchronize(d->h2d);
    for (auto &p : d->pending) {
        (void)hipEventDestroy(p.start);
        (void)hipEventDestroy(p.stop);
    }
    for (auto e : d->event_pool) (void)hipEventDestroy(e);
    (void)hipEventDestroy(d->fence_main);
    if (d->fence_bg) (void)hipEventDestroy(d->fence_bg);
    (void)hipStreamDestroy(d->stream);
    if (d->bg) (void)hipStreamDestroy(d->bg);
    for (int i = 0; i < FDEV_MAX_CHUNKS; i++)
        if (d->h2d_done[i]) (void)hipEventDestroy(d->h2d_done[i]);
    if (d->fence_d2h) (void)hipEventDestroy(d->fence_d2h);
    if (d->h2d) (void)hipStreamDestroy(d->h2d);
    if (d->sig_cnt) (void)hipFree(d->sig_cnt);
    if (d->sig_flag) (void)hipHostFree(d->sig_flag);
    if (d->gate_dw) (void)hipFree(d->gate_dw);
    if (d->fence_pre) (void)hipEventDestroy(d->fence_pre);
    if (d->nofence_main) (void)hipEventDestroy(d->nofence_main);
    if (d->nofence_bg) (void)hipEventDestroy(d->nofence_bg);
    if (d->trace) fclose(d->trace);
    delete d;
}

int fdev_device(const ftar_dev *d) { return d->device; }

int fdev_physical_id(ftar_dev *d, char *out, size_t n)
{
    if (n < 16) return 13;
    HIPCHK(hipDeviceGetPCIBusId(out, (int)n, d->device));
    return 0;
}

// Round 1 saw one refused export (hipIpcGetMemHandle: invalid argument) when a sweep
// re-allocated the workspace at every size, and round 2's 8-rank regrowth test saw it
// once more, on a fresh 18 MiB block.  tools/ipc_probe.hip found no refusal in isolation;
// the pattern both failures share is an allocation made right after this process closed
// its imports of the peers' old blocks (ftar_ensure_workspace closed, freed, then
// allocated), so the fresh block could land on an address range an import had just
// released.  ftar_ensure_workspace now allocates and exports the new blocks while every
// old mapping is still in place.  A refusal is still handled, bounded and visible: the
// refused block is held while ONE more is tried (so the retry lands at another address),
// the event is printed and counted (ftar_stats.export_retries; tests assert it stays 0).
int fdev_alloc_shared(ftar_dev *d, size_t bytes, void **ptr, void *handle)
{
    HIPCHK(hipSetDevice(d->device));
    void *held = nullptr;
    hipError_t e = hipSuccess;
    for (int attempt = 0; attempt < 2; attempt++) {
        void *p = nullptr;
        e = hipMalloc(&p, bytes);
        if (e != hipSuccess) break;
        hipIpcMemHandle_t h;
        e = hipIpcGetMemHandle(&h, p);
        if (e == hipSuccess) {
            memcpy(handle, &h, FDEV_HANDLE_BYTES);
            *ptr = p;
            if (held) (void)hipFree(held);
            // the last FDEV_FLAG_BYTES start zeroed: the peer-wait flag of a W buffer never
            // holds a token before its owner publishes one (fdev_peer_wait)
            if (bytes >= FDEV_FLAG_BYTES) {
                HIPCHK(hipMemsetAsync((char *)p + bytes - FDEV_FLAG_BYTES, 0, FDEV_FLAG_BYTES, d->stream));
                HIPCHK(hipStreamSynchronize(d->stream));
            }
            return 0;
        }
        (void)hipGetLastError();
        fprintf(stderr, "ftar: device %d: IPC export of a fresh %zu B block at %p refused (%s)%s\n", d->device, bytes,
                p, hipGetErrorString(e), attempt ? "" : ": re-allocating");
        d->export_retries++;
        if (held) (void)hipFree(held);
        held = p;
    }
    if (held) (void)hipFree(held);
    return set_err(e, "hipMalloc + hipIpcGetMemHandle");
}

int fdev_export_retries(const ftar_dev *d) { return d->export_retries; }

int fdev_alloc_plain(ftar_dev *d, size_t bytes, void **ptr)
{
    HIPCHK(hipSetDevice(d->device));
    HIPCHK(hipMalloc(ptr, bytes));
    return 0;
}

int fdev_free(ftar_dev *d, void *ptr)
{
    if (!ptr) return 0;
    HIPCHK(hipSetDevice(d->device));
    HIPCHK(hipFree(ptr));
    return 0;
}

int fdev_import(ftar_dev *d, const void *handle, void **ptr)
{
    HIPCHK(hipSetDevice(d->device));
    hipIpcMemHandle_t h;
    memcpy(&h, handle, FDEV_HANDLE_BYTES);
    HIPCHK(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
    return 0;
}

int fdev_export_range(ftar_dev *d, const void *ptr, size_t bytes, void *handle, uint64_t *id, size_t *offset)
{
    HIPCHK(hipSetDevice(d->device));
    unsigned long long bid = 0;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    // only this device's HBM is exported; pinned host memory (which the kernels may read
    // and write in place) is staged instead
    if (hipPointerGetAttributes(&a, ptr) != hipSuccess || a.type != hipMemoryTypeDevice || a.device != d->device) {
        (void)hipGetLastError();
        return 1;
    }
    if (hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)ptr) != hipSuccess || bid == 0 ||
        hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr) != hipSuccess) {
        (void)hipGetLastError();
        return 1;
    }
    size_t off = (size_t)((const char *)ptr - (const char *)base);
    if (off + bytes > size) return 1;
    int k = 0, victim = 0;
    for (; k < 4 && d->exp[k].id != bid; k++)
        if (d->exp[k].used < d->exp[victim].used) victim = k;
    if (k == 4) {
        hipIpcMemHandle_t h;
        if (hipIpcGetMemHandle(&h, base) != hipSuccess) {
            (void)hipGetLastError();
            return 1;
        }
        k = victim;
        memcpy(d->exp[k].handle, &h, FDEV_HANDLE_BYTES);
        d->exp[k].id = bid;
    }
    d->exp[k].used = ++d->exp_clock;
    memcpy(handle, d->exp[k].handle, FDEV_HANDLE_BYTES);
    *id = bid;
    *offset = off;
    return 0;
}

int fdev_check_ptr(ftar_dev *d, const void *ptr, size_t bytes)
{
    // one attribute query per buffer and call: a cache keyed on the address would also
    // accept a freed-and-reallocated smaller block at the same address
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    if (hipPointerGetAttributes(&a, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return 1; // not memory the runtime knows (pageable host memory)
    }
    if (a.type == hipMemoryTypeUnregistered) return 1;
    if (a.type == hipMemoryTypeHost) return !host_same_va(a) || !range_inside(ptr, bytes);
    if (a.type == hipMemoryTypeDevice) {
        if (a.device != d->device) return 1; // another GPU's memory: the kernels run on ours
        if (!range_inside(ptr, bytes)) return 1; // the whole range inside one allocation
    }
    return 0;
}

int fdev_host_pinned(const void *ptr)
{
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    if (!ptr || hipPointerGetAttributes(&a, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return host_same_va(a);
}

int fdev_unimport(ftar_dev *d, void *ptr)
{
    if (!ptr) return 0;
    HIPCHK(hipSetDevice(d->device));
    HIPCHK(hipIpcCloseMemHandle(ptr));
    return 0;
}

// ---- FTAR_TRACE ---------------------------------------------------------------------------
// A launch's line: `L <n> s=<m|b> sig=<tag> rel=<0|1> acq=<0|1> fence=<0|1> gate=<seq> eng=<k|sdma>
// r=<regions read> w=<regions written> sw=<staged before the gate> stag=<tag>`, a region as
// owner:name:offset:bytes (only the registered ones: the workspaces, the exported send buffers and
// their peer mappings).  `rel` = the kernel releases its stores at system scope before it signals
// (signal_done), `acq` = it invalidates before its loads (signal_acquire), `fence` = a fenced marker
// was queued right in front of it.  tests/fence_check.py checks the cross-rank rules on the lines.
static void tr(ftar_dev *d, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static void tr(ftar_dev *d, const char *fmt, ...)
{
    if (!d->trace) return;
    va_list ap;
    va_start(ap, fmt);
    vfprintf(d->trace, fmt, ap);
    va_end(ap);
    fputc('\n', d->trace);
}

struct TrRange {
    const void *p;
    size_t n;
};

static void tr_fmt(const ftar_dev *d, const std::vector<TrRange> &v, std::string &out)
{
    char buf[160];
    for (const TrRange &r : v) {
        if (!r.p || !r.n) continue;
        const uintptr_t a = (uintptr_t)r.p;
        for (const ftar_dev::Region &g : d->regions)
            if (a >= g.base && a < g.base + g.bytes) {
                snprintf(buf, sizeof(buf), "%d:%s:%zu:%zu,", g.owner, g.name.c_str(), (size_t)(a - g.base), r.n);
                out += buf;
                break;
            }
    }
    if (out.empty()) out = "-";
}

// The regions of a launch: "r=... w=..." (the relaunch of a gated plan reuses the text)
static std::string tr_rw(const ftar_dev *d, const std::vector<TrRange> &rd, const std::vector<TrRange> &wr)
{
    if (!d->trace) return std::string();
    std::string a, b;
    tr_fmt(d, rd, a);
    tr_fmt(d, wr, b);
    return "r=" + a + " w=" + b;
}

static void tr_launch(ftar_dev *d, hipStream_t st, const ftar::KSignal *sig, const std::string &rw, unsigned gate,
                      const char *eng, const std::string &staged = std::string(), unsigned stag = 0)
{
    if (!d->trace) return;
    const bool rel = sig && sig->cnt;
    const bool acq = sig && (sig->cnt || sig->gate) && sig->acquire;
    tr(d, "L %llu s=%c sig=%u rel=%d acq=%d fence=%d gate=%u eng=%s %s sw=%s stag=%u", ++d->tr_n,
       st == d->stream ? 'm' : 'b', rel ? sig->tag : 0u, rel ? 1 : 0, acq ? 1 : 0, d->tr_fenced, gate, eng, rw.c_str(),
       staged.empty() ? "-" : staged.c_str(), stag);
    d->tr_fenced = 0;
}

static void seg_ranges(const fdev_seg *segs, int nseg, size_t es, std::vector<TrRange> &rd, std::vector<TrRange> &wr)
{
    for (int i = 0; i < nseg; i++) {
        const size_t b = segs[i].n * es;
        rd.push_back({segs[i].x, b});
        if (segs[i].kind != FDEV_COPY) rd.push_back({segs[i].y, b});
        wr.push_back({segs[i].out, b});
        wr.push_back({segs[i].out2, b});
    }
}

static void batch_ranges(const ftar::TreeBatch &B, int nsrc, size_t es, std::vector<TrRange> &rd,
                         std::vector<TrRange> &wr)
{
    for (int t = 0; t < B.nt; t++) {
        for (int j = 0; j < nsrc; j++) rd.push_back({B.t[t].src[j], B.t[t].n * es});
        wr.push_back({B.t[t].out, B.t[t].n * es});
    }
}

// The background stream exists only in ranks that use it (Raben's step-0 redundancy
// copy with a spare): every stream is a hardware queue, and ranks that share a GPU (a
// spare beside its partner, the one-GPU test box) time-slice once the device's queue
// slots run out.
static int ensure_bg(ftar_dev *d)
{
    if (d->bg) return 0;
    HIPCHK(hipStreamCreateWithFlags(&d->bg, hipStreamNonBlocking));
    // default (fenced) event: see sync_stream
    HIPCHK(hipEventCreateWithFlags(&d->fence_bg, hipEventDisableTiming));
    return 0;
}

static hipEvent_t get_event(ftar_dev *d)
{
    if (!d->event_pool.empty()) {
        hipEvent_t e = d->event_pool.back();
        d->event_pool.pop_back();
        return e;
    }
    // pooled events only time kernels and order streams of this device: no system fence
    // (the cross-GPU visibility fence is sync_stream's dedicated marker)
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

// Bookkeeping of every launch or copy on a stream of this rank.  On the main stream: a
// launch of at most flag_max workgroups that may signal gets the completion signal
// (returned in *sig).  After a signal drain no marker packet has invalidated the caches
// (need_acquire): a signalled launch then invalidates them itself, per workgroup, for its
// own loads (`acquire`; an XCD's invalidate does nothing for the others, so need_acquire
// stays set), and any other launch is preceded by a fenced marker, which invalidates them
// device-wide as the drain's marker used to and clears need_acquire.  A background-stream
// launch gets such a marker on its own stream.
static void note_launch(ftar_dev *d, hipStream_t st, unsigned grid, bool can_signal, ftar::KSignal *sig)
{
    if (sig) *sig = ftar::KSignal{};
    // anything queued behind a closed gate would wait for it: the gated launch is given up
    // (opened as skip; it returns untouched) -- its caller finds the gate no longer pending
    if (d->gate_pending) (void)fdev_gate_open(d, 1);
    d->tr_fenced = 0;
    const bool acquire = d->need_acquire && d->tr_drop != 2; // tr_drop 2: TEST-ONLY, acquires left out
    if (st != d->stream) {
        if (acquire && d->fence_bg) {
            (void)hipEventRecord(d->fence_bg, st);
            d->tr_fenced = 1;
        }
        return;
    }
    if (can_signal && sig && d->flag_sync && grid <= d->flag_max) {
        *sig = ftar::KSignal{};
        sig->cnt = d->sig_cnt;
        sig->flag = d->sig_flag;
        sig->tag = ++d->sig_tag;
        sig->acquire = (unsigned)acquire;
        d->signalled++;
    } else {
        if (acquire) {
            (void)hipEventRecord(d->fence_main, st);
            d->tr_fenced = 1;
        }
        d->need_acquire = 0;
        d->unsignalled++;
    }
}

// The kernel's view of fdev segments, and their algorithmic link / HBM bytes.
static void seg_inputs(const fdev_seg *segs, int nseg, size_t es, ftar::SegIn *in, double *link, double *hbm)
{
    for (int i = 0; i < nseg; i++) {
        in[i].kind = segs[i].kind == FDEV_COPY ? ftar::kCopy : ftar::kReduce;
        in[i].out = segs[i].out;
        in[i].x = segs[i].x;
        in[i].y = segs[i].y;
        in[i].n = segs[i].n;
        in[i].out2 = segs[i].out2;
        double b = (double)segs[i].n * (double)es;
        int nread = segs[i].kind == FDEV_COPY ? 1 : 2;
        int nremote = ((segs[i].remote & FDEV_REMOTE_X) ? 1 : 0) +
                      ((segs[i].kind != FDEV_COPY && (segs[i].remote & FDEV_REMOTE_Y)) ? 1 : 0);
        int rout = (segs[i].remote & FDEV_REMOTE_OUT) ? 1 : 0;
        *link += b * (nremote + rout);
        *hbm += b * (1 - rout + nread - nremote + (segs[i].out2 ? 1 : 0));
    }
}

// [a, a + na) and [b, b + nb) overlap
static bool overlaps(const void *a, size_t na, const void *b, size_t nb)
{
    const char *x = (const char *)a, *y = (const char *)b;
    return a && b && x < y + nb && y < x + na;
}

static int run_on(ftar_dev *d, hipStream_t st, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    size_t es = esize_of(dtype);
    if (es == 0 || op < 0 || op >= ftar::kNumOps || nseg < 0 || nseg > FDEV_MAX_SEGS || tag < 0 || tag >= FDEV_NTAGS) {
        snprintf(g_err, sizeof(g_err), "fdev_run: bad arguments");
        return 13;
    }
    ftar::SegIn in[FDEV_MAX_SEGS];
    double link = 0, hbm = 0;
    seg_inputs(segs, nseg, es, in, &link, &hbm);
    d->ctr.link_bytes += link;
    d->ctr.hbm_bytes += hbm;
    ftar::KSegList L;
    unsigned grid = ftar::plan_segments(in, nseg, es, d->max_blocks, &L);
    const bool behind_wait = d->pw_pending && st == d->stream;
    if (behind_wait) d->pw_pending = 0;
    if (grid == 0) return 0;
    L.nt_store = nt_store();
    note_launch(d, st, grid, true, &L.sig);
    if (behind_wait) {
        // behind a peer wait: the wait's verdict decides.  No acquire of its own: the fenced
        // marker in front of the flag (fdev_peer_wait) invalidated this GPU's caches after
        // everything this rank read before, and since then only the wait kernel has read peer
        // memory (the flag words, a page of their own) -- no line of what this launch reads can
        // be stale (tests/fence_check.py's acquire rule checks exactly that on the logs)
        L.sig.vword = d->gate_dw + 48;
        L.sig.vval = d->pw_vval;
        d->pw_armed = 1;
    }
    if (d->trace) {
        std::vector<TrRange> rd, wr;
        seg_ranges(segs, nseg, es, rd, wr);
        tr_launch(d, st, &L.sig, tr_rw(d, rd, wr), 0, "k");
        if (behind_wait) d->pw_launch_n = d->tr_n;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (d->profiling) {
        e0 = get_event(d);
        e1 = get_event(d);
        if (e0) (void)hipEventRecord(e0, st);
    }
    hipError_t e = ftar::launch_segments(dtype, op, L, grid, st);
    if (e != hipSuccess) return set_err(e, "segment_kernel launch");
    if (d->profiling && e0 && e1) {
        (void)hipEventRecord(e1, st);
        d->pending.push_back(Pending{e0, e1, tag});
    }
    return 0;
}

int fdev_tree(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, unsigned remote_mask, void *out,
              size_t n, int tag)
{
    return fdev_tree_out(d, dtype, op, src, nsrc, remote_mask, out, nullptr, 0, 0, n, tag);
}

int fdev_tree_out(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, unsigned remote_mask, void *out,
                  void *const *more, int nmore, int more_remote, size_t n, int tag)
{
    size_t es = esize_of(dtype);
    if (es == 0 || op < 0 || op >= ftar::kNumOps || tag < 0 || tag >= FDEV_NTAGS ||
        !(nsrc == 2 || nsrc == 4 || nsrc == 8 || nsrc == 16) || nmore < 0 || nmore > ftar::kMaxMore) {
        snprintf(g_err, sizeof(g_err), "fdev_tree: bad arguments");
        return 13;
    }
    if (n == 0) return 0;
    int nremote = __builtin_popcount(remote_mask & ((1u << nsrc) - 1));
    const int mr = more_remote ? nmore : 0; // extra destinations in peers' HBM, or in ours
    d->ctr.link_bytes += (double)n * (double)es * (nremote + mr);
    d->ctr.hbm_bytes += (double)n * (double)es * (nsrc - nremote + 1 + nmore - mr);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (d->profiling) {
        e0 = get_event(d);
        e1 = get_event(d);
        if (e0) (void)hipEventRecord(e0, d->stream);
    }
    note_launch(d, d->stream, ~0u, false, nullptr);
    if (d->trace) {
        std::vector<TrRange> rd, wr;
        for (int j = 0; j < nsrc; j++) rd.push_back({src[j], n * es});
        wr.push_back({out, n * es});
        for (int o = 0; o < nmore; o++) wr.push_back({more[o], n * es});
        tr_launch(d, d->stream, nullptr, tr_rw(d, rd, wr), 0, "k");
    }
    // pieces of at most max_blocks vector workgroups (plan_tree refuses larger bodies)
    const unsigned u = (nsrc == 4 || nsrc == 8) ? d->tree_unroll : 1u;
    const size_t piece = (size_t)d->max_blocks * 256 * u * (16 / es);
    for (size_t off = 0; off < n; off += piece) {
        ftar::TreeArgs A;
        memset(&A, 0, sizeof(A));
        for (int j = 0; j < nsrc; j++) A.src[j] = (const char *)src[j] + off * es;
        A.out = (char *)out + off * es;
        A.nmore = nmore;
        for (int o = 0; o < nmore; o++) A.more[o] = (char *)more[o] + off * es;
        A.n = n - off < piece ? n - off : piece;
        A.nt_store = nt_store();
        A.unroll = u;
        unsigned grid = ftar::plan_tree(&A, nsrc, es, d->max_blocks + 1);
        if (grid == 0) {
            snprintf(g_err, sizeof(g_err), "fdev_tree: plan failed");
            return 13;
        }
        hipError_t e = ftar::launch_tree(dtype, op, nsrc, A, grid, d->stream);
        if (e != hipSuccess) return set_err(e, "tree_kernel launch");
    }
    if (d->profiling && e0 && e1) {
        (void)hipEventRecord(e1, d->stream);
        d->pending.push_back(Pending{e0, e1, tag});
    }
    return 0;
}

// Gate words: sig_flag[16 .. 23], gate `seq` in slot seq % kGateSlots; the slot's timeout
// word sig_flag[32 + slot] (a workgroup that gave the gate up writes the gate's value).
static unsigned *gate_word(ftar_dev *d, unsigned seq) { return d->sig_flag + 16 + seq % ftar::kGateSlots; }
static unsigned *gate_err(ftar_dev *d, unsigned seq) { return d->sig_flag + 32 + seq % ftar::kGateSlots; }

// Whether a launch of `grid` workgroups may be queued behind a gate now (see
// fdev_tree_batch_gated): a fenced marker or an unsignalled launch would have to drain
// behind the closed gate, a profiled launch would time the wait.
static bool can_gate(const ftar_dev *d, unsigned grid)
{
    return d->flag_sync && !d->profiling && !d->gate_pending && !d->unsignalled && !d->force_fence && grid > 0 &&
           grid <= d->flag_max;
}

// The gate fields of a launch about to be queued gated; its bytes are counted when it runs.
static ftar::KSignal arm_gate(ftar_dev *d, double link, double hbm)
{
    d->gate_link = link;
    d->gate_hbm = hbm;
    d->pre_gate_any = d->signalled > 0;
    d->pre_gate_tag = d->sig_tag;
    d->gate_seq++;
    d->signalled++;
    __atomic_store_n(gate_err(d, d->gate_seq), 0u, __ATOMIC_RELAXED); // the slot's last gate was verified
    // the workgroups invalidate their caches once the gate opens (acquire = 1): whatever
    // the drains before it did, the peers' data is read fresh
    ftar::KSignal k{};
    k.cnt = d->sig_cnt;
    k.flag = d->sig_flag;
    k.tag = ++d->sig_tag;
    k.acquire = d->tr_drop == 2 ? 0u : 1u; // tr_drop 2: TEST-ONLY
    k.gate = gate_word(d, d->gate_seq);
    k.gate_val = 2u * d->gate_seq;
    k.err = gate_err(d, d->gate_seq);
    k.gate_ticks = d->gate_ticks;
    return k;
}

// A short gated launch of several workgroups waits with ONE of them polling the host word
// over PCIe, the others polling the device word it relays the verdict through (the relayed
// form of the mid-size launches, signal_gate): up to 64 uncached PCIe pollers per launch
// slowed the peers sharing a GPU 2x at 1 MiB (RD, 4 ranks: 194 vs 93 us ungated).
static void relay_gate(ftar_dev *d, ftar::KSignal &sig, unsigned grid)
{
    if (!d->gate_dw || grid < d->relay_min) return;
    sig.gate_poll = d->gate_dw + d->gate_seq % ftar::kGateSlots;
    sig.gate_dev = d->gate_dw + 32 + d->gate_seq % ftar::kGateSlots;
}

// Keep the plan of the gate just armed (d->gate_seq) for a relaunch: the same launch with
// no signal, gate or staging phase.
static void keep_plan(ftar_dev *d, int batch, int dtype, int op, int nsrc, unsigned grid, const ftar::KSegList *L,
                      const ftar::TreeBatch *B)
{
    ftar_dev::GatedPlan &g = d->gp[d->gate_seq & 1];
    g.valid = 1;
    g.opened = 0;
    g.batch = batch;
    g.dtype = dtype;
    g.op = op;
    g.nsrc = nsrc;
    g.grid = grid;
    g.seq = d->gate_seq;
    if (batch) {
        g.B = *B;
        g.B.sig = ftar::KSignal{};
    } else {
        g.L = *L;
        g.L.sig = ftar::KSignal{};
    }
}

// The TreeBatch of fdev_tree_batch(_gated): the grid (0 = a tree beyond the workgroup
// budget, or nothing to do when B->nt == 0), link and HBM bytes.
static int build_batch(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, const unsigned *remote_mask,
                       void *const *out, const size_t *n, int ntree, int tag, ftar::TreeBatch *B, unsigned *grid,
                       double *link, double *hbm)
{
    size_t es = esize_of(dtype);
    if (es == 0 || op < 0 || op >= ftar::kNumOps || tag < 0 || tag >= FDEV_NTAGS || ntree < 1 || ntree > ftar::kMaxBatch ||
        !(nsrc == 2 || nsrc == 4 || nsrc == 8)) {
        snprintf(g_err, sizeof(g_err), "fdev_tree_batch: bad arguments");
        return 13;
    }
    memset(B, 0, sizeof(*B));
    B->nt = 0;
    *link = *hbm = 0;
    for (int t = 0; t < ntree; t++) {
        if (n[t] == 0) continue;
        ftar::TreeArgs &A = B->t[B->nt++];
        for (int j = 0; j < nsrc; j++) A.src[j] = src[t * nsrc + j];
        A.out = out[t];
        A.n = n[t];
        A.nt_store = nt_store();
        int nremote = __builtin_popcount(remote_mask[t] & ((1u << nsrc) - 1));
        *link += (double)n[t] * (double)es * nremote;
        *hbm += (double)n[t] * (double)es * (nsrc - nremote + 1);
    }
    *grid = B->nt ? ftar::plan_tree_batch(B, nsrc, es, d->max_blocks + 1) : 0;
    return 0;
}

int fdev_tree_batch_staged_gated(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc,
                                 const unsigned *remote_mask, void *const *out, const size_t *n, int ntree, int tag,
                                 void *stage_dst, const void *stage_src, size_t stage_n, int *gated)
{
    *gated = 0;
    if (!can_gate(d, 1)) return 0;
    ftar::TreeBatch B;
    unsigned grid = 0;
    double link, hbm;
    int rc = build_batch(d, dtype, op, src, nsrc, remote_mask, out, n, ntree, tag, &B, &grid, &link, &hbm);
    if (rc) return rc;
    // a one-shot of up to 4x the signal limit's workgroups still waits at its gate: its vector
    // workgroups take several chunks each (cap_tree_batch; the same tree per element)
    if (grid > d->flag_max && grid <= 4 * d->flag_max) {
        const unsigned g = ftar::cap_tree_batch(&B, d->flag_max);
        if (g) grid = g;
    }
    if (!can_gate(d, grid)) return 0;
    // only a launch that never writes what it reads is gated: a gate the device gave up on
    // is relaunched whole, and some workgroups may have run already
    const size_t es = esize_of(dtype);
    for (int t = 0; t < B.nt; t++)
        for (int k = 0; k < B.nt; k++)
            for (int j = 0; j < nsrc; j++)
                if (overlaps(B.t[t].out, B.t[t].n * es, B.t[k].src[j], B.t[k].n * es)) return 0;
    unsigned stage_tag = 0;
    if (stage_dst && stage_n) {
        stage_tag = ++d->sig_tag; // the launch raises the flag twice: staged, then done
        d->ctr.hbm_bytes += 2.0 * (double)stage_n * (double)es;
    }
    B.sig = arm_gate(d, link, hbm);
    relay_gate(d, B.sig, grid);
    keep_plan(d, 1, dtype, op, nsrc, grid, nullptr, &B);
    if (stage_tag) {
        B.sig.stage_src = stage_src;
        B.sig.stage_dst = stage_dst;
        B.sig.stage_n = stage_n;
        B.sig.stage_es = (unsigned)esize_of(dtype);
        B.sig.stage_tag = stage_tag;
        B.sig.stage_cnt = d->sig_cnt + 16; // its own counter, 64 B from the completion counter
        d->pre_gate_any = 1;               // the drain before the barrier waits for "staged"
        d->pre_gate_tag = stage_tag;
    }
    if (d->trace) {
        std::vector<TrRange> rd, wr, sw;
        batch_ranges(B, nsrc, es, rd, wr);
        const std::string rw = tr_rw(d, rd, wr);
        d->gp[d->gate_seq & 1].tr_rw = rw;
        std::string st;
        if (stage_tag) {
            sw.push_back({stage_dst, stage_n * es});
            tr_fmt(d, sw, st);
        }
        tr_launch(d, d->stream, &B.sig, rw, d->gate_seq, "k", st, stage_tag);
    }
    hipError_t e = ftar::launch_tree_batch(dtype, op, nsrc, B, grid, d->stream);
    if (e != hipSuccess) return set_err(e, "tree_batch_kernel launch (gated)");
    d->gate_pending = 1;
    *gated = 1;
    return 0;
}

int fdev_tree_batch_gated(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc,
                          const unsigned *remote_mask, void *const *out, const size_t *n, int ntree, int tag,
                          int *gated)
{
    return fdev_tree_batch_staged_gated(d, dtype, op, src, nsrc, remote_mask, out, n, ntree, tag, nullptr, nullptr, 0,
                                        gated);
}

int fdev_gate_open(ftar_dev *d, int skip)
{
    if (!d->gate_pending) return 0;
    tr(d, "G %u %s", d->gate_seq, skip ? "skip" : "go");
    __atomic_store_n(gate_word(d, d->gate_seq), 2u * d->gate_seq + (skip ? 1u : 0u), __ATOMIC_RELEASE);
    if (!skip) {
        d->ctr.link_bytes += d->gate_link;
        d->ctr.hbm_bytes += d->gate_hbm;
    }
    d->gate_pending = 0;
    d->big_pending = 0;
    // a launch opened as go is checked at the drain that completes it (verify_gate); one given
    // up needs no check: its step launches normally, and the kept plan must never run after it
    ftar_dev::GatedPlan &g = d->gp[d->gate_seq & 1];
    if (g.valid && g.seq == d->gate_seq) {
        if (skip) g.valid = 0;
        else g.opened = 1;
    }
    return 0;
}

int fdev_gate_pending(const ftar_dev *d) { return d->gate_pending; }

int fdev_gate_relaunches(const ftar_dev *d) { return d->gate_relaunches; }

int fdev_set_knob(ftar_dev *d, int knob, int value)
{
    switch (knob) {
    case FDEV_KNOB_FLAG_SYNC:
        if (value && !d->sig_flag) return 13; // the pinned words were never set up (FTAR_FLAG_SYNC=0 at open)
        if (d->gate_pending) (void)fdev_gate_open(d, 1);
        d->flag_sync = value != 0;
        return 0;
    case FDEV_KNOB_TREE_UNROLL:
        if (value != 1 && value != 2 && value != 4) return 13;
        d->tree_unroll = (unsigned)value;
        return 0;
    default: return 13;
    }
}

int fdev_get_knob(const ftar_dev *d, int knob)
{
    switch (knob) {
    case FDEV_KNOB_FLAG_SYNC: return d->flag_sync;
    case FDEV_KNOB_TREE_UNROLL: return (int)d->tree_unroll;
    default: return -1;
    }
}

int fdev_tree_batch(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, const unsigned *remote_mask,
                    void *const *out, const size_t *n, int ntree, int tag)
{
    ftar::TreeBatch B;
    unsigned grid = 0;
    double link, hbm;
    int rc = build_batch(d, dtype, op, src, nsrc, remote_mask, out, n, ntree, tag, &B, &grid, &link, &hbm);
    if (rc || B.nt == 0) return rc;
    if (grid == 0) { // a tree beyond the workgroup budget: one (split) launch per tree
        for (int t = 0; t < ntree; t++) {
            int rc = fdev_tree(d, dtype, op, src + (size_t)t * nsrc, nsrc, remote_mask[t], out[t], n[t], tag);
            if (rc) return rc;
        }
        return 0;
    }
    d->ctr.link_bytes += link;
    d->ctr.hbm_bytes += hbm;
    note_launch(d, d->stream, grid, true, &B.sig);
    if (d->trace) {
        std::vector<TrRange> rd, wr;
        batch_ranges(B, nsrc, esize_of(dtype), rd, wr);
        tr_launch(d, d->stream, &B.sig, tr_rw(d, rd, wr), 0, "k");
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (d->profiling) {
        e0 = get_event(d);
        e1 = get_event(d);
        if (e0) (void)hipEventRecord(e0, d->stream);
    }
    hipError_t e = ftar::launch_tree_batch(dtype, op, nsrc, B, grid, d->stream);
    if (e != hipSuccess) return set_err(e, "tree_batch_kernel launch");
    if (d->profiling && e0 && e1) {
        (void)hipEventRecord(e1, d->stream);
        d->pending.push_back(Pending{e0, e1, tag});
    }
    return 0;
}

int fdev_run(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    return run_on(d, d->stream, dtype, op, segs, nseg, tag);
}

// A mid-size launch (more workgroups than signal their completion cheaply) queued behind a
// gate: a fenced marker is recorded first -- the drain before the barrier waits for it, i.e.
// for everything queued before the gated launch, and its system-scope release makes that
// work visible to the peers as the usual drain does -- then the launch, its grid capped at
// big_blocks workgroups (each loops over its share of tiles: a waiting launch occupies a
// part of the device, so ranks sharing a GPU still run), its gate relayed through device
// words.  It does not signal: after the gate opens it is drained by a fenced marker.
static int run_gated_relayed(ftar_dev *d, int dtype, int op, const ftar::SegIn *in, int nseg, size_t es, double link,
                             double hbm, int *gated)
{
    if (!d->flag_sync || !d->gate_dw || d->profiling || d->gate_pending) return 0;
    ftar::KSegList L;
    unsigned grid = ftar::plan_segments(in, nseg, es, d->big_blocks, &L);
    if (grid == 0) return 0;
    L.nt_store = nt_store();
    HIPCHK(hipEventRecord(d->fence_pre, d->stream)); // the work before the gate, released and drainable
    tr(d, "M pre");
    d->need_acquire = 0;
    L.sig = arm_gate(d, link, hbm);
    d->signalled--; // arm_gate counted a signalled launch: this one drains through a marker
    L.sig.cnt = nullptr;
    L.sig.flag = nullptr;
    L.sig.gate_poll = d->gate_dw + d->gate_seq % ftar::kGateSlots;
    L.sig.gate_dev = d->gate_dw + 32 + d->gate_seq % ftar::kGateSlots;
    keep_plan(d, 0, dtype, op, 0, grid, &L, nullptr);
    if (d->trace) {
        std::vector<TrRange> rd, wr;
        for (int i = 0; i < nseg; i++) {
            rd.push_back({in[i].x, in[i].n * es});
            if (in[i].kind != ftar::kCopy) rd.push_back({in[i].y, in[i].n * es});
            wr.push_back({in[i].out, in[i].n * es});
            wr.push_back({in[i].out2, in[i].n * es});
        }
        const std::string rw = tr_rw(d, rd, wr);
        d->gp[d->gate_seq & 1].tr_rw = rw;
        d->tr_fenced = 0;
        tr_launch(d, d->stream, &L.sig, rw, d->gate_seq, "k");
    }
    hipError_t e = ftar::launch_segments(dtype, op, L, grid, d->stream);
    if (e != hipSuccess) return set_err(e, "segment_kernel launch (gated, relayed)");
    d->gate_pending = 1;
    d->big_pending = 1;
    *gated = 1;
    return 0;
}

int fdev_run_gated(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag, void *stage_dst,
                   const void *stage_src, size_t stage_n, int *gated)
{
    *gated = 0;
    size_t es = esize_of(dtype);
    if (es == 0 || op < 0 || op >= ftar::kNumOps || nseg < 0 || nseg > FDEV_MAX_SEGS || tag < 0 || tag >= FDEV_NTAGS) {
        snprintf(g_err, sizeof(g_err), "fdev_run_gated: bad arguments");
        return 13;
    }
    ftar::SegIn in[FDEV_MAX_SEGS];
    double link = 0, hbm = 0;
    seg_inputs(segs, nseg, es, in, &link, &hbm);
    // only a launch that never writes what it reads is gated (see fdev_tree_batch_staged_gated)
    for (int i = 0; i < nseg; i++)
        for (int k = 0; k < nseg; k++) {
            const size_t ni = segs[i].n * es, nk = segs[k].n * es;
            for (void *o : {segs[i].out, segs[i].out2})
                if (overlaps(o, ni, segs[k].x, nk) || (segs[k].kind != FDEV_COPY && overlaps(o, ni, segs[k].y, nk)))
                    return 0;
        }
    ftar::KSegList L;
    unsigned grid = ftar::plan_segments(in, nseg, es, d->max_blocks, &L);
    if (grid > d->flag_max && !stage_dst)
        return run_gated_relayed(d, dtype, op, in, nseg, es, link, hbm, gated);
    if (!can_gate(d, grid)) return 0;
    L.nt_store = nt_store();
    unsigned stage_tag = 0;
    if (stage_dst && stage_n) {
        stage_tag = ++d->sig_tag; // the launch raises the flag twice: staged, then done
        d->ctr.hbm_bytes += 2.0 * (double)stage_n * (double)es;
    }
    L.sig = arm_gate(d, link, hbm);
    relay_gate(d, L.sig, grid);
    keep_plan(d, 0, dtype, op, 0, grid, &L, nullptr);
    if (stage_tag) {
        L.sig.stage_src = stage_src;
        L.sig.stage_dst = stage_dst;
        L.sig.stage_n = stage_n;
        L.sig.stage_es = (unsigned)es;
        L.sig.stage_tag = stage_tag;
        L.sig.stage_cnt = d->sig_cnt + 16;
        d->pre_gate_any = 1;
        d->pre_gate_tag = stage_tag;
    }
    if (d->trace) {
        std::vector<TrRange> rd, wr, sw;
        seg_ranges(segs, nseg, es, rd, wr);
        const std::string rw = tr_rw(d, rd, wr);
        d->gp[d->gate_seq & 1].tr_rw = rw;
        std::string st;
        if (stage_tag) {
            sw.push_back({stage_dst, stage_n * es});
            tr_fmt(d, sw, st);
        }
        d->tr_fenced = 0;
        tr_launch(d, d->stream, &L.sig, rw, d->gate_seq, "k", st, stage_tag);
    }
    hipError_t e = ftar::launch_segments(dtype, op, L, grid, d->stream);
    if (e != hipSuccess) return set_err(e, "segment_kernel launch (gated)");
    d->gate_pending = 1;
    *gated = 1;
    return 0;
}

int fdev_run_bg(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    int rc = ensure_bg(d);
    if (rc) return rc;
    hipEvent_t e = get_event(d);
    if (!e) return set_err(hipErrorOutOfMemory, "hipEventCreate");
    HIPCHK(hipEventRecord(e, d->stream));
    HIPCHK(hipStreamWaitEvent(d->bg, e, 0));
    d->event_pool.push_back(e);
    return run_on(d, d->bg, dtype, op, segs, nseg, tag);
}

int fdev_copy(ftar_dev *d, int bg, void *dst, const void *src, size_t bytes, int remote, int tag)
{
    if (tag < 0 || tag >= FDEV_NTAGS) return 13;
    if (bytes == 0) return 0;
    hipStream_t st = d->stream;
    if (bg) { // ordered after the main stream, like fdev_run_bg
        int rc = ensure_bg(d);
        if (rc) return rc;
        hipEvent_t e = get_event(d);
        if (!e) return set_err(hipErrorOutOfMemory, "hipEventCreate");
        HIPCHK(hipEventRecord(e, d->stream));
        HIPCHK(hipStreamWaitEvent(d->bg, e, 0));
        d->event_pool.push_back(e);
        st = d->bg;
    }
    if (remote) {
        d->ctr.link_bytes += (double)bytes;
        d->ctr.hbm_bytes += (double)bytes; // the local write
    } else {
        d->ctr.hbm_bytes += 2.0 * (double)bytes;
    }
    note_launch(d, st, ~0u, false, nullptr);
    if (d->trace) tr_launch(d, st, nullptr, tr_rw(d, {{src, bytes}}, {{dst, bytes}}), 0, "sdma");
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (d->profiling) {
        e0 = get_event(d);
        e1 = get_event(d);
        if (e0) (void)hipEventRecord(e0, st);
    }
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
    if (d->profiling && e0 && e1) {
        (void)hipEventRecord(e1, st);
        d->pending.push_back(Pending{e0, e1, tag});
    }
    return 0;
}

int fdev_order_after(ftar_dev *d, void *user_stream)
{
    if (d->gate_pending) (void)fdev_gate_open(d, 1); // nothing waits behind a closed gate
    // An idle caller stream has nothing our kernels must wait for (its kernels completed,
    // their stores released to this device).  A busy one is waited for on the host, never
    // by queuing a GPU-side dependency: an event recorded on the caller's stream is a
    // marker there, which the NEXT call's hipStreamQuery then finds pending (the runtime
    // reports completion of the caller's stream with a lag), so the wait was queued again
    // on every call -- and a cross-queue wait behind a marker on an otherwise idle queue
    // cost 30-50 us per call on one MI355X (tools/_exp_nullq.hip, profiles/r03/nullq/).
    // The call blocks until its own kernels are done anyway; waiting for the caller's
    // pending work first costs nothing extra.
    hipStream_t s = (hipStream_t)user_stream;
    hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) (void)hipGetLastError();
    d->user_host_waits++;
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

int fdev_user_host_waits(const ftar_dev *d) { return d->user_host_waits; }

static int harvest(ftar_dev *d);

// Waits for everything enqueued on `st` by spinning on a fenced marker event.  Its
// system-scope sequentially consistent fence is what makes a step's results visible to
// the peers that pull them next -- the writeback puts this GPU's dirty L2 lines in HBM
// (peers read our HBM over xGMI, not our L2) -- and its invalidation drops this GPU's
// cached copies of peer memory, so the next step's pulls (issued after the barrier,
// with no peer reads in between) fetch the peers' new windows.  Without it the
// visibility of a kernel's stores to other GPUs would rest on the runtime's default
// packet fences.
static int sync_stream(ftar_dev *d, hipStream_t st, int (*poll)(void *), void *arg)
{
    hipEvent_t fence = st == d->bg ? d->fence_bg : d->fence_main;
    if (d->tr_drop == 1) { // TEST-ONLY (FTAR_TRACE_DROP=release): the drain without its system fence
        hipEvent_t &nf = st == d->bg ? d->nofence_bg : d->nofence_main;
        if (!nf) HIPCHK(hipEventCreateWithFlags(&nf, hipEventDisableTiming | hipEventDisableSystemFence));
        fence = nf;
    }
    HIPCHK(hipEventRecord(fence, st));
    for (;;) {
        hipError_t e = hipEventQuery(fence);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) return set_err(e, "hipEventQuery");
        if (poll) {
            int r = poll(arg);
            if (r) return r;
        }
    }
    tr(d, "D %s %c", d->tr_drop == 1 ? "nf" : "mk", st == d->bg ? 'b' : 'm');
    return 0;
}

// Waits for the signal of launch `tag` (its last workgroup's store into the pinned flag
// word), polling the failure detector; a device error surfaces through hipStreamQuery.
static int wait_signal(ftar_dev *d, unsigned tag, int (*poll)(void *), void *arg)
{
    for (unsigned spins = 1;; spins++) {
        if ((int)(__atomic_load_n(d->sig_flag, __ATOMIC_ACQUIRE) - tag) >= 0) return 0;
        if (poll) {
            int r = poll(arg);
            if (r) return r;
        }
        if ((spins & 255) == 0) {
            hipError_t e = hipStreamQuery(d->stream);
            if (e == hipSuccess) { // the stream drained: the flag is there, or fall back
                if ((int)(__atomic_load_n(d->sig_flag, __ATOMIC_ACQUIRE) - tag) >= 0) return 0;
                return sync_stream(d, d->stream, poll, arg);
            }
            if (e != hipErrorNotReady) return set_err(e, "hipStreamQuery");
        }
    }
}

// The gates opened as go have completed (every drain covers the launches queued before any
// still-pending gate): did the device give one up (its gate stayed closed past the timeout,
// or a late workgroup found the slot overtaken)?  Then its workgroups (some or all) returned
// without touching memory, and the plan runs again ungated -- after a fenced marker
// (device-wide acquire: the peers' current data) and drained through one (release: visible
// to the peers before this rank arrives anywhere).  Any launch pending behind its own gate is
// given up first (nothing waits behind a closed gate); its step then launches normally.
static int verify_gate(ftar_dev *d, int (*poll)(void *), void *arg)
{
    int redo = 0;
    for (unsigned k = 0; k < 2; k++) {
        // the older of the two first, and a later one again after a relaunch (it may have
        // read what the given-up one should have written): the steps' order is kept
        ftar_dev::GatedPlan &g = d->gp[(d->gate_seq + 1 + k) & 1];
        if (!g.valid || !g.opened) continue;
        g.valid = 0;
        unsigned *err = gate_err(d, g.seq);
        if (__atomic_load_n(err, __ATOMIC_ACQUIRE) != 2u * g.seq && !redo) continue;
        __atomic_store_n(err, 0u, __ATOMIC_RELAXED);
        if (d->gate_pending) (void)fdev_gate_open(d, 1);
        fprintf(stderr, "ftar: device %d: gated launch %u %s: relaunched\n", d->device, g.seq,
                redo++ ? "ran after a relaunched one" : "was given up by the device (gate timeout)");
        HIPCHK(hipEventRecord(d->fence_main, d->stream));
        d->tr_fenced = 1;
        tr_launch(d, d->stream, nullptr, g.tr_rw, 0, "k");
        hipError_t e = g.batch ? ftar::launch_tree_batch(g.dtype, g.op, g.nsrc, g.B, g.grid, d->stream)
                               : ftar::launch_segments(g.dtype, g.op, g.L, g.grid, d->stream);
        if (e != hipSuccess) return set_err(e, "relaunch of a timed-out gated launch");
        d->gate_relaunches++;
        int rc = sync_stream(d, d->stream, poll, arg);
        d->need_acquire = 0;
        d->unsignalled = d->signalled = d->force_fence = 0;
        if (rc) return rc;
    }
    return 0;
}

static int spin(hipEvent_t e, int (*poll)(void *), void *arg);

int fdev_sync(ftar_dev *d, int (*poll)(void *), void *arg)
{
    int rc;
    if (d->gate_pending && d->big_pending) {
        // a mid-size launch waits on its closed gate: the fenced marker recorded just before
        // it covers (and released) everything queued earlier
        rc = spin(d->fence_pre, poll, arg);
        d->need_acquire = 0;
        d->pre_gate_any = 0;
        d->signalled = d->force_fence = 0;
        d->unsignalled = 1; // the gated launch, drained through a marker after its gate opens
        if (rc) return rc;
        tr(d, "D pre");
        rc = verify_gate(d, poll, arg);
        if (rc) return rc;
        return harvest(d);
    }
    if (d->gate_pending) {
        // a launch waits on its closed gate: drain what was queued before it (all of it
        // signalled, the gated launch checked; nothing is queued behind it, see note_launch),
        // never a marker behind the gate
        rc = d->pre_gate_any ? wait_signal(d, d->pre_gate_tag, poll, arg) : 0;
        if (!rc && d->pre_gate_any) tr(d, "D sig %u", d->pre_gate_tag);
        d->need_acquire = 1;
        d->pre_gate_any = 0;
        d->unsignalled = d->force_fence = 0;
        d->signalled = 1; // the gated launch, drained after its gate opens
        if (rc) return rc;
        // an earlier gated launch among them (RD: step s, opened; step s + 1 pending) has
        // completed too: check it now, before step s + 1 can read its result
        rc = verify_gate(d, poll, arg);
        if (rc) return rc;
        return harvest(d);
    }
    if (!d->unsignalled && !d->signalled && !d->force_fence) {
        rc = 0; // nothing queued since the last drain
    } else if (!d->unsignalled && d->signalled && !d->force_fence) {
        // only signalled launches: each workgroup released its stores at system scope before
        // the last one raised the flag, so the data is visible to the peers and the host
        rc = wait_signal(d, d->sig_tag, poll, arg);
        if (!rc) tr(d, "D sig %u", d->sig_tag);
        d->need_acquire = 1;
    } else {
        rc = sync_stream(d, d->stream, poll, arg);
        d->need_acquire = 0;
    }
    d->unsignalled = d->signalled = d->force_fence = 0;
    if (rc) return rc;
    rc = verify_gate(d, poll, arg); // the gated launch has completed: did its gate time out?
    if (rc) return rc;
    return harvest(d);
}

void fdev_fence_next_drain(ftar_dev *d) { d->force_fence = 1; }

int fdev_peer_wait(ftar_dev *d, void *flag, void *const *peer_flags, int npeers, uint64_t token,
                   int (*poll)(void *), void *arg)
{
    (void)poll;
    (void)arg;
    if (!d->sig_flag || !d->gate_dw || !flag || npeers < 1 || npeers > ftar::kMaxPeers) {
        snprintf(g_err, sizeof(g_err), "fdev_peer_wait: unavailable (%s) or bad arguments",
                 d->sig_flag ? "flag words" : "FTAR_FLAG_SYNC=0");
        return 13;
    }
    if (d->gate_pending) (void)fdev_gate_open(d, 1); // nothing waits behind a closed gate
    ftar::PeerWait W{};
    W.own = (unsigned long long *)flag;
    for (int i = 0; i < npeers; i++) W.peer[i] = (const unsigned long long *)peer_flags[i];
    W.npeers = npeers;
    W.token = (unsigned long long)token;
    d->pw_seq++;
    d->pw_vval = 2u * d->pw_seq;
    __atomic_store_n(d->sig_flag + 48, 0u, __ATOMIC_RELAXED); // verdict
    __atomic_store_n(d->sig_flag + 49, 0u, __ATOMIC_RELEASE); // abort word
    W.abort_word = d->sig_flag + 49;
    W.verdict_dev = d->gate_dw + 48;
    W.verdict_host = d->sig_flag + 48;
    W.vval = d->pw_vval;
    W.ticks = d->gate_ticks;
    // release: everything this rank queued so far is in HBM, device-wide, before its flag
    if (d->tr_drop == 1) { // TEST-ONLY (FTAR_TRACE_DROP=release): the flag without the release
        if (!d->nofence_main)
            HIPCHK(hipEventCreateWithFlags(&d->nofence_main, hipEventDisableTiming | hipEventDisableSystemFence));
        HIPCHK(hipEventRecord(d->nofence_main, d->stream));
    } else {
        HIPCHK(hipEventRecord(d->fence_main, d->stream));
    }
    if (d->trace) {
        std::string own, peers;
        tr_fmt(d, {{flag, 8}}, own);
        std::vector<TrRange> pr;
        for (int i = 0; i < npeers; i++) pr.push_back({peer_flags[i], 8});
        tr_fmt(d, pr, peers);
        if (d->tr_drop != 1) tr(d, "M pub"); // the fenced marker in front of the flag (a release, not a drain)
        tr(d, "F %llu w=%s", (unsigned long long)token, own.c_str());
        tr(d, "V %llu r=%s", (unsigned long long)token, peers.c_str());
    }
    hipError_t e = ftar::launch_peer_wait(W, d->stream);
    if (e != hipSuccess) return set_err(e, "peer_wait_kernel launch");
    d->unsignalled++; // drained through a fenced marker
    d->need_acquire = d->tr_drop == 1; // the marker invalidated the caches (unless it was dropped)
    d->pw_pending = 1;
    d->pw_armed = 0;
    return 0;
}

void fdev_peer_wait_abort(ftar_dev *d)
{
    if (d->sig_flag && d->pw_vval) __atomic_store_n(d->sig_flag + 49, d->pw_vval, __ATOMIC_RELEASE);
}

int fdev_peer_wait_verdict(ftar_dev *d)
{
    d->pw_pending = 0;
    if (!d->pw_armed) return 1;
    d->pw_armed = 0;
    if (__atomic_load_n(d->sig_flag + 48, __ATOMIC_ACQUIRE) == d->pw_vval) return 1;
    tr(d, "S %llu", d->pw_launch_n); // the launch behind the wait returned untouched
    return 0;
}

int fdev_busy(ftar_dev *d)
{
    hipError_t e = hipStreamQuery(d->stream);
    if (e == hipErrorNotReady) return 1;
    if (e != hipSuccess) (void)hipGetLastError();
    return 0;
}

int fdev_sync_bg(ftar_dev *d, int (*poll)(void *), void *arg)
{
    if (d->gate_pending) (void)fdev_gate_open(d, 1); // the background stream follows the main one
    if (!d->bg) return harvest(d); // never used: nothing queued
    int rc = sync_stream(d, d->bg, poll, arg);
    if (rc) return rc;
    return harvest(d);
}

/* collect the timings of every event pair whose stop event has completed */
static int harvest(ftar_dev *d)
{
    std::vector<Pending> still;
    for (auto &p : d->pending) {
        if (hipEventQuery(p.stop) != hipSuccess) {
            still.push_back(p);
            continue;
        }
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess) {
            d->ctr.ms[p.tag] += ms;
            d->ctr.launches[p.tag]++;
        }
        d->event_pool.push_back(p.start);
        d->event_pool.push_back(p.stop);
    }
    d->pending.swap(still);
    return 0;
}

// The D2H copies ride on the background stream (idle in every call the pipeline runs
// in: it only carries a spare's redundancy copy, joined before each call returns), so a
// rank needs at most four streams -- null, main, background, H2D -- one hardware queue
// each (GPU_MAX_HW_QUEUES = 4); a fifth would share a queue and serialize the copies.
static int ensure_pipe(ftar_dev *d)
{
    if (d->h2d) return 0;
    int rc = ensure_bg(d);
    if (rc) return rc;
    HIPCHK(hipStreamCreateWithFlags(&d->h2d, hipStreamNonBlocking));
    d->d2h = d->bg;
    // default (fenced) events: a landed chunk is visible to the peers that pull it
    for (int i = 0; i < FDEV_MAX_CHUNKS; i++) HIPCHK(hipEventCreateWithFlags(&d->h2d_done[i], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&d->fence_d2h, hipEventDisableTiming));
    return 0;
}

static int spin(hipEvent_t e, int (*poll)(void *), void *arg)
{
    for (;;) {
        hipError_t r = hipEventQuery(e);
        if (r == hipSuccess) return 0;
        if (r != hipErrorNotReady) return set_err(r, "hipEventQuery");
        if (poll) {
            int rc = poll(arg);
            if (rc) return rc;
        }
    }
}

int fdev_h2d_async(ftar_dev *d, void *dst, const void *src, size_t bytes, int slot)
{
    if (slot < 0 || slot >= FDEV_MAX_CHUNKS) return 13;
    int rc = ensure_pipe(d);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, d->h2d));
    HIPCHK(hipEventRecord(d->h2d_done[slot], d->h2d));
    return 0;
}

int fdev_wait_h2d(ftar_dev *d, int slot, int (*poll)(void *), void *arg)
{
    if (slot < 0 || slot >= FDEV_MAX_CHUNKS || !d->h2d) return 13;
    return spin(d->h2d_done[slot], poll, arg);
}

int fdev_d2h_async(ftar_dev *d, void *dst, const void *src, size_t bytes)
{
    if (d->gate_pending) (void)fdev_gate_open(d, 1);
    int rc = ensure_pipe(d);
    if (rc) return rc;
    hipEvent_t e = get_event(d);
    if (!e) return set_err(hipErrorOutOfMemory, "hipEventCreate");
    HIPCHK(hipEventRecord(e, d->stream));
    HIPCHK(hipStreamWaitEvent(d->d2h, e, 0));
    d->event_pool.push_back(e);
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, d->d2h));
    return 0;
}

int fdev_sync_d2h(ftar_dev *d, int (*poll)(void *), void *arg)
{
    if (d->gate_pending) (void)fdev_gate_open(d, 1);
    if (!d->d2h) return 0;
    HIPCHK(hipEventRecord(d->fence_d2h, d->d2h));
    return spin(d->fence_d2h, poll, arg);
}

int fdev_h2d(ftar_dev *d, void *dst, const void *src, size_t bytes)
{
    note_launch(d, d->stream, ~0u, false, nullptr);
    if (d->trace) tr_launch(d, d->stream, nullptr, tr_rw(d, {}, {{dst, bytes}}), 0, "h2d");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, d->stream));
    return fdev_sync(d, nullptr, nullptr);
}

int fdev_d2h(ftar_dev *d, void *dst, const void *src, size_t bytes)
{
    note_launch(d, d->stream, ~0u, false, nullptr);
    if (d->trace) tr_launch(d, d->stream, nullptr, tr_rw(d, {{src, bytes}}, {}), 0, "d2h");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, d->stream));
    return fdev_sync(d, nullptr, nullptr);
}

void fdev_profiling(ftar_dev *d, int on) { d->profiling = on; }

void fdev_counters_reset(ftar_dev *d) { memset(&d->ctr, 0, sizeof(d->ctr)); }

void fdev_counters_get(ftar_dev *d, fdev_counters *out) { *out = d->ctr; }

int fdev_set_reduce_variant(int v)
{
    if (v < 0 || v > 1) return 13;
    g_reduce_variant = v;
    return 0;
}

// An operand of the local reduce: memory of device `dev` (the whole range inside one
// allocation) or pinned host memory, which the kernel reads and writes in place over PCIe
// (zero copy: the reads use the link's host-to-device direction while the stores use the
// other).  Pageable or unknown memory is refused before any launch: a kernel touching it
// would fault the GPU.
static int check_local_ptr(const void *ptr, size_t bytes, int dev)
{
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    if (hipPointerGetAttributes(&a, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return 1;
    }
    if (a.type == hipMemoryTypeHost) return !host_same_va(a) || !range_inside(ptr, bytes);
    if (a.type != hipMemoryTypeDevice || a.device != dev) return 1;
    return !range_inside(ptr, bytes);
}

int fdev_trace_open(ftar_dev *d, const char *path)
{
    if (d->trace) return 0;
    d->trace = fopen(path, "w");
    if (!d->trace) {
        snprintf(g_err, sizeof(g_err), "FTAR_TRACE: cannot open %s", path);
        return 13;
    }
    setvbuf(d->trace, nullptr, _IOLBF, 0); // a killed rank leaves every line it wrote
#ifdef FTAR_TEST_HOOKS
    // TEST-ONLY (lib/libftar_hooks.so): drop a release or an acquire, so that
    // tests/test_gpu_fences.py can show the fence checker fails without it
    const char *dr = getenv("FTAR_TRACE_DROP");
    d->tr_drop = !dr ? 0 : !strcmp(dr, "release") ? 1 : !strcmp(dr, "acquire") ? 2 : 0;
#endif
    tr(d, "# ftar trace: device %d, flag_sync %d, drop %d", d->device, d->flag_sync, d->tr_drop);
    return 0;
}

void fdev_trace_region(ftar_dev *d, const void *base, size_t bytes, int owner, const char *name)
{
    if (!d->trace || !base) return;
    for (ftar_dev::Region &g : d->regions)
        if (g.base == (uintptr_t)base) {
            g.bytes = bytes;
            g.owner = owner;
            g.name = name;
            tr(d, "R %d %s %zu", owner, name, bytes);
            return;
        }
    d->regions.push_back(ftar_dev::Region{(uintptr_t)base, bytes, owner, name});
    tr(d, "R %d %s %zu", owner, name, bytes);
}

void fdev_trace_unregion(ftar_dev *d, const void *base)
{
    if (!d->trace || !base) return;
    for (size_t i = 0; i < d->regions.size(); i++)
        if (d->regions[i].base == (uintptr_t)base) {
            tr(d, "U %d %s", d->regions[i].owner, d->regions[i].name.c_str());
            d->regions.erase(d->regions.begin() + (long)i);
            return;
        }
}

// A write this rank's own launches did not make (the caller's send buffer, exported to the
// peers as it is): `X owner:name:offset:bytes`
void fdev_trace_external_write(ftar_dev *d, const void *p, size_t bytes)
{
    if (!d->trace) return;
    std::string w;
    tr_fmt(d, {{p, bytes}}, w);
    tr(d, "X %s", w.c_str());
}

void fdev_trace_note(ftar_dev *d, const char *fmt, ...)
{
    if (!d->trace) return;
    va_list ap;
    va_start(ap, fmt);
    vfprintf(d->trace, fmt, ap);
    va_end(ap);
    fputc('\n', d->trace);
}

int fdev_reduce_local(const void *in, void *inout, size_t n, int dtype, int op, void *stream)
{
    size_t es = esize_of(dtype);
    if (es == 0 || op < 0 || op >= ftar::kNumOps) {
        snprintf(g_err, sizeof(g_err), "reduce_local: bad dtype/op");
        return 13;
    }
    if (n == 0) return 0;
    if (process_knobs()) return 13; // FTAR_NT_STORE / FTAR_BLOCKS_PER_CU refused (g_err names it)
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    if (n > SIZE_MAX / es || check_local_ptr(in, n * es, dev) || check_local_ptr(inout, n * es, dev)) {
        snprintf(g_err, sizeof(g_err), "reduce_local: operands must be memory of device %d or pinned host memory", dev);
        return 13;
    }
    hipDeviceProp_t prop;
    static int cached_dev = -1;
    static unsigned cached_blocks = 2048;
    if (cached_dev != dev) {
        HIPCHK(hipGetDeviceProperties(&prop, dev));
        cached_blocks = (unsigned)prop.multiProcessorCount * blocks_per_cu();
        cached_dev = dev;
    }
    hipStream_t s = (hipStream_t)stream;
    bool aligned = (((uintptr_t)in | (uintptr_t)inout) & 15) == 0 && (n * es) % 16 == 0;
    if (g_reduce_variant == 1 && aligned) {
        size_t nv = n * es / 16;
        size_t tiles = (nv + ftar::kTileVecs - 1) / ftar::kTileVecs;
        unsigned grid = tiles < cached_blocks ? (unsigned)tiles : cached_blocks;
        hipError_t e = ftar::launch_reduce_lds(dtype, op, inout, in, nv, grid, s, nt_store());
        if (e != hipSuccess) return set_err(e, "reduce_lds_kernel launch");
        return 0;
    }
    // MPI_Reduce_local(in, inout): inout = inout <op> in  -> x = inout, y = in
    ftar::SegIn seg{ftar::kReduce, inout, inout, in, n, nullptr};
    ftar::KSegList L;
    unsigned grid = ftar::plan_segments(&seg, 1, es, cached_blocks, &L);
    if (grid == 0) return 0;
    L.nt_store = nt_store();
    hipError_t e = ftar::launch_segments(dtype, op, L, grid, s);
    if (e != hipSuccess) return set_err(e, "segment_kernel launch");
    return 0;
}

} // extern "C"
