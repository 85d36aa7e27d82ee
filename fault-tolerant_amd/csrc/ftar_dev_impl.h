// ftar_dev_impl.h -- what the four parts of libftar's HIP runtime glue share (internal; the
// schedules see ftar_dev.h only): the per-rank device state `struct ftar_dev`, the process
// knobs and the error text, and the helpers one part calls in another.
//   ftar_dev_hip.cpp     device open / close, knobs, exportable HBM and IPC mappings, local reduce
//   ftar_dev_launch.cpp  kernel launches and copies, completion signals, drains, the peer wait
//   ftar_dev_gate.cpp    launches queued behind a gate, their verdicts and relaunches
//   ftar_dev_trace.cpp   FTAR_TRACE (tests/fence_check.py)
#ifndef FTAR_DEV_IMPL_H
#define FTAR_DEV_IMPL_H

#include <hip/hip_runtime.h>

#include <stdio.h>

#include <string>
#include <vector>

#include "ftar_dev.h"
#include "ftar_kernels.h"

namespace fdevi {

extern char g_err[512];        // fdev_last_error()
extern int g_reduce_variant;   // fdev_set_reduce_variant
extern long long g_nt, g_bpc;  // FTAR_NT_STORE, FTAR_BLOCKS_PER_CU (process_knobs)

// the process-wide knobs, read and checked once: 0, or 13 (FTAR_ERR_ARG) with g_err naming
// the refused value
int process_knobs();
bool env_knob(const char *name, long long lo, long long hi, long long dflt, long long *out);
unsigned nt_store();
unsigned blocks_per_cu();
int set_err(hipError_t e, const char *what); // g_err = what + the runtime's text; 101 (FTAR_ERR_DEVICE)
size_t esize_of(int dtype);
bool host_same_va(const hipPointerAttribute_t &a);
bool range_inside(const void *ptr, size_t bytes);

#define HIPCHK(call)                                                                                        \
    do {                                                                                                    \
        hipError_t _e = (call);                                                                             \
        if (_e != hipSuccess) return fdevi::set_err(_e, #call);                                             \
    } while (0)

struct Pending { // a timed launch: its event pair, harvested into ftar_dev::ctr
    hipEvent_t start, stop;
    int tag;
};

} // namespace fdevi

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
    std::vector<fdevi::Pending> pending;
    std::vector<hipEvent_t> event_pool;
    fdev_counters ctr;
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

namespace fdevi {

// ---- ftar_dev_launch.cpp
int ensure_bg(ftar_dev *d);
hipEvent_t get_event(ftar_dev *d);
void note_launch(ftar_dev *d, hipStream_t st, unsigned grid, bool can_signal, ftar::KSignal *sig);
void seg_inputs(const fdev_seg *segs, int nseg, size_t es, ftar::SegIn *in, double *link, double *hbm);
bool overlaps(const void *a, size_t na, const void *b, size_t nb);
int build_batch(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, const unsigned *remote_mask,
                void *const *out, const size_t *n, int ntree, int tag, ftar::TreeBatch *B, unsigned *grid,
                double *link, double *hbm);
int sync_stream(ftar_dev *d, hipStream_t st, int (*poll)(void *), void *arg);
int harvest(ftar_dev *d);
int spin(hipEvent_t e, int (*poll)(void *), void *arg);

// ---- ftar_dev_gate.cpp
int verify_gate(ftar_dev *d, int (*poll)(void *), void *arg);

// ---- ftar_dev_trace.cpp
struct TrRange {
    const void *p;
    size_t n;
};
void tr(ftar_dev *d, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void tr_fmt(const ftar_dev *d, const std::vector<TrRange> &v, std::string &out);
std::string tr_rw(const ftar_dev *d, const std::vector<TrRange> &rd, const std::vector<TrRange> &wr);
void tr_launch(ftar_dev *d, hipStream_t st, const ftar::KSignal *sig, const std::string &rw, unsigned gate,
               const char *eng, const std::string &staged = std::string(), unsigned stag = 0);
void seg_ranges(const fdev_seg *segs, int nseg, size_t es, std::vector<TrRange> &rd, std::vector<TrRange> &wr);
void batch_ranges(const ftar::TreeBatch &B, int nsrc, size_t es, std::vector<TrRange> &rd, std::vector<TrRange> &wr);

} // namespace fdevi

#endif
